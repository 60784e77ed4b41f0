"""ORACLE — test infrastructure only.

CPU restatement of the reference's hot path, used ONLY as the checker by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg.  The product (basecount_amd/) never
imports this module.

* ``bcount``     -> liboracle.so ``oracle_bcount``  (restates count.cpp:7-99, see bcount_oracle.c)
* ``stats``      -> liboracle.so ``oracle_stats``   (restates main.py:10-79, see stats_oracle.c)
* ``get_stats_py`` pure-Python restatement of main.py:14-79 (rows), small cases only
* ``summary`` / ``amplicons``  numpy restatement of main.py:469-551 (np.mean / np.median / round)
* ``ref_bcount`` the reference's OWN compiled count.cpp (oracle/_ref, built by oracle/Makefile)

Pinning: tests/test_oracle.py checks the C restatements against the golden fixtures that
tests/golden/make_golden.py produced by running the reference itself (its compiled count.cpp and
its Python main.py over our BAM decoder through oracle/pysam_shim).
"""
from __future__ import annotations

import ctypes as C
import glob
import importlib.util
import math
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        # ORACLE_LIB_DIR: the sanitizer build (oracle/_asan, scripts/asan.sh)
        path = os.path.join(os.environ.get("ORACLE_LIB_DIR") or HERE, "liboracle.so")
        if not os.path.exists(path):
            raise ImportError("oracle/liboracle.so missing: run `make -C oracle`")
        L = C.CDLL(path)
        L.oracle_bcount.argtypes = [C.c_int64, C.c_uint32, C.c_int64] + [C.c_void_p] * 8 + [
            C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
        L.oracle_bcount.restype = C.c_int
        L.oracle_stats.argtypes = [C.c_void_p, C.c_int64, C.c_int, C.c_double, C.c_double,
                                   C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.oracle_stats.restype = None
        L.oracle_bcount_mt.argtypes = L.oracle_bcount.argtypes + [C.c_int]
        L.oracle_bcount_mt.restype = C.c_int
        L.oracle_stats_mt.argtypes = L.oracle_stats.argtypes + [C.c_int]
        L.oracle_stats_mt.restype = None
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data if a is not None and a.size else None


def bcount(ref_len: int, mbq: int, b: dict, nthreads: int = 0):
    """Oracle counts [ref_len][6] uint32 for a batch dict (bc_reads layout), plus
    (bad_read, bad_pos) — (-1, -1) when no counted event fell outside the reference.
    nthreads > 0: the all-cores driver (mt_oracle.c), same results."""
    out = np.zeros((max(ref_len, 0), 6), np.uint32)
    br, bp = C.c_int64(-1), C.c_int64(-1)
    arrs = [np.ascontiguousarray(b[k], dt) for k, dt in
            (("pos", np.int32), ("cig_beg", np.uint32), ("cig_n", np.uint32),
             ("seq_nib", np.uint32), ("cigar", np.uint32), ("seq", np.uint8))]
    q = b.get("qual")
    q = None if q is None else np.ascontiguousarray(q, np.uint8)
    args = [int(ref_len), int(mbq), int(arrs[0].size), *[_p(a) for a in arrs], _p(q),
            _p(out) if out.size else None, C.byref(br), C.byref(bp)]
    if nthreads > 0:
        if lib().oracle_bcount_mt(*args, int(nthreads)) < 0:
            raise MemoryError("oracle_bcount_mt: per-thread histograms")
    else:
        lib().oracle_bcount(*args)
    return out, (br.value, bp.value)


def norm_factors(show_n: bool):
    k = 6 if show_n else 5
    return 1 / math.log2(k), 1 / math.log2(k - 1)


def stats(counts6: np.ndarray, show_n: bool, nthreads: int = 0):
    """(cov[L] i32, pc[k][L], ent[L], sec[L]) exactly as main.py:14-79 computes them."""
    c = np.ascontiguousarray(counts6, np.uint32)
    L = c.shape[0]
    k = 6 if show_n else 5
    nf, nf2 = norm_factors(show_n)
    cov = np.zeros(L, np.int32)
    pc = np.zeros((k, L))
    ent = np.zeros(L)
    sec = np.zeros(L)
    if L and nthreads > 0:
        lib().oracle_stats_mt(_p(c), L, int(show_n), nf, nf2, _p(cov), _p(pc), _p(ent), _p(sec),
                              int(nthreads))
    elif L:
        lib().oracle_stats(_p(c), L, int(show_n), nf, nf2, _p(cov), _p(pc), _p(ent), _p(sec))
    return cov, pc, ent, sec


def get_stats_py(base_counts, ref, show_n_bases=False, long_format=False):
    """Pure-Python restatement of main.py:14-79 (rows with Python int/float types)."""
    bases = ["A", "C", "G", "T", "DS", "N"]
    if not show_n_bases:
        bases.pop(5)
    k = len(bases)
    nf = 1 / math.log2(k)
    nf2 = 1 / math.log2(k - 1)

    def ent(ps):
        return sum([-(x * math.log2(x)) if x != 0 else 0 for x in ps])

    data = []
    for p, bc in enumerate(base_counts):
        bc = list(bc)
        if not show_n_bases:
            bc.pop(5)
        pcs, e, e2 = [-1] * k, 1, 1
        cov = sum(bc)
        if cov != 0:
            probs = [c / cov for c in bc]
            pcs = [100 * x for x in probs]
            e = nf * ent(probs)
            sb = list(bc)
            sb.pop(int(np.argmax(bc)))
            c2 = sum(sb)
            if c2 != 0:
                e2 = nf2 * ent([c / c2 for c in sb])
        if long_format:
            for base, cnt, pcv in zip(bases, bc, pcs):
                data.append([ref, p + 1, cov, base, cnt, pcv, e, e2])
        else:
            data.append([ref, p + 1, cov] + bc + pcs + [e, e2])
    return data


def summary(cov: np.ndarray, ent: np.ndarray, num_reads: int, ref: str, dp: int):
    """main.py:469-499 over per-position arrays (int-typed values restored)."""
    L = int(cov.size)
    avg_cov = np.mean(cov.astype(np.int64))
    avg_ent = np.mean(ent)
    pc_cov = 100 * (int(np.count_nonzero(cov)) / L)  # len([c for c in coverages if c != 0])
    return {
        "reference_name": ref,
        "reference_length": round(L, dp),
        "num_reads": round(num_reads, dp),
        "pc_reference_coverage": round(pc_cov, dp),
        "avg_depth": round(avg_cov, dp),
        "avg_entropy": round(avg_ent, dp),
    }


def amplicons(cov, ent, sec, tiles):
    """main.py:519-551: per tile [start, end] (inclusive) mean/median of cov, ent, sec."""
    out = []
    L = cov.size
    for start, end in tiles:
        lo, hi = max(start, 0), min(end, L - 1)
        if lo > hi:
            out.append([-1] * 6)
            continue
        cs = cov[lo:hi + 1].astype(np.int64)
        es, ss = ent[lo:hi + 1], sec[lo:hi + 1]
        out.append([np.mean(cs), np.median(cs), np.mean(es), np.median(es), np.mean(ss),
                    np.median(ss)])
    return out


def summary_amplicons_py(rows, tiles):
    """main.py:469-551 as the reference runs it after get_stats (records -> Python lists, then per
    tile a scan of every position, np.mean / np.median of the window); returns the summary means
    and the six amplicon vectors.  Used only as the C4 CPU baseline's workload (bench.py)."""
    coverages = [r[2] for r in rows]
    entropies = [r[-2] for r in rows]
    secondary_entropies = [r[-1] for r in rows]
    avg = (np.mean(coverages), np.mean(entropies), 100 * (len([c for c in coverages if c != 0]) / len(rows)))
    vecs = [[] for _ in range(6)]
    for start, end in tiles:
        cd, ed, sd = [], [], []
        for j, (c, e, s2) in enumerate(zip(coverages, entropies, secondary_entropies)):
            if start <= j <= end:
                cd.append(c)
                ed.append(e)
                sd.append(s2)
        for k, d in enumerate((cd, ed, sd)):
            vecs[2 * k].append(np.mean(d) if d else -1)
            vecs[2 * k + 1].append(np.median(d) if d else -1)
    return avg, vecs


def ref_bcount():
    """The reference's own compiled count.bcount (oracle/_ref), or None when not built."""
    hits = glob.glob(os.path.join(HERE, "_ref", "count*.so"))
    if not hits:
        return None
    spec = importlib.util.spec_from_file_location("count", hits[0])
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.bcount


# ---------------------------------------------------------------- reference-equivalent text
BASES = ["A", "C", "G", "T", "DS", "N"]


def _typed(cov, cnt, pcs, e, s, k):
    if cov == 0:
        return [-1] * k, 1, 1
    nz = sum(1 for v in cnt if v)
    return pcs, e, (1 if nz <= 1 else s)


def rows_text(ref, counts6, show_n, long_format, dp):
    """main.py:457-466 text for one reference from oracle counts (pure Python str(round))."""
    k = 6 if show_n else 5
    cov, pc, ent, sec = stats(counts6, show_n)
    cnts = counts6[:, :k].tolist()
    pcl = pc.T.tolist()
    out = []
    for p in range(counts6.shape[0]):
        c = cnts[p]
        pcs, e, s = _typed(int(cov[p]), c, pcl[p], float(ent[p]), float(sec[p]), k)
        if long_format:
            rows = [[ref, p + 1, int(cov[p]), BASES[j], c[j], pcs[j], e, s] for j in range(k)]
        else:
            rows = [[ref, p + 1, int(cov[p])] + c + pcs + [e, s]]
        for row in rows:
            out.append("\t".join(str(round(x, dp)) if not isinstance(x, str) else x for x in row))
    return "".join(line + "\n" for line in out)


def batch_from_bam(f, t, mmq):
    """Accepted reads of reference t (main.py:165) in the bc_reads layout."""
    sel = (f.tid == t) & ((f.flag & 4) == 0) & (f.mapq.astype(np.int64) >= mmq)
    idx = np.nonzero(sel)[0]
    return dict(pos=f.pos[idx], cig_beg=f.cig_off[:-1][idx].astype(np.uint32),
                cig_n=(f.cig_off[1:] - f.cig_off[:-1])[idx].astype(np.uint32),
                seq_nib=(2 * f.seq_off[:-1][idx] + f.qstart[idx].astype(np.uint64)).astype(
                    np.uint32),
                cigar=f.cigar, seq=f.seq, qual=f.qual), int(idx.size)


def summary_text(ref, counts6, show_n, num_reads, dp, tiles=None, nthreads: int = 0):
    """main.py:469-595 text for one reference from oracle counts."""
    cov, pc, ent, sec = stats(counts6, show_n, nthreads=nthreads)
    del pc
    s = summary(cov, ent, num_reads, ref, dp)
    out = "".join(f"{kk}\t{v}\n" for kk, v in s.items())
    if tiles is not None:
        amps = amplicons(cov, ent, sec, tiles)
        names = ["mean_coverage_amplicon_vector", "median_coverage_amplicon_vector",
                 "mean_entropy_amplicon_vector", "median_entropy_amplicon_vector",
                 "mean_secondary_entropy_amplicon_vector",
                 "median_secondary_entropy_amplicon_vector"]
        for j, name in enumerate(names):
            vec = [a[j] for a in amps]
            out += f"{name}\t" + (", ".join(str(round(x, dp)) for x in vec) if vec else "-") + "\n"
    return out


def split_blocks(text: str, summary_mode: bool):
    """Output text -> (header, {reference: block}) so multi-reference outputs can be compared
    independently of the set iteration order (main.py:92)."""
    lines = text.splitlines(keepends=True)
    parts, header = {}, ""
    if summary_mode:
        cur = None
        for ln in lines:
            if ln.startswith("reference_name\t"):
                cur = ln.split("\t", 1)[1].rstrip("\n")
                parts[cur] = []
            parts[cur].append(ln)
    else:
        header = lines[0] if lines else ""
        for ln in lines[1:]:
            parts.setdefault(ln.split("\t", 1)[0], []).append(ln)
    return header, {k: "".join(v) for k, v in parts.items()}
