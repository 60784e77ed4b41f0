"""The oracle (oracle/) pinned against the reference itself: the golden fixtures were produced by
running the reference's compiled count.cpp and its Python main.py (tests/golden/make_golden.py)."""
import gzip
import json
import os

import numpy as np
import pytest

import oracle as O
from basecount_amd.bam import BamFile
from basecount_amd.count import pack
from basecount_amd.scheme import load_scheme


def _vectors(golden):
    with open(os.path.join(golden, "bcount", "vectors.json")) as fh:
        return json.load(fh)


def test_oracle_bcount_matches_reference_vectors(golden):
    vec = _vectors(golden)
    assert len(vec) >= 15
    for name, v in vec.items():
        b = pack(v["reads"], v["qualities"], v["starts"], [[tuple(t) for t in c] for c in v["ctuples"]])
        out, (br, bp) = O.bcount(v["ref_len"], v["mbq"], b)
        if "error" in v:
            assert br >= 0, name
            assert v["error"][1] == (f"vector::_M_range_check: __n (which is {bp}) >= "
                                     f"this->size() (which is {v['ref_len']})")
        else:
            assert br == -1, name
            assert out.tolist() == v["expected"], name


def test_oracle_matches_compiled_reference_on_random_reads():
    ref = O.ref_bcount()
    if ref is None:
        pytest.skip("oracle/_ref not built (reference sources absent)")
    rng = np.random.default_rng(5)
    for trial in range(20):
        L = int(rng.integers(50, 400))
        reads, quals, starts, ctuples = [], [], [], []
        for _ in range(int(rng.integers(0, 60))):
            ops = [(0, int(rng.integers(1, 20)))]
            for _ in range(int(rng.integers(0, 4))):
                ops.append((int(rng.choice([0, 1, 2, 3, 6, 7, 8, 9])), int(rng.integers(1, 6))))
            ops.append((0, int(rng.integers(1, 20))))
            span = sum(n for o, n in ops if o in (0, 2, 3, 7, 8))
            q = sum(n for o, n in ops if o in (0, 1, 7, 8))
            if span >= L:
                continue
            reads.append("".join(rng.choice(list("ACGTN=RYacgt"), q)))
            quals.append(rng.integers(0, 45, q).tolist())
            starts.append(int(rng.integers(0, L - span)))
            ctuples.append(ops)
        mbq = int(rng.choice([0, 10, 30]))
        exp = ref(L, mbq, reads, quals, starts, ctuples)
        out, (br, _) = O.bcount(L, mbq, pack(reads, quals, starts, ctuples))
        assert br == -1 and out.tolist() == exp, trial


def _cases(manifest, kinds):
    for name, c in sorted(manifest.items()):
        if c["returncode"] != 0:
            continue
        a = c["args"]
        summ = "--summarise" in a or "--summarise-with-bed" in a
        if ("summary" in kinds) == summ:
            yield name, c


def _opt(args, flag, default):
    return args[args.index(flag) + 1] if flag in args else default


def _oracle_output(golden, c):
    a = c["args"]
    f = BamFile(os.path.join(golden, c["bam"]))
    mbq = int(_opt(a, "--min-base-quality", 0))
    mmq = int(_opt(a, "--min-mapping-quality", 0))
    dp = int(_opt(a, "--decimal-places", 3))
    show_n = "--show-n-bases" in a
    long_format = "--long-format" in a
    refs = set(f.references)
    if "--references" in a:
        refs = set(x for x in a[a.index("--references") + 1:] if not x.startswith("--"))
    bed = _opt(a, "--summarise-with-bed", None)
    blocks = {}
    for t, (ref, L) in enumerate(zip(f.references, f.lengths)):
        if ref not in refs:
            continue
        b, nreads = O.batch_from_bam(f, t, mmq)
        counts, (br, _) = O.bcount(L, mbq, b)
        assert br == -1
        if "--summarise" in a or bed:
            tiles = None
            if bed:
                sch = load_scheme(os.path.join(golden, bed))
                tiles = [(x[2]["inside_start"], x[2]["inside_end"]) for x in sch]
            blocks[ref] = O.summary_text(ref, counts, show_n, nreads, dp, tiles)
        else:
            blocks[ref] = O.rows_text(ref, counts, show_n, long_format, dp)
    return blocks


@pytest.mark.parametrize("kind", ["rows", "summary"])
def test_oracle_reproduces_reference_cli(golden, manifest, kind):
    n = 0
    for name, c in _cases(manifest, kind):
        with open(os.path.join(golden, c["stdout"]), "rb") as fh:
            exp = gzip.decompress(fh.read()).decode()
        _, exp_blocks = O.split_blocks(exp, kind == "summary")
        got = _oracle_output(golden, c)
        assert got == exp_blocks, name
        n += 1
    assert n >= 10


@pytest.mark.parametrize("nthreads", [1, 3, 8])
def test_all_cores_oracle_matches_single_thread(nthreads):
    """The all-cores CPU baseline (mt_oracle.c) computes exactly what the single-thread
    restatement does, including the first out-of-range read."""
    from basecount_amd import synth

    rs = synth.make_reads([("a", 4_000)], 3_000, True, 12)
    b = synth.batch_arrays(rs, 0, 0)
    for L, mbq in ((4_000, 0), (4_000, 20), (2_500, 0)):
        e1, bad1 = O.bcount(L, mbq, b)
        e2, bad2 = O.bcount(L, mbq, b, nthreads=nthreads)
        assert bad1 == bad2
        if bad1[0] < 0:
            assert np.array_equal(e1, e2)
            for show_n in (False, True):
                s1 = O.stats(e1, show_n)
                s2 = O.stats(e1, show_n, nthreads=nthreads)
                assert all(np.array_equal(x, y) for x, y in zip(s1, s2))
