"""Generate the golden fixtures in tests/golden/ by running the REFERENCE itself.

Run in the build container only (needs /root/reference, oracle/_ref and the pysam shim):

    python tests/golden/make_golden.py

What it writes (all data, no reference source):
  *.bam / *.bed            seeded synthetic inputs + hand-built edge cases
  cli/<case>.out.gz        stdout of the reference CLI (basecount.main:run, main.py:378-595)
  cli/<case>.err           exception line(s) when the reference raises
  manifest.json            case -> {bam, args, stdout / error}
  bcount/<case>.json       inputs and outputs of the reference's compiled count.bcount
                           (count.cpp:7-99) on the accepted reads of each edge-case reference

The reference runs with PYTHONHASHSEED=0 (it iterates a set of reference names, main.py:92) and
PYTHONDONTWRITEBYTECODE=1 (never write into /root/reference).
"""
from __future__ import annotations

import gzip
import hashlib
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from basecount_amd import synth  # noqa: E402
from basecount_amd.bam import BamFile, pack_seq, write_bam  # noqa: E402

REF = "/root/reference"
OPS = "MIDNSHP=XB"


def parse_cigar(s: str):
    out, num = [], ""
    for ch in s:
        if ch.isdigit():
            num += ch
        else:
            out.append((int(num) << 4) | OPS.index(ch))
            num = ""
    return out


class Builder:
    def __init__(self, refs):
        self.refs = refs
        self.recs = []

    def add(self, tid, pos, cigar, seq, qual=None, flag=0, mapq=60):
        if qual is None:
            qual = [30] * len(seq)
        self.recs.append((tid, pos, flag, mapq, parse_cigar(cigar) if cigar else [], seq, qual))

    def write(self, path):
        n = len(self.recs)
        tid = np.array([r[0] for r in self.recs], np.int32)
        pos = np.array([r[1] for r in self.recs], np.int32)
        flag = np.array([r[2] for r in self.recs], np.uint16)
        mapq = np.array([r[3] for r in self.recs], np.uint8)
        cig_off = np.zeros(n + 1, np.uint64)
        cig_off[1:] = np.cumsum([len(r[4]) for r in self.recs])
        cigar = np.array([w for r in self.recs for w in r[4]], np.uint32)
        l_seq = np.array([len(r[5]) for r in self.recs], np.int32)
        seqs = [pack_seq(r[5]) if r[5] else np.zeros(0, np.uint8) for r in self.recs]
        seq_off = np.zeros(n + 1, np.uint64)
        seq_off[1:] = np.cumsum([s.size for s in seqs])
        seq = np.concatenate(seqs) if n else np.zeros(0, np.uint8)
        quals = [np.array(r[6] if r[6] != "missing" else [0xFF] * len(r[5]), np.uint8)
                 for r in self.recs]
        qual_off = np.zeros(n + 1, np.uint64)
        qual_off[1:] = np.cumsum([q.size for q in quals])
        qual = np.concatenate(quals) if n else np.zeros(0, np.uint8)
        write_bam(path, [r[0] for r in self.refs], [r[1] for r in self.refs], tid, pos, flag,
                  mapq, cig_off, cigar, l_seq, seq_off, seq, qual_off, qual, level=6)


def rand_read(rng, L, alphabet="ACGT"):
    """Random CIGAR over M/I/D/N/=/X/P with optional S/H ends, staying inside [0, L)."""
    ops = []
    if rng.random() < 0.3:
        ops.append(("H", int(rng.integers(1, 5))))
    if rng.random() < 0.5:
        ops.append(("S", int(rng.integers(1, 6))))
    span = 0
    nmid = int(rng.integers(1, 6))
    for k in range(nmid):
        op = "M" if k == 0 or k == nmid - 1 else str(rng.choice(list("MIDN=XP")))
        ln = int(rng.integers(1, 30 if op in "M=X" else 6))
        ops.append((op, ln))
        if op in "MDN=X":
            span += ln
    if rng.random() < 0.5:
        ops.append(("S", int(rng.integers(1, 6))))
    if rng.random() < 0.3:
        ops.append(("H", int(rng.integers(1, 5))))
    qlen = sum(ln for op, ln in ops if op in "MIS=X")
    seq = "".join(rng.choice(list(alphabet), qlen))
    qual = rng.integers(0, 42, qlen).tolist()
    pos = int(rng.integers(0, max(1, L - span)))
    return pos, "".join(f"{ln}{op}" for op, ln in ops), seq, qual


def build_edge(path):
    b = Builder([("chrA", 60), ("chrB", 200), ("chrC", 1000), ("chrD", 30)])
    rng = np.random.default_rng(11)
    b.add(0, 0, "10M", "ACGTNACGTN", list(range(0, 50, 5)))
    b.add(0, 5, "3S7M2S", "TTTACGTACGGG", [10, 20, 30, 40, 2, 15, 25, 35, 41, 5, 5, 5])
    b.add(0, 10, "4M2I4M", "AAAACCGGGG", [40] * 10, mapq=20)
    b.add(0, 12, "3M3D3M", "CCCGGG", [25] * 6, mapq=30)
    b.add(0, 15, "2H5M", "ACGTA", [35] * 5, mapq=45)
    b.add(0, 20, "5M10N5M", "AAAAATTTTT", [12] * 10)
    b.add(0, 20, "5=2X3M", "A=RYKMNACG", [38] * 10)
    b.add(0, 25, "4M1P4M", "GGGGCCCC", [39] * 8, mapq=0)
    b.add(0, 30, "10M", "CCCCCCCCCC", [40] * 10, flag=4)          # unmapped, tid set
    b.add(0, 30, "3M2S3M", "ACGTTGCA", [30] * 8)                  # mid-read soft clip
    b.add(0, 50, "10M", "TTTTTTTTTT", [41] * 10, flag=256 | 1024)  # last base = 59 (in range)
    b.add(0, 40, "5M", "NNNNN", [33] * 5, flag=512)
    b.add(0, 33, "1S3M1S", "GACGT", [20] * 5, mapq=59)
    b.add(0, 44, "2M1I2M1D2M", "ACGTACG", [18, 22, 19, 40, 3, 0, 41])
    b.add(2, 100, "3M2B3M", "ACGTAC", [30] * 6)                   # op 9 'B' is ignored
    for _ in range(60):
        t = int(rng.choice([0, 1, 1, 2]))
        L = [60, 200, 1000][t]
        pos, cig, seq, qual = rand_read(rng, L, alphabet="ACGTACGTACGTN=R")
        b.add(t, pos, cig, seq, qual, mapq=int(rng.integers(0, 61)),
              flag=int(rng.choice([0, 0, 0, 16, 256, 2048])))
    for _ in range(40):  # a dense pile on chrC for entropy variety
        pos, cig, seq, qual = rand_read(rng, 120)
        b.add(2, 400 + pos, cig, seq, qual, mapq=int(rng.integers(20, 61)))
    b.add(-1, -1, "", "ACGT", [30] * 4, flag=4, mapq=0)             # unmapped, no reference
    b.write(path)


def build_errors():
    out = {}
    b = Builder([("chrA", 60)])
    b.add(0, 0, "10M", "ACGTACGTAC")
    b.add(0, 57, "5M", "ACGTA", [40, 40, 40, 10, 10])   # 60,61 out of range (qual 10)
    b.write(os.path.join(HERE, "err_range.bam"))
    out["err_range"] = "err_range.bam"
    b = Builder([("chrA", 60)])
    b.add(0, 0, "10M", "ACGTACGTAC")
    b.add(0, 55, "2M5D", "AC")                          # deletion runs past the end
    b.write(os.path.join(HERE, "err_range_del.bam"))
    b = Builder([("chrA", 60)])
    b.add(0, 0, "10M", "ACGTACGTAC")
    b.add(0, 5, "", "ACGTA")                             # mapped, no CIGAR -> None
    b.write(os.path.join(HERE, "err_nocigar.bam"))
    b = Builder([("chrA", 60)])
    b.add(0, 0, "10M", "ACGTACGTAC")
    b.add(0, 5, "5M", "ACGTA", "missing")                # QUAL absent -> None
    b.write(os.path.join(HERE, "err_noqual.bam"))
    b = Builder([("chrA", 60), ("chrB", 40)])
    for i in range(7):
        b.add(i % 2, 3 * i, "5M", "ACGTA")
    b.add(1, 38, "4M", "ACGT")                            # out of range on chrB (ordinal 7)
    b.add(0, 2, "", "ACG")                                # no CIGAR on chrA   (ordinal 8)
    b.add(0, 58, "4M", "GGGG")                            # out of range chrA  (ordinal 9)
    b.write(os.path.join(HERE, "err_order.bam"))
    return out


def run_ref(args, hashseed="0"):
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1", PYTHONHASHSEED=hashseed,
               PYTHONPATH=os.pathsep.join([os.path.join(REPO, "oracle", "pysam_shim"),
                                           os.path.join(REPO, "oracle", "_ref"), REF, REPO]))
    code = "import sys; sys.argv=['basecount']+sys.argv[1:]; import basecount.main as M; M.run()"
    p = subprocess.run([sys.executable, "-c", code] + args, env=env, capture_output=True)
    return p.returncode, p.stdout, p.stderr.decode()


def exc_line(stderr: str) -> str:
    lines = [ln for ln in stderr.strip().splitlines()]
    for i, ln in enumerate(lines):
        if not ln.startswith(" ") and (":" in ln) and ("Error" in ln.split(":")[0]
                                                      or "Exception" in ln.split(":")[0]):
            last = i
    return lines[last] if lines else ""


# Cases added after the first generation (run with --add: the BAMs and the other cases are kept).
# dp 17: more digits than a double holds, so the raw entropies are compared bit for bit through
# the CLI (byte identity must not rest on rounding hiding one-ulp log2 differences).
ADDED = {
    "edge_dp17_shown": ("edge.bam", ["--decimal-places", "17", "--show-n-bases"]),
    "edge_long_dp17": ("edge.bam", ["--long-format", "--decimal-places", "17"]),
    "mixed_dp17": ("mixed.bam", ["--decimal-places", "17"]),
    "mixed_bed_dp16": ("mixed.bam", ["--summarise-with-bed", "scheme.bed", "--decimal-places", "16"]),
}


def add_cases():
    with open(os.path.join(HERE, "manifest.json")) as fh:
        cases = json.load(fh)
    os.chdir(HERE)
    for name, (bam, args) in ADDED.items():
        rc, out, err = run_ref([bam] + args)
        rec = {"bam": bam, "args": args, "returncode": rc, "hashseed": "0"}
        assert rc == 0, err
        fn = f"cli/{name}.out.gz"
        with open(os.path.join(HERE, fn), "wb") as fh:
            fh.write(gzip.compress(out, compresslevel=9, mtime=0))
        rec["stdout"] = fn
        rec["sha256"] = hashlib.sha256(out).hexdigest()
        cases[name] = rec
        print(name, rc)
    with open(os.path.join(HERE, "manifest.json"), "w") as fh:
        json.dump(cases, fh, indent=1, sort_keys=True)


def main():
    if "--add" in sys.argv:
        return add_cases()
    os.makedirs(os.path.join(HERE, "cli"), exist_ok=True)
    os.makedirs(os.path.join(HERE, "bcount"), exist_ok=True)
    synth.write_bam(synth.make_config("c1"), os.path.join(HERE, "c1.bam"), level=6)
    mixed = synth.make_reads([("MN908947.3", 29_903)], 4000, mixed=True, seed=3)
    synth.write_bam(mixed, os.path.join(HERE, "mixed.bam"), level=6)
    with open(os.path.join(HERE, "scheme.bed"), "w") as fh:
        fh.write(synth.artic_bed())
    with open(os.path.join(HERE, "edge.bed"), "w") as fh:  # tiles hitting every edge-case contig
        fh.write("chrA\t0\t4\tEX_1_LEFT\t1\t+\nchrA\t28\t31\tEX_1_RIGHT\t1\t-\n"
                 "chrA\t20\t25\tEX_2_LEFT\t2\t+\nchrA\t2\t6\tEX_2_LEFT_alt2\t2\t+\n"
                 "chrA\t70\t75\tEX_2_RIGHT\t2\t-\nchrA\t500\t505\tEX_3_LEFT\t1\t+\n"
                 "chrA\t990\t1200\tEX_3_RIGHT\t1\t-\nchrA\t5\t9\tEX_4_RIGHT\t1\t-\n")
    build_edge(os.path.join(HERE, "edge.bam"))
    build_errors()

    cases = {}

    def case(name, bam, args, hashseed="0"):
        rc, out, err = run_ref([bam] + args, hashseed)
        rec = {"bam": bam, "args": args, "returncode": rc, "hashseed": hashseed}
        if rc == 0:
            fn = f"cli/{name}.out.gz"
            with open(os.path.join(HERE, fn), "wb") as fh:
                fh.write(gzip.compress(out, compresslevel=9, mtime=0))
            rec["stdout"] = fn
            rec["sha256"] = hashlib.sha256(out).hexdigest()
        else:
            rec["error"] = exc_line(err)
            rec["stdout_prefix_sha256"] = hashlib.sha256(out).hexdigest()
        cases[name] = rec
        print(name, rc, rec.get("error", ""))

    os.chdir(HERE)
    case("c1_default", "c1.bam", [])
    case("c1_long", "c1.bam", ["--long-format"])
    case("c1_shown", "c1.bam", ["--show-n-bases"])
    case("c1_summary", "c1.bam", ["--summarise"])
    case("c1_bed", "c1.bam", ["--summarise-with-bed", "scheme.bed"])
    case("c1_q20_m30", "c1.bam", ["--min-base-quality", "20", "--min-mapping-quality", "30"])
    case("c1_dp5", "c1.bam", ["--decimal-places", "5"])
    case("mixed_default", "mixed.bam", [])
    case("mixed_shown_long", "mixed.bam", ["--show-n-bases", "--long-format"])
    case("mixed_q20_m30", "mixed.bam", ["--min-base-quality", "20", "--min-mapping-quality", "30"])
    case("mixed_bed", "mixed.bam", ["--summarise-with-bed", "scheme.bed"])
    case("mixed_bed_dp1_shown", "mixed.bam",
         ["--summarise-with-bed", "scheme.bed", "--decimal-places", "1", "--show-n-bases"])
    for mbq in (0, 20, 40):
        for mmq in (0, 30, 60):
            a = ["--min-base-quality", str(mbq), "--min-mapping-quality", str(mmq)]
            case(f"edge_q{mbq}_m{mmq}", "edge.bam", a + ["--show-n-bases"])
            case(f"edge_q{mbq}_m{mmq}_wide5", "edge.bam", a)
            case(f"edge_q{mbq}_m{mmq}_bed", "edge.bam", a + ["--summarise-with-bed", "edge.bed"])
    case("edge_long", "edge.bam", ["--long-format"])
    case("edge_long_shown_dp0", "edge.bam", ["--long-format", "--show-n-bases",
                                              "--decimal-places", "0"])
    case("edge_summary_dp7", "edge.bam", ["--summarise", "--decimal-places", "7"])
    case("edge_chunk3", "edge.bam", ["--chunk-size", "3", "--show-n-bases"])
    case("edge_refs_subset", "edge.bam", ["--references", "chrA"])
    case("edge_refs_all", "edge.bam", ["--references", "chrA", "chrB", "--references", "chrC",
                                       "chrD", "chrA"])
    case("edge_refs_invalid", "edge.bam", ["--references", "chrZ"])
    case("edge_mbq_twice", "edge.bam", ["--min-base-quality", "1", "--min-base-quality", "2"])
    case("err_range", "err_range.bam", [])
    case("err_range_q20", "err_range.bam", ["--min-base-quality", "20"])
    case("err_range_del", "err_range_del.bam", [])
    case("err_nocigar", "err_nocigar.bam", [])
    case("err_noqual", "err_noqual.bam", [])
    case("err_order", "err_order.bam", [])
    case("err_order_chunk3", "err_order.bam", ["--chunk-size", "3"])
    case("err_order_chunk8", "err_order.bam", ["--chunk-size", "8"])
    case("err_order_chunk9", "err_order.bam", ["--chunk-size", "9"])
    case("err_order_m1", "err_order.bam", ["--chunk-size", "8", "--summarise"])
    for seed in ("1", "2", "5", "6"):
        case(f"err_order_chunk7_h{seed}", "err_order.bam", ["--chunk-size", "7"], seed)
        case(f"edge_default_h{seed}", "edge.bam", [], seed)
        case(f"edge_bed_h{seed}", "edge.bam", ["--summarise-with-bed", "edge.bed"], seed)
    with open(os.path.join(HERE, "manifest.json"), "w") as fh:
        json.dump(cases, fh, indent=1, sort_keys=True)

    # ---- count.bcount vectors from the reference's own compiled count.cpp ----------------
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    from oracle import ref_bcount

    bcount = ref_bcount()
    f = BamFile(os.path.join(HERE, "edge.bam"))
    vec = {}
    for t, (name, L) in enumerate(zip(f.references, f.lengths)):
        reads, quals, starts, ctuples = [], [], [], []
        for i in range(f.n_records):
            if f.tid[i] != t or (f.flag[i] & 4):
                continue
            reads.append(f.query_alignment_sequence(i))
            quals.append(f.query_alignment_qualities(i).tolist())
            starts.append(int(f.pos[i]))
            ctuples.append(f.cigartuples(i))
        for mbq in (0, 20, 40):
            res = bcount(L, mbq, reads, quals, starts, ctuples)
            vec[f"edge_{name}_q{mbq}"] = dict(ref_len=L, mbq=mbq, reads=reads, qualities=quals,
                                              starts=starts, ctuples=ctuples, expected=res)
    # adapter-only inputs: letters outside the BAM alphabet, empty batch, range error
    vec["letters"] = dict(ref_len=12, mbq=0, reads=["ACGTNacgtn=XY."], qualities=[[30] * 14],
                          starts=[0], ctuples=[[(0, 12), (1, 2)]],
                          expected=bcount(12, 0, ["ACGTNacgtn=XY."], [[30] * 14], [0],
                                          [[(0, 12), (1, 2)]]))
    vec["empty"] = dict(ref_len=5, mbq=7, reads=[], qualities=[], starts=[], ctuples=[],
                        expected=bcount(5, 7, [], [], [], []))
    try:
        bcount(8, 0, ["ACGTACGT"], [[30] * 8], [4], [[(0, 8)]])
    except IndexError as e:
        vec["range"] = dict(ref_len=8, mbq=0, reads=["ACGTACGT"], qualities=[[30] * 8],
                            starts=[4], ctuples=[[(0, 8)]], error=["IndexError", str(e)])
    with open(os.path.join(HERE, "bcount", "vectors.json"), "w") as fh:
        json.dump(vec, fh)
    print("bcount vectors:", len(vec))


if __name__ == "__main__":
    main()
