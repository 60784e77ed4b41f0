"""End-to-end timing of the CLI path: BAM decode -> HBM -> kernels -> TSV.

    python scripts/e2e.py [--config c2|c3|c5] [--summarise]

Writes the config's synthetic BAM, then times (wall clock, warm): the host decode
(BGZF inflate + record decode + read selection), get_basecounts (upload + kernels + download),
the byte-exact formatter, and the whole `basecount BAM` run with its output sent to a file.
Prints one JSON line.  (The reference's own CLI cannot run on the GPU box; its C2 time in the
build container is in SURVEY §3: ~1.1-1.4 s.)
"""
import argparse
import contextlib
import io
import json
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from basecount_amd import fmt, main as M, synth  # noqa: E402
from basecount_amd.bam import BamFile  # noqa: E402


def _t(fn, reps=3):
    best = float("inf")
    out = None
    for _ in range(reps):
        t0 = time.perf_counter()
        out = fn()
        best = min(best, time.perf_counter() - t0)
    return best, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--summarise", action="store_true")
    ap.add_argument("--profile", action="store_true", help="cProfile get_basecounts (stderr)")
    args = ap.parse_args()
    rs = synth.make_config(args.config)
    tmp = tempfile.mkdtemp(prefix="bc_e2e_")
    bam = os.path.join(tmp, f"{args.config}.bam")
    synth.write_bam(rs, bam)
    res = {"config": args.config, "bam_bytes": os.path.getsize(bam), "reads": int(rs.n),
           "positions": int(sum(rs.lengths)), "mode": "summary" if args.summarise else "rows"}

    def decode():
        with BamFile(bam) as f:
            return f.select(0, [True] * len(f.references)).n_accepted
    res["decode_s"], _ = _t(decode)

    mode = "summary" if args.summarise else "rows"
    res["get_basecounts_s"], data = _t(lambda: M.get_basecounts(bam, _mode=mode))
    if args.profile:
        import cProfile
        import pstats
        pr = cProfile.Profile()
        pr.enable()
        M.get_basecounts(bam, _mode=mode)
        pr.disable()
        pstats.Stats(pr, stream=sys.stderr).sort_stats("tottime").print_stats(25)

    if not args.summarise:
        def format_all():
            n = 0
            for ref, v in data.items():
                d = v["rows"].d
                n += len(fmt.rows_text(ref, d.counts, d.pc, d.ent, d.sec, 3, False))
            return n
        res["format_s"], res["tsv_bytes"] = _t(format_all)

    out_path = os.path.join(tmp, "out.tsv")
    argv = [bam] + (["--summarise"] if args.summarise else [])

    def cli():
        with open(out_path, "w") as fh, contextlib.redirect_stdout(fh):
            M.run(argv)
    res["cli_s"], _ = _t(cli)
    res["cli_positions_per_s"] = res["positions"] / res["cli_s"]
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
