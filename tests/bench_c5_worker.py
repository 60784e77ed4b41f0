"""Worker for tests/test_dist.py::test_bench_c5_sharding_world4: one rank of bench.py's C5 leg at
N > 1 with the counting replaced by the oracle (no GPU here), scaled down.  Every rank takes its
contigs by bench.contig_plan (LPT on length), generates them with synth.contig_reads (a contig's
reads independent of the rank holding it) and computes the four summary numbers of main.py:469-499
for each; the per-contig summaries are gathered to rank 0 over the gloo group (the rehearsal of
bench.py's gather step), which checks them against one process computing every contig.

    python tests/bench_c5_worker.py OUT_JSON          (RANK / WORLD_SIZE / MASTER_* from env)
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path[:0] = [REPO, os.path.join(REPO, "oracle")]

import bench  # noqa: E402
import oracle as O  # noqa: E402  (the checker: tests only)
from basecount_amd import synth  # noqa: E402
from basecount_amd.dist import Group  # noqa: E402

SCALE, READS = 4000, 300
CONTIGS = [(n, L // SCALE) for n, L in synth.GRCH38]


def summaries(indices):
    c = synth.CONFIGS["c5"]
    rs = synth.contig_reads(CONTIGS, indices, READS, c["mixed"], c["seed"])
    out = []
    for t, L in enumerate(rs.lengths):
        cnt, (bad, _) = O.bcount(L, 0, synth.batch_arrays(rs, t, 0))
        assert bad == -1
        cov, _, ent, _ = O.stats(cnt, False)
        out.append([float(np.mean(cov.astype(np.int64))), float(np.mean(ent)), float(np.count_nonzero(cov)),
                    float(cov.astype(np.int64).sum())])
    return out


def main():
    group = Group("gloo")
    rank, world = group.rank, group.world
    owner, mine = bench.contig_plan(CONTIGS, world, rank)
    mine_s = summaries(mine)
    # what bench.py gathers per step: every contig's 4 summary doubles, rank by rank
    parts = group.gather_bytes(np.asarray(mine_s, np.float64).tobytes())
    loads = [v[0] for v in group.all_gather_ints([sum(CONTIGS[i][1] for i in mine)])]
    # the full-size plan too (positions per rank at GRCh38 lengths)
    _, full_mine = bench.contig_plan(list(synth.GRCH38), world, rank)
    full_loads = [v[0] for v in group.all_gather_ints([sum(synth.GRCH38[i][1] for i in full_mine)])]
    if rank == 0:
        got = {}
        for r, part in enumerate(parts):
            vals = np.frombuffer(part, np.float64).reshape(-1, 4).tolist()
            idx = [i for i, (n, _) in enumerate(CONTIGS) if owner[n] == r]
            got.update({CONTIGS[i][0]: v for i, v in zip(idx, vals)})
        want = dict(zip([n for n, _ in CONTIGS], summaries(range(len(CONTIGS)))))
        with open(sys.argv[1], "w") as fh:
            json.dump({"got": got, "want": want, "loads": loads, "full_loads": full_loads,
                       "owner": owner}, fh)
    group.close()


if __name__ == "__main__":
    main()
