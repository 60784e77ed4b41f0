"""Worker for tests/test_dist.py: runs basecount_amd.main.run() as one rank of a gloo group
(or as a single process), with get_basecounts replaced by a deterministic CPU stand-in so the
sharding / error exchange / output ordering of the CLI is exercised without a GPU.

    python tests/dist_worker.py MODE [cli args...]     (RANK / WORLD_SIZE / MASTER_* from env)
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from basecount_amd import main as M  # noqa: E402

REFS = {"chrA": 1000, "chrB": 37, "chrC": 0, "chrD": 4000, "chrE": 250}


def fake_get_basecounts(bam, references=None, min_base_quality=0, min_mapping_quality=0,
                        chunk_size=1000000, show_n_bases=False, long_format=False, *, device=None,
                        _mode="rows", _tiles=None, _group=None):
    from basecount_amd.dist import shard

    k = 6 if show_n_bases else 5
    refs = dict(REFS, chrC=3) if (_mode == "summary" and not os.environ.get("FAKE_EMPTY_REF")) else REFS
    nreads = {r: 3 * L // 7 + 1 for r, L in refs.items()}
    from basecount_amd.dist import agree_order

    # the set order of this process (PYTHONHASHSEED), as main.py:92 iterates it; with a group,
    # rank 0's order (agree_order), exactly as the real get_basecounts does
    order = list(set(REFS))
    owner = None
    mine = order
    if _group is not None:
        order = agree_order(_group, order)
        owner = shard(order, {r: refs[r] + 100 * nreads[r] for r in order}, _group.world)
        mine = [r for r in order if owner[r] == _group.rank]
    out = {}
    for ref in mine:
        L = refs[ref]
        rng = np.random.default_rng(sum(map(ord, ref)))
        counts = rng.integers(0, 9, (k, L)).astype(np.int32)
        counts[:, ::5] = 0
        cov = counts.sum(0).astype(np.int32)
        with np.errstate(invalid="ignore", divide="ignore"):
            pc = np.where(cov > 0, 100.0 * (counts / np.maximum(cov, 1)), -1.0)
        ent = rng.random(L)
        sec = rng.random(L)
        if _mode == "rows":
            out[ref] = {"rows": M.Rows(ref, M.RefData(counts, pc, ent, sec, cov), long_format),
                        "num_reads": nreads[ref]}
        else:
            s = {"L": L}
            if L:
                s.update(avg_cov=np.float64(cov.mean()), avg_ent=np.float64(ent.mean()),
                         nnz=int((cov > 0).sum()))
                if _tiles is not None:
                    t = _tiles(ref)
                    if t is not None:
                        amp = rng.random((len(t), 6))
                        s["amplicons"] = (amp, [i % 3 == 0 for i in range(len(t))])
            out[ref] = {"summary": s, "num_reads": nreads[ref], "length": L}
    if _group is not None:
        return out, owner, order
    return out


M.get_basecounts = fake_get_basecounts
if __name__ == "__main__":
    M.run(sys.argv[1:])
