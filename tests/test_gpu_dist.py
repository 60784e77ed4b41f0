"""Multi-rank CLI on the GPU: two ranks share the box's one GPU (the exchange over gloo, since
RCCL needs one GPU per rank), each counting its shard of the references with the HIP kernels;
the output must be byte-identical to a single process (and to the reference's goldens)."""
import gzip
import json
import os
import socket
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
GOLD = os.path.join(HERE, "golden")


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _cli(world, args, tmp_path, name, hashseed):
    out = tmp_path / f"{name}.out"
    env = dict(os.environ, PYTHONPATH=REPO, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()),
               BASECOUNT_DIST_BACKEND="gloo", PYTHONHASHSEED=str(hashseed))
    with open(out, "ab") as fh:
        procs = []
        for r in range(world):
            e = dict(env, WORLD_SIZE=str(world), RANK=str(r), LOCAL_RANK=str(r)) if world > 1 else env
            procs.append(subprocess.Popen([sys.executable, "-m", "basecount_amd", *args], stdout=fh,
                                          stderr=subprocess.PIPE, env=e, cwd=GOLD))
        errs = [p.communicate(timeout=600)[1] for p in procs]
    assert [p.returncode for p in procs] == [0] * world, [e.decode()[-1500:] for e in errs]
    return out.read_bytes()


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["edge_default_h1", "edge_long", "edge_summary_dp7", "edge_bed_h1"])
def test_cli_two_ranks_match_golden(tmp_path, case):
    man = json.load(open(os.path.join(GOLD, "manifest.json")))[case]
    args = [man["bam"], *man["args"]]
    multi = _cli(2, args, tmp_path, "multi", man["hashseed"])
    single = _cli(1, args, tmp_path, "single", man["hashseed"])
    with gzip.open(os.path.join(GOLD, man["stdout"])) as fh:
        gold = fh.read()
    assert single == gold
    assert multi == gold
