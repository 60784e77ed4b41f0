"""The multi-rank launch paths on CPU (no GPU): bench.py --gpus N starting its own ranks, and the
RCCL id rendezvous of dist.py with a stub id, 2 and 3 ranks."""
import json
import os
import socket
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
BENCH = os.path.join(REPO, "bench.py")


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(BASECOUNT_DIST_BACKEND="gloo", HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="")
    env.update(kw)
    return env


@pytest.mark.parametrize("n", [2, 3])
def test_bench_gpus_n_starts_n_ranks(n):
    """bench.py --gpus N without a launcher runs N rank processes in one process group."""
    p = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--launch-check"], env=_env(),
                       capture_output=True, timeout=240)
    assert p.returncode == 0, p.stderr.decode()[-3000:]
    lines = [ln for ln in p.stdout.decode().splitlines() if ln.startswith("{")]
    assert len(lines) == 1  # only rank 0 prints on stdout
    got = json.loads(lines[0])
    assert got["n_gpus"] == n and got["ranks"] == list(range(n))
    assert len(set(got["pids"])) == n and os.getpid() not in got["pids"]


def test_bench_failing_rank_fails_the_job():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-check"],
                       env=_env(BASECOUNT_DIST_BACKEND="no-such-backend"), capture_output=True, timeout=240)
    assert p.returncode != 0
    assert b"no-such-backend" in p.stderr


def test_bench_world_size_must_match_gpus():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-check"],
                       env=_env(WORLD_SIZE="3", RANK="0", LOCAL_RANK="0"), capture_output=True, timeout=120)
    assert p.returncode != 0 and b"WORLD_SIZE=3" in p.stderr


_RDZV = """
import sys
sys.path.insert(0, {repo!r})
from basecount_amd.dist import rendezvous_init
rank, world = int(sys.argv[1]), int(sys.argv[2])
# init: the id itself (the RCCL communicator's stand-in)
uid = rendezvous_init(rank, world, lambda: bytes(range(128)), lambda u: u, timeout=60)
sys.stdout.write(uid.hex())
"""


@pytest.mark.parametrize("world", [2, 3])
def test_rendezvous_id_every_rank_gets_rank0s_bytes(world):
    """dist.rendezvous_init: rank 0's id reaches every rank (the RCCL id handshake, without RCCL)."""
    env = _env(MASTER_ADDR="127.0.0.1", BASECOUNT_RDZV_PORT=str(_free_port()))
    code = _RDZV.format(repo=REPO)
    # the non-root ranks start first: they must wait for the root's socket
    procs = [subprocess.Popen([sys.executable, "-c", code, str(r), str(world)], env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE) for r in reversed(range(world))]
    outs = [p.communicate(timeout=120) for p in procs]
    assert [p.returncode for p in procs] == [0] * world, [o[1].decode()[-2000:] for o in outs]
    assert {o[0].decode() for o in outs} == {bytes(range(128)).hex()}


def test_rendezvous_port_taken_fails_fast():
    """A port already bound by someone else: rank 0 says so at once, the others give up within
    their (short) timeout instead of hanging for minutes."""
    import time

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        s.listen(1)
        port = s.getsockname()[1]
        env = _env(MASTER_ADDR="127.0.0.1", BASECOUNT_RDZV_PORT=str(port), BASECOUNT_RDZV_TIMEOUT="3")
        code = _RDZV.format(repo=REPO).replace(", timeout=60", "")
        t0 = time.monotonic()
        p = subprocess.run([sys.executable, "-c", code, "0", "2"], env=env, capture_output=True, timeout=60)
        assert p.returncode != 0 and b"rendezvous port" in p.stderr
        assert time.monotonic() - t0 < 30
