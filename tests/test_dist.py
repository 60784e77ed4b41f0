"""Multi-process (one process per GPU) CLI paths on CPU: gloo, world_size 2.

The counting itself needs a GPU; these tests cover what the ranks exchange: reference
sharding, the per-reference gather to rank 0 and the ordered per-position output, checked to
be byte-identical to a single process."""
import os
import socket
import subprocess
import sys

import pytest

from basecount_amd.dist import shard

HERE = os.path.dirname(os.path.abspath(__file__))
WORKER = os.path.join(HERE, "dist_worker.py")


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(world: int, args, tmp_path, name, expect_fail=False, extra_env=None, rank_env=None):
    out = tmp_path / f"{name}.out"
    env = dict(os.environ, **dict({"PYTHONHASHSEED": "0"}, **(extra_env or {})), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()),
               WORLD_SIZE=str(world), BASECOUNT_DIST_BACKEND="gloo", CUDA_VISIBLE_DEVICES="",
               HIP_VISIBLE_DEVICES="")
    with open(out, "ab") as fh:
        procs = []
        for r in range(world):
            e = dict(env, RANK=str(r), LOCAL_RANK=str(r), **((rank_env or {}).get(r, {})))
            if world == 1:
                for v in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
                    e.pop(v)
            procs.append(subprocess.Popen([sys.executable, WORKER, *args], stdout=fh,
                                          stderr=subprocess.PIPE, env=e))
        errs = [p.communicate(timeout=240)[1] for p in procs]
    codes = [p.returncode for p in procs]
    if expect_fail:  # rank 0 (which prints) raises; the launcher then fails the job
        assert codes[0] != 0, codes
        return out.read_bytes(), [e.decode().strip().splitlines()[-1] for e in errs]
    assert codes == [0] * world, (codes, [e.decode()[-2000:] for e in errs])
    return out.read_bytes()


def test_shard_is_lpt_and_deterministic():
    w = {"a": 10, "b": 9, "c": 5, "d": 5, "e": 1}
    o = shard(list(w), w, 2)
    assert o == shard(list(reversed(list(w))), w, 2)
    loads = [sum(w[r] for r in w if o[r] == i) for i in range(2)]
    assert sorted(loads) == [15, 15]
    assert set(shard(list(w), w, 8).values()) <= set(range(8))


@pytest.mark.parametrize("args", [["x.bam"], ["x.bam", "--long-format", "--show-n-bases"],
                                  ["x.bam", "--summarise", "--decimal-places", "5"]])
def test_cli_world2_matches_single_process(tmp_path, args):
    single = _run(1, args, tmp_path, "single")
    multi = _run(2, args, tmp_path, "multi")
    assert len(single) > 500
    assert multi == single


@pytest.mark.parametrize("args", [["x.bam"], ["x.bam", "--summarise"]])
def test_cli_ranks_with_different_hash_seeds(tmp_path, args):
    """torchrun does not pin PYTHONHASHSEED: each rank iterates set(references) in its own order
    (main.py:92).  Rank 0's order is broadcast (dist.agree_order), so the output is the single
    process's with rank 0's seed."""
    seeds = {0: {"PYTHONHASHSEED": "1"}, 1: {"PYTHONHASHSEED": "2"}}
    single = _run(1, args, tmp_path, "single", extra_env={"PYTHONHASHSEED": "1"})
    other = _run(1, args, tmp_path, "other", extra_env={"PYTHONHASHSEED": "2"})
    assert single != other  # the two seeds do order the references differently
    multi = _run(2, args, tmp_path, "multi", rank_env=seeds)
    assert multi == single


def test_gather_layout_ragged():
    """bc_gather_layout (C-ABI, host arithmetic): rank payloads concatenated in rank order."""
    import numpy as np

    from basecount_amd.device import BcError
    from basecount_amd.dist import gather_layout

    for sizes in ([0], [5], [3, 0, 1003, 7], [0, 0, 0], list(range(8))):
        offs = gather_layout(sizes)
        assert offs == [0] + np.cumsum(sizes).tolist()
        # emulate the root's receive buffer: every payload lands whole at its offset
        payloads = [bytes([r + 1]) * n for r, n in enumerate(sizes)]
        buf = bytearray(offs[-1])
        for r, p in enumerate(payloads):
            buf[offs[r]: offs[r + 1]] = p
        assert [bytes(buf[offs[r]: offs[r + 1]]) for r in range(len(sizes))] == payloads
    with pytest.raises(BcError):
        gather_layout([4, -1])
    with pytest.raises(BcError):
        gather_layout([2 ** 62, 2 ** 62])


def test_cli_world2_summary_with_bed(tmp_path):
    bed = os.path.join(HERE, "golden", "scheme.bed")
    args = ["x.bam", "--summarise-with-bed", bed]
    assert _run(2, args, tmp_path, "multi") == _run(1, args, tmp_path, "single")


def _gather_worker(path):
    # run by subprocess: exercise Group.gather_bytes / all_gather_ints with ragged payloads
    from basecount_amd.dist import Group

    g = Group("gloo")
    got = g.gather_bytes(b"r" * (3 + 1000 * g.rank))
    ints = g.all_gather_ints([g.rank, 7])
    if g.rank == 0:
        with open(path, "w") as fh:
            fh.write(repr(([len(x) for x in got], ints)))
    g.close()


def test_gather_bytes_ragged(tmp_path):
    path = tmp_path / "g.txt"
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), WORLD_SIZE="2")
    code = ("import sys; sys.path.insert(0, %r); sys.path.insert(0, %r); import test_dist as t; "
            "t._gather_worker(%r)" % (os.path.dirname(HERE), HERE, str(path)))
    procs = [subprocess.Popen([sys.executable, "-c", code], env=dict(env, RANK=str(r), LOCAL_RANK=str(r)))
             for r in range(2)]
    assert [p.wait(timeout=240) for p in procs] == [0, 0]
    assert path.read_text() == repr(([3, 1003], [[0, 7], [1, 7]]))


def test_cli_world2_same_error_as_single_process(tmp_path):
    """A zero-length reference makes the summary raise ZeroDivisionError (main.py:479); rank 0
    raises it after the same output as a single process."""
    env = {"FAKE_EMPTY_REF": "1"}
    s_out, s_err = _run(1, ["x.bam", "--summarise"], tmp_path, "single", True, env)
    m_out, m_err = _run(2, ["x.bam", "--summarise"], tmp_path, "multi", True, env)
    strip = lambda line: line.split("]: ", 1)[1] if line.startswith("[rank") else line  # noqa: E731
    assert s_err[0].startswith("ZeroDivisionError") and strip(m_err[0]) == s_err[0]
    assert m_out == s_out


def _comm_worker(path, fail_rank, fail_what):
    # run by subprocess: the communicator vote with stand-ins for the RCCL id, init and destroy
    import time

    from basecount_amd.dist import CommInitAbandoned, CommInitError, env, rendezvous_init

    world, rank, _ = env()
    destroyed = []

    def make_id():
        if fail_what == "id" and rank == fail_rank:
            raise RuntimeError("no id")
        return bytes(range(128))

    def init(uid):
        assert uid == bytes(range(128))
        if fail_what == "init" and rank == fail_rank:
            raise RuntimeError("init refused")
        if fail_what == "hang" and rank == fail_rank:
            time.sleep(600)
        return 1000 + rank

    if fail_what == "late" and rank == fail_rank:  # a straggler: arrives after the init timeout
        time.sleep(5)
    t0 = time.monotonic()
    code = 0
    try:
        res = repr(rendezvous_init(rank, world, make_id, init, timeout=30, init_timeout=3,
                                   destroy=destroyed.append))
    except CommInitError as e:
        res = "CommInitError: " + str(e)
    except CommInitAbandoned as e:  # what bench.py / the CLI do: end the process, non-zero
        res, code = "CommInitAbandoned: " + str(e), 4
    with open(f"{path}.{rank}", "w") as fh:
        fh.write(f"{time.monotonic() - t0:.1f} {destroyed!r} {res}")
    if code:
        os._exit(code)


@pytest.mark.parametrize("fail_rank,fail_what", [(None, None), (1, "init"), (0, "init"), (0, "id"),
                                                 (1, "hang"), (0, "hang"), (2, "late")])
def test_comm_init_is_agreed_by_every_rank(tmp_path, fail_rank, fail_what):
    """the RCCL group comes up on every rank or on none.
    * A failing init on one rank makes every rank raise CommInitError within seconds, after the
      ranks whose init succeeded destroyed their communicator (nothing left behind for the
      bench's gloo fallback);
    * an init still blocked at the timeout makes every rank raise CommInitAbandoned instead, and
      every process exits non-zero within seconds (no fallback next to an abandoned init thread,
      and no destroy either: it could block beside the stuck peers);
    * a rank that reaches the rendezvous later than the init timeout does not fail the others:
      rank 0 hands out the id only once every rank is connected."""
    world = 3
    path = tmp_path / "c"
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), WORLD_SIZE=str(world),
               BASECOUNT_RDZV_PORT=str(_free_port()))
    code = ("import sys; sys.path.insert(0, %r); sys.path.insert(0, %r); import test_dist as t; "
            "t._comm_worker(%r, %r, %r)" % (os.path.dirname(HERE), HERE, str(path), fail_rank, fail_what))
    procs = [subprocess.Popen([sys.executable, "-c", code], env=dict(env, RANK=str(r), LOCAL_RANK=str(r)))
             for r in range(world)]
    codes = [p.wait(timeout=120) for p in procs]
    assert codes == [4 if fail_what == "hang" else 0] * world
    res = [(tmp_path / f"c.{r}").read_text().split(" ", 2) for r in range(world)]
    assert all(float(t) < 20 for t, _, _ in res)
    if fail_rank is None or fail_what == "late":
        assert [r for _, _, r in res] == [repr(1000 + r) for r in range(world)]
        assert all(d == "[]" for _, d, _ in res)
        return
    want = "CommInitAbandoned" if fail_what == "hang" else "CommInitError"
    assert all(r.startswith(want) for _, _, r in res), res
    if fail_what != "id":
        assert all(f"rank {fail_rank}" in r for _, _, r in res), res
    # every communicator that did come up was destroyed before the error -- except on a hang
    # verdict, where the process ends at once (os._exit) and a destroy next to peers stuck in
    # init could block it from getting there
    for r, (_, d, _) in enumerate(res):
        up = fail_what == "init" and r != fail_rank
        assert d == (f"[{1000 + r}]" if up else "[]"), (r, d)


def test_bench_c5_sharding_world4(tmp_path):
    """bench.py's N > 1 C5 leg rehearsed on 4 gloo ranks (the counting by the
    oracle, contigs scaled down 4000x): the LPT plan keeps every rank's positions within one
    chr1 of the mean (at GRCh38 lengths too), and the per-contig summaries gathered to rank 0
    equal one process computing every contig (a contig's reads do not depend on its rank)."""
    import json

    from basecount_amd import synth

    out = tmp_path / "c5.json"
    world = 4
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), WORLD_SIZE=str(world),
               BASECOUNT_DIST_BACKEND="gloo", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="",
               BASECOUNT_RDZV_PORT=str(_free_port()))
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "bench_c5_worker.py"), str(out)],
                              env=dict(env, RANK=str(r), LOCAL_RANK=str(r)), stderr=subprocess.PIPE)
             for r in range(world)]
    errs = [p.communicate(timeout=240)[1] for p in procs]
    assert [p.returncode for p in procs] == [0] * world, [e.decode()[-2000:] for e in errs]
    res = json.loads(out.read_text())
    assert res["got"] == res["want"]
    assert sorted(set(res["owner"].values())) == list(range(world))
    for loads, contigs in ((res["loads"], [(n, L // 4000) for n, L in synth.GRCH38]), (res["full_loads"], synth.GRCH38)):
        longest = max(L for _, L in contigs)
        assert sum(loads) == sum(L for _, L in contigs)
        assert max(loads) - min(loads) <= longest  # LPT: within one chr1
        assert max(loads) <= sum(loads) / world + longest

