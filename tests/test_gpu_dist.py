"""Multi-rank CLI on the GPU: two ranks share the box's one GPU (the exchange over gloo, since
RCCL needs one GPU per rank), each counting its shard of the references with the HIP kernels;
the output must be byte-identical to a single process (and to the reference's goldens)."""
import gzip
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
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


@pytest.mark.gpu
def test_rccl_group_world1(monkeypatch):
    """The product's RCCL group through the C-ABI (bc_comm_*) at world size 1 — the one size a
    one-GPU box can run (RCCL refuses two ranks on one GPU; N > 1 runs in the driver's 8-GPU
    bench): rendezvous, all-gather, broadcast, ragged host gather, device gather, barrier."""
    import ctypes as C

    import numpy as np

    from basecount_amd import device as D
    from basecount_amd.dist import Group, agree_order
    from basecount_amd.main import context

    for v in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(v, raising=False)
    g = Group("rccl")
    try:
        assert (g.world, g.rank) == (1, 0)
        assert g.all_gather_ints([3, -7, 2 ** 40]) == [[3, -7, 2 ** 40]]
        assert g.broadcast_bytes(b"chr1\x00chr2") == b"chr1\x00chr2"
        assert g.broadcast_bytes(b"") == b""
        assert agree_order(g, ["b", "a", "c"]) == ["b", "a", "c"]
        assert g.gather_bytes(b"x" * 1003) == [b"x" * 1003]
        assert g.gather_bytes(b"") == [b""]
        g.barrier()
        ctx = context()
        src = ctx.alloc(64).upload(np.arange(16, dtype=np.float32))
        dst = ctx.alloc(64)
        sizes = np.array([64], np.int64)
        D.check(D.lib().bc_gather_dev(g.h, src.ptr, 64, dst.ptr, sizes.ctypes.data, 0))
        assert np.array_equal(dst.download(np.float32, 16), np.arange(16, dtype=np.float32))
        # a wrong own size is an argument error, not a hang
        bad = np.array([8], np.int64)
        assert D.lib().bc_gather_dev(g.h, src.ptr, 64, dst.ptr, bad.ctypes.data, 0) == D.BC_E_ARG
        # the split-reference histogram sum (RCCL reduce; the identity at world 1), in place
        h = ctx.alloc(4 * 1000).upload(np.arange(1000, dtype=np.int32))
        g.reduce_i32(h, 1000, 0)
        assert np.array_equal(h.download(np.int32, 1000), np.arange(1000, dtype=np.int32))
        assert D.lib().bc_reduce_i32_dev(g.h, h.ptr, h.ptr, 1000, 1) == D.BC_E_ARG  # no rank 1
    finally:
        g.close()


@pytest.mark.gpu
def test_cli_rccl_world1_matches_golden(tmp_path):
    """get_basecounts with the RCCL group (world 1) through the whole sharded CLI path."""
    man = json.load(open(os.path.join(GOLD, "manifest.json")))["edge_summary_dp7"]
    env = dict(os.environ, PYTHONPATH=REPO, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()),
               PYTHONHASHSEED=str(man["hashseed"]))
    code = ("import sys\n"
            "from basecount_amd import main as M, dist\n"
            "args = M.build_parser().parse_args(sys.argv[1:])\n"
            "g = dist.Group('rccl')\n"
            "M._run(args, None, 0, 0, 1000000, None, 7, g)\n"
            "g.close()\n")
    p = subprocess.run([sys.executable, "-c", code, man["bam"], *man["args"]], cwd=GOLD, env=env,
                       capture_output=True, timeout=300)
    assert p.returncode == 0, p.stderr.decode()[-2000:]
    with gzip.open(os.path.join(GOLD, man["stdout"])) as fh:
        assert p.stdout == fh.read()


@pytest.mark.gpu
def test_bench_gpus_2_rehearsal():
    """`bench.py --gpus 2` as the driver runs it (no launcher: the script starts its two ranks),
    both ranks on the box's one GPU with the exchange over gloo (RCCL refuses two ranks on one
    GPU): one JSON line from rank 0 with n_gpus 2 whose headline is C5 (strong scaling, every
    contig's summary gathered from both ranks), C2 weak scaling and C3 split as extras, parity
    true."""
    env = dict(os.environ, BASECOUNT_DIST_BACKEND="gloo")
    for v in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(v, None)
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "5",
                        "--warmup", "2"], env=env, capture_output=True, timeout=600, cwd=REPO)
    assert p.returncode == 0, p.stderr.decode()[-3000:]
    lines = [ln for ln in p.stdout.decode().splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["comm"] == "gloo" and d["parity_vs_oracle"]
    assert d["scaling"] == "strong" and d["gather_bytes"] == 32 * 24 and d["config"]["contigs_per_rank"] >= 1
    assert d["config"]["workload"].startswith("C5") and "c5" not in d["extra"]
    c2 = d["extra"]["c2"]  # every rank its own C2-shaped contig
    assert c2["parity_vs_oracle"] and c2["scaling"] == "weak" and c2["gather_ms"] is not None
    sp = d["extra"]["c3_split"]  # C3's one contig split over the two ranks, histograms reduced
    assert sp["parity_vs_oracle"] and sp["reads_per_rank"] == 500_000 and sp["scaling"] == "strong"


# ------------------------------------------------------------------ sharded decode
CONTIGS6 = [("c0", 30_000), ("c1", 5_000), ("c2", 80_000), ("c3", 12_000), ("c4", 50_000), ("c5", 9_000)]


def _ranks(world, args, tmp_path, name, extra_env=None, cwd=None, timeout=100):
    """Run the CLI on `world` ranks (gloo); (return codes, stdout bytes, stderr texts)."""
    out = tmp_path / f"{name}.out"
    env = dict(os.environ, PYTHONPATH=REPO, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()),
               BASECOUNT_DIST_BACKEND="gloo", PYTHONHASHSEED="0", BASECOUNT_HANG_DUMP=str(timeout - 20),
               **(extra_env or {}))
    from conftest import progress

    progress(f"{world} rank(s): {' '.join(args[1:])} {extra_env or ''}")
    with open(out, "wb") as fh:
        procs = []
        for r in range(world):
            e = dict(env, WORLD_SIZE=str(world), RANK=str(r), LOCAL_RANK=str(r)) if world > 1 else env
            procs.append(subprocess.Popen([sys.executable, "-m", "basecount_amd", *args], stdout=fh,
                                          stderr=subprocess.PIPE, env=e, cwd=cwd))
        # one deadline for all ranks; a rank still running then (a collective that never
        # completes) fails the test with every rank's stderr, which holds its stack
        # (BASECOUNT_HANG_DUMP) instead of hanging the session
        deadline, errs = time.monotonic() + timeout, []
        try:
            for p in procs:
                errs.append(p.communicate(timeout=max(1.0, deadline - time.monotonic()))[1].decode())
        except subprocess.TimeoutExpired:
            for p in procs:
                p.kill()
            errs = [p.communicate()[1].decode(errors="replace") for p in procs]
            raise AssertionError(f"{world} ranks still running after {timeout} s: {args}\n" +
                                 "\n".join(f"--- rank {r}\n{e[-6000:]}" for r, e in enumerate(errs)))
    return [p.returncode for p in procs], out.read_bytes(), errs


def _last_line(err: str) -> str:
    """The exception line (torch.distributed prefixes a rank's traceback lines with [rankN]:)."""
    import re

    lines = [re.sub(r"^\[rank\d+\]:\s*", "", ln) for ln in err.strip().splitlines() if ln.strip()]
    return lines[-1] if lines else ""


@pytest.fixture(scope="module")
def shard_bams(tmp_path_factory):
    from basecount_amd import synth

    d = tmp_path_factory.mktemp("shard")
    rs = synth.make_reads(CONTIGS6, 4_000, True, 21)
    ok = str(d / "grouped.bam")
    synth.write_bam(rs, ok)
    # one read of c3 (its last: the file stays sorted) runs past the reference end
    last_c3 = int(np.flatnonzero(rs.tid == 3)[-1])
    rs.pos[last_c3] = CONTIGS6[3][1] - 10
    bad = str(d / "range_error.bam")
    synth.write_bam(rs, bad)
    return ok, bad


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_sharded_decode_cli_matches_one_process(shard_bams, tmp_path, world):
    """Each rank decodes only its references' byte range (BASECOUNT_SHARD_DECODE=require: a
    range that misses is an error); output and errors byte-identical to one process, also in
    2,500-record batches (the ranges stream) and with a KeyError / IndexError to raise."""
    ok, bad = shard_bams
    cases = [(ok, []), (ok, ["--summarise"]), (ok, ["--min-base-quality", "20", "--show-n-bases", "--long-format"]),
             (ok, ["--references", "c2", "c4"]), (ok, ["--chunk-size", "3000", "--min-mapping-quality", "30"]),
             (bad, []), (bad, ["--summarise"])]
    for i, (bam, args) in enumerate(cases):
        rc1, out1, err1 = _ranks(1, [bam, *args], tmp_path, f"s{i}")
        for batch in (None, "2500"):
            env = {"BASECOUNT_SHARD_DECODE": "require"}
            if batch:
                env["BASECOUNT_BATCH_RECORDS"] = batch
            rcn, outn, errn = _ranks(world, [bam, *args], tmp_path, f"m{i}{batch}", env)
            if rc1[0] == 0:
                assert rcn == [0] * world, (args, [e[-1500:] for e in errn])
                assert outn == out1, args
            else:
                assert all(r != 0 for r in rcn), (args, rcn)
                assert _last_line(errn[0]) == _last_line(err1[0]), (args, errn[0][-800:])
                assert outn == out1 == b""


@pytest.mark.gpu
def test_sharded_decode_halves_the_c5_decode(tmp_path):
    """C5 (24 contigs, 1.2 M reads) --summarise on two ranks, each decoding
    its half of the file: the slower rank's decode phase well under one process's, output
    identical."""
    import re

    from basecount_amd import synth

    bam = str(tmp_path / "c5.bam")
    synth.write_bam(synth.make_config("c5"), bam)
    env = {"BASECOUNT_HIP_TIMING": "1", "BASECOUNT_SHARD_DECODE": "require"}

    def decode_ms(err):
        m = re.findall(r"host decode: ([0-9.]+) ms", err)
        assert m, err[-1500:]
        return float(m[-1])

    best1, best2 = [], []
    for rep in range(2):  # the first run of each pays the page cache / library warm-up
        rc1, out1, err1 = _ranks(1, [bam, "--summarise"], tmp_path, f"one{rep}", env)
        rc2, out2, err2 = _ranks(2, [bam, "--summarise"], tmp_path, f"two{rep}", env)
        assert rc1 == [0] and rc2 == [0, 0], (err1[0][-1500:], [e[-1500:] for e in err2])
        assert out2 == out1
        best1.append(decode_ms(err1[0]))
        best2.append(max(decode_ms(e) for e in err2))
    print(f"C5 decode: one rank {min(best1):.1f} ms, two ranks (slower) {min(best2):.1f} ms")
    assert min(best2) < 0.75 * min(best1), (best1, best2)


@pytest.fixture(scope="module")
def single_contig_bams(tmp_path_factory):
    """One 29,903-bp contig (C2/C3-like), mixed CIGARs: its reads are split over the ranks."""
    from basecount_amd import synth

    d = tmp_path_factory.mktemp("split")
    rs = synth.make_reads([("MN908947.3", 29_903)], 40_000, True, 23)
    ok = str(d / "one.bam")
    synth.write_bam(rs, ok)
    # a read in the middle of the file (a later rank's range) runs past the end: the file stays
    # sorted if it is the last read (so the error comes from the last rank)
    rs.pos[-1] = 29_903 - 20
    bad = str(d / "one_range_error.bam")
    synth.write_bam(rs, bad)
    two = synth.make_reads([("a", 20_000), ("b", 9_000)], 15_000, True, 24)
    pair = str(d / "two.bam")
    synth.write_bam(two, pair)
    return ok, bad, pair


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_split_reference_cli_matches_one_process(single_contig_bams, tmp_path, world):
    """a single contig's reads split over the ranks by position, each rank counting
    its byte range of the file, the histograms summed into the owner (reduce), kernel 2 there.
    Rows, long format, summaries and the range error identical to one process."""
    ok, bad, pair = single_contig_bams
    cases = [(ok, []), (ok, ["--long-format", "--show-n-bases", "--min-base-quality", "20"]),
             (ok, ["--summarise"]), (pair, ["--summarise", "--min-mapping-quality", "30"]), (pair, []),
             (pair, ["--references", "a"]),  # KeyError: 'b' (its reads fall in another rank's range)
             (pair, ["--chunk-size", "2000"]), (bad, [])]
    for i, (bam, args) in enumerate(cases):
        rc1, out1, err1 = _ranks(1, [bam, *args], tmp_path, f"s{i}")
        env = {"BASECOUNT_SHARD_DECODE": "require", "BASECOUNT_HIP_TIMING": "1"}
        rcn, outn, errn = _ranks(world, [bam, *args], tmp_path, f"m{i}", env)
        if rc1[0] == 0:
            assert rcn == [0] * world, (args, [e[-1500:] for e in errn])
            assert outn == out1, args
            assert any("host reduce" in e for e in errn), "no histogram was reduced"
        else:
            assert all(r != 0 for r in rcn), (args, rcn)
            assert _last_line(errn[0]) == _last_line(err1[0]), (args, errn[0][-800:])


@pytest.mark.gpu
@pytest.mark.parametrize("shard_decode", ["0", "1"])
def test_ungrouped_file_restarts_on_every_rank(tmp_path, shard_decode):
    """a file not grouped by reference (A..., B..., A...) makes only the rank owning A
    see A come back; the ranks vote after the batch loop and all restart in accumulate mode
    together (a per-rank restart desynchronised their collectives).  With the sharded decode the
    ranges miss and every rank decodes the whole file.  Output identical to one process."""
    from basecount_amd import synth

    rs = synth.make_reads([("A", 6_000), ("B", 4_000)], 6_000, True, 31)
    # the file order: A's first half, all of B, A's second half (each part coordinate-sorted)
    ia, ib = np.flatnonzero(rs.tid == 0), np.flatnonzero(rs.tid == 1)
    order = np.concatenate([ia[: ia.size // 2], ib, ia[ia.size // 2:]])
    bam = str(tmp_path / "aba.bam")
    synth.write_bam(synth.subset(rs, order), bam)
    for args in ([], ["--summarise"]):
        rc1, out1, err1 = _ranks(1, [bam, *args], tmp_path, "one")
        env = {"BASECOUNT_SHARD_DECODE": shard_decode, "BASECOUNT_BATCH_RECORDS": "1500"}
        rc2, out2, err2 = _ranks(2, [bam, *args], tmp_path, "two", env)
        assert rc1 == [0] and rc2 == [0, 0], (err1[0][-1500:], [e[-1500:] for e in err2])
        assert out2 == out1 and len(out1) > 100


@pytest.mark.gpu
def test_damaged_block_near_a_cut_fails_every_rank_alike(shard_bams, tmp_path):
    """with the sharded decode, a damaged BGZF block near a rank's cut used to fail the
    probe (or the range open) on that rank only while the others waited in the shard merge.  Now
    it is a miss on that rank, every rank decodes the whole file and raises the one process's
    error."""
    ok, _ = shard_bams
    data = bytearray(open(ok, "rb").read())
    for frac in (0.35, 0.5, 0.65):
        at = int(len(data) * frac)
        bad = bytearray(data)
        bad[at: at + 96] = bytes(range(96))
        path = str(tmp_path / f"damaged{frac}.bam")
        open(path, "wb").write(bad)
        rc1, out1, err1 = _ranks(1, [path], tmp_path, f"one{frac}")
        rc2, out2, err2 = _ranks(2, [path], tmp_path, f"two{frac}")
        assert rc1[0] != 0, "the damaged file decoded"
        assert all(r != 0 for r in rc2), rc2
        assert _last_line(err2[0]) == _last_line(err1[0]), (err2[0][-800:], err1[0][-800:])
