"""Benchmark: reference positions/sec of the pileup hot path on MI355X.

A step = one pass of the hot path over one batch already resident in HBM: ONE launch of the
fused k_pileup kernel = kernel 1 (CIGAR-expand + base counting, count.cpp:22-97) and kernel 2
(per-position coverage / percentages / entropies, main.py:29-78).  Workload at N=1: BASELINE config 2 (1 contig 29,903 bp, 100,000 reads x 150 bp,
all-M CIGAR).  At N>1 every rank runs its own contig of that shape (contig sharding, weak
scaling, no collective inside the step); the per-contig results are gathered to rank 0 over
RCCL once after the timed region (reported as gather_ms).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c5] [--launch graph|eager]

The K timed steps are captured into one hipGraph and launched once (default; --launch eager
issues them one by one): the same kernels on the same data, without the per-launch host and
command-processor gaps that a ~15 us step otherwise pays.

C5 (24 human-chromosome-sized contigs, 3.09 Gb, 1.2 M reads) is summary-shaped: the per-position
percentages are not stored (main.py's --summarise never prints them).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (REPO, os.path.join(REPO, "oracle")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)

WORKLOADS = {
    "c2": "C2: 1 contig 29,903 bp, 100,000 reads x 150 bp, all-M CIGAR (per rank)",
    "c3": "C3: 1 contig 29,903 bp, 1,000,000 reads x 150 bp, mixed M/I/D/=/X/S CIGAR (per rank)",
    "c5": "C5: 24 contigs with GRCh38 chr1-22,X,Y lengths (3.09 Gb), 50,000 reads x 150 bp each, "
          "all-M CIGAR; contigs sharded over the ranks",
}


def read_bytes(b: dict, mbq: int, l_seq: np.ndarray) -> int:
    """Algorithmic bytes of the read batch (roofline): per read 16 B of read index
    (pos, cig_beg, cig_n, seq_nib) + 4 B per CIGAR word + ceil(l_seq/2) B of packed SEQ (+ l_seq
    B of QUAL when mbq > 0)."""
    n = int(b["pos"].size)
    nb = 16 * n + 4 * int(b["cig_n"].sum()) + int(((l_seq + 1) // 2).sum())
    return nb + (int(l_seq.sum()) if mbq > 0 else 0)


def kernel_bytes(kernel: str, rb: int, L: int, k: int, with_pc: bool = True) -> int:
    """Algorithmic HBM bytes of one launch: the fused k_pileup reads the batch and writes per
    position k int32 counts, int32 coverage, k f64 percentages (when requested) and two f64
    entropies; k_rc reads the batch and writes the counts; k_stats reads the counts and writes
    the statistics."""
    stats_out = L * (4 + (8 * k if with_pc else 0) + 16)
    return {"pileup": rb + 4 * k * L + stats_out, "rc": rb + 4 * k * L, "stats": 4 * k * L + stats_out}[kernel]


def cpu_baseline(rs, b, L: int, budget_s: float = 10.0) -> dict:
    """The reference's CPU path on the same workload: its own compiled count.bcount (oracle/_ref,
    pybind11, Python-list arguments as main.py:146 passes them) + get_stats (main.py:14-79,
    restated in oracle.get_stats_py).  Single thread, like the reference."""
    import oracle as O

    ref = O.ref_bcount()
    n = int(b["pos"].size)
    if ref is not None:
        # pysam-shaped arguments (built once, untimed): clipped strings, qualities, starts, tuples
        seqs = rs.seq.reshape(n, -1)
        nt = np.frombuffer(b"=ACMGRSVTWYHKDBN", np.uint8)
        codes = np.empty((n, seqs.shape[1] * 2), np.uint8)
        codes[:, 0::2], codes[:, 1::2] = seqs >> 4, seqs & 15
        reads = [bytes(nt[row]).decode() for row in codes]
        quals = [q for q in rs.qual.reshape(n, -1).tolist()]
        starts = b["pos"].tolist()
        ctuples = [[(0, 150)]] * n
        done, t0 = 0, time.perf_counter()
        while True:
            counts = ref(L, 0, reads, quals, starts, ctuples)
            O.get_stats_py(counts, "ref")
            done += 1
            if time.perf_counter() - t0 > budget_s:
                break
        dt = (time.perf_counter() - t0) / done
        kind, what = "reference", ("reference count.cpp (pybind11 bcount, list arguments) + "
                                   "get_stats main.py:14-79 (Python)")
    else:
        done, t0 = 0, time.perf_counter()
        while True:
            counts, _ = O.bcount(L, 0, b)
            O.stats(counts, False)
            done += 1
            if time.perf_counter() - t0 > budget_s:
                break
        dt = (time.perf_counter() - t0) / done
        kind, what = "port", "oracle C restatement of bcount + get_stats"
    return {"value": L / dt, "unit": "positions/s", "cores": 1, "kind": kind,
            "sample": f"{what}; full C2 workload ({n} reads, {L} positions) x {done} runs, "
                      f"{dt * 1e3:.1f} ms per run, BAM decode excluded"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="c2", choices=sorted(WORKLOADS))
    ap.add_argument("--mbq", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    ap.add_argument("--launch", choices=["graph", "eager"], default="graph",
                    help="graph: the K timed steps are captured into ONE hipGraph and launched once")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = torch = None
    if world > 1:
        # torch's bundled HIP runtime must initialise before libbasecount_hip's (/opt/rocm) one:
        # the other order leaves torch without devices ("two HIP runtimes")
        import torch
        import torch.distributed as dist

        # one process per GPU; BASECOUNT_DIST_BACKEND=gloo lets ranks share a GPU (rehearsals)
        backend = os.environ.get("BASECOUNT_DIST_BACKEND", "nccl")
        dev = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(dev)
        sys.stdout.flush()
        saved = os.dup(1)  # the backends log connection messages on fd 1: rank 0 prints ONE line
        try:
            os.dup2(2, 1)
            if backend == "nccl":
                dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
            else:
                dist.init_process_group(backend)
        finally:
            os.dup2(saved, 1)
            os.close(saved)

    from basecount_amd import device as D
    from basecount_amd import synth
    from basecount_amd.main import norm_factors

    # ---- workload: this rank's contigs -----------------------------------------------------
    # c2 / c3: one contig of the config's shape per rank (weak scaling); c5: the 24 GRCh38-sized
    # contigs, sharded over the ranks by LPT (strong scaling: the total work is fixed)
    c = synth.CONFIGS[args.config]
    per_contig = c.get("per_contig", False)
    if per_contig:
        from basecount_amd.dist import shard

        contigs = list(c["contigs"])
        owner = shard([n for n, _ in contigs], dict(contigs), world)
        mine = [(n, L) for n, L in contigs if owner[n] == rank]
        rs = synth.make_reads(mine, c["reads"], c["mixed"], c["seed"] + 1000 * rank)
        total_positions = sum(L for _, L in contigs)
    else:
        name = "MN908947.3" if world == 1 else f"contig{rank}"
        rs = synth.make_reads([(name, c["contigs"][0][1])], c["reads"], c["mixed"],
                              c["seed"] + 1000 * rank)
        total_positions = world * rs.lengths[0]
    ncols = k = 5
    want_pc = not per_contig  # c5 is only ever summarised: no per-position percentages
    ctx = D.Context(local % max(1, D.device_count()) if world > 1 else 0)  # own stream
    nf, nf2 = norm_factors(k)
    work = []  # one entry per contig, resident in HBM before anything is timed
    for t, L in enumerate(rs.lengths):
        b = synth.batch_arrays(rs, t, 0)
        reads = D.DeviceReads(ctx, b)
        assert reads.r.sorted == 1
        bufs = dict(counts=ctx.alloc(4 * ncols * L), cov=ctx.alloc(4 * L),
                    pc=ctx.alloc(8 * k * L) if want_pc else None, ent=ctx.alloc(8 * L), sec=ctx.alloc(8 * L))
        work.append((t, L, b, reads, bufs))

    def ptr(x):
        return x.ptr if x is not None else None

    def step():
        # one pass of the hot path over every contig of this rank: kernel 1 + kernel 2
        for _, L, _, reads, o in work:
            ctx.pileup(reads, L, args.mbq, k, nf, nf2, o["counts"].ptr, o["cov"].ptr, ptr(o["pc"]),
                       o["ent"].ptr, o["sec"].ptr)

    for _ in range(args.warmup):
        step()
    ctx.sync()
    assert ctx.range_error() == -1

    def barrier():
        if dist:
            dist.barrier()

    # ---- timed region: K eager back-to-back steps, bracketed by barrier + device sync; hipEvents
    # on the library's stream (the stream every launch goes to) around the region give the
    # on-device time per step ---------------------------------------------------------------
    graph = None
    if args.launch == "graph":  # the same K steps, replayed from one captured graph
        graph = ctx.capture(lambda: [step() for _ in range(args.steps)])
        graph.launch()  # untimed replay (first-launch setup)
        ctx.sync()
    barrier()
    ctx.sync()
    t0 = time.perf_counter()
    ctx.event_record(0)
    if graph is not None:
        graph.launch()
    else:
        for _ in range(args.steps):
            step()
    ctx.event_record(1)
    ctx.sync()
    barrier()
    elapsed = time.perf_counter() - t0
    dev_step = ctx.event_elapsed_ms(0, 1) * 1e-3 / args.steps  # s per step on the device
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # ---- which kernels a step launches (library timing facility, per-launch event pairs) -------
    ctx.timing(True)
    step()
    launched = sorted(ctx.timing_report())
    ctx.timing(False)

    def region(fn, reps):  # on-device seconds per call: hipEvents around `reps` back-to-back calls
        ctx.sync()
        ctx.event_record(2)
        for _ in range(reps):
            fn()
        ctx.event_record(3)
        return ctx.event_elapsed_ms(2, 3) * 1e-3 / reps

    # per-kernel time per step, each timed as a region of back-to-back launches of that kernel
    # alone (a one-kernel step: the step region itself)
    kern_s = {}
    if launched == ["pileup"]:
        # eager launches: the kernel's own average duration (what rocprofv3's kernel trace
        # reports); a graph replay hides part of the launch gap and would flatter the roofline
        kern_s["pileup"] = dev_step if graph is None else region(step, max(3, min(args.steps, 100)))
    else:  # deep batches: k_rc + k_stats (bc_count on the same batch launches k_rc alone)
        reps = max(3, min(args.steps, 50))

        def count_only():
            for _, L, _, reads, o in work:
                ctx.count(reads, L, args.mbq, k, o["counts"].ptr)

        def stats_only():
            for _, L, _, _, o in work:
                ctx.stats(o["counts"].ptr, L, k, nf, nf2, o["cov"].ptr, ptr(o["pc"]), o["ent"].ptr,
                          o["sec"].ptr)

        kern_s["rc"] = region(count_only, reps)
        kern_s["stats"] = region(stats_only, reps)
        step()  # restore the step's outputs (the count-only regions accumulated into the counts)
        ctx.sync()
    dom = max(kern_s, key=kern_s.get)

    # ---- correctness of what was timed (rank-local) -----------------------------------------
    import oracle as O

    parity = True
    small = min(work, key=lambda w: w[1])  # full oracle check on the smallest contig
    for t, L, b, reads, o in work:
        if (t, L) == small[:2]:
            got = o["counts"].download(np.int32, ncols * L).reshape(ncols, L)
            exp, _ = O.bcount(L, args.mbq, b)
            parity = parity and bool(np.array_equal(got, exp[:, :ncols].T.astype(np.int32)))
            _, _, oent, _ = O.stats(exp, False)
            parity = parity and float(np.max(np.abs(o["ent"].download(np.float64, L) - oent))) <= 1e-6
            del got, exp, oent
        if args.mbq == 0 and not c["mixed"]:
            # size-independent check on every contig: all-M reads without N bases put every
            # reference-consuming event into the coverage (a checksum of checksums)
            cov_sum = int(o["cov"].download(np.int32, L).astype(np.int64).sum())
            parity = parity and cov_sum == synth.ref_events(rs, t)

    # ---- gather per-contig coverage to rank 0 over RCCL (output step, outside the timing) ----
    gather_ms = None
    if dist and not per_contig:
        L0, o0 = work[0][1], work[0][4]
        covt = torch.from_numpy(o0["cov"].download(np.int32, L0))
        if backend == "nccl":
            covt = covt.cuda()
            torch.cuda.synchronize()
        g0 = time.perf_counter()
        bufs = [torch.zeros_like(covt) for _ in range(world)]
        dist.all_gather(bufs, covt)  # per-contig coverage of every rank (RCCL over xGMI)
        if backend == "nccl":
            torch.cuda.synchronize()
        gather_ms = (time.perf_counter() - g0) * 1e3

    events = synth.ref_events(rs)
    ms = elapsed / args.steps * 1e3
    positions = total_positions * args.steps
    kbytes = sum(kernel_bytes(dom, read_bytes(b, args.mbq, rs.l_seq[rs.tid == t]), L, k, want_pc)
                 for t, L, b, _, _ in work)
    achieved = kbytes / kern_s[dom] / 1e9
    kernel_names = {"pileup": "k_pileup (fused kernel 1 + 2)", "rc": "k_rc (read-chunked kernel 1)",
                    "stats": "k_stats (kernel 2)"}
    traffic = None
    pmc = os.path.join(REPO, "profiles", "kernel1_pmc.json")
    if os.path.exists(pmc):
        with open(pmc) as fh:
            pm = json.load(fh).get(args.config, {})
        if pm and pm.get("mbq", 0) == args.mbq and pm.get("kernel", "pileup") == dom and world == 1:
            traffic = pm.get("hbm_bytes_per_launch")
    n_reads = sum(int(w[2]["pos"].size) for w in work)

    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline and not per_contig:
            b0, L0 = work[0][2], work[0][1]
            cpu = cpu_baseline(rs, b0, L0, args.cpu_budget)
        value = positions / elapsed
        line = {
            "metric": "reference positions/sec (kernel 1 + kernel 2, inputs resident in HBM)",
            "value": value,
            "unit": "positions/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms,
            "higher_is_better": True,
            "scaling": "strong" if per_contig else "weak",
            "vs_baseline": None,
            "dtype": "int32 counts / f64 stats",
            "data": "synthetic (seeded, BASELINE config shape)",
            "config": {"workload": WORKLOADS[args.config], "reads_per_rank": n_reads,
                       "positions_per_rank": int(sum(w[1] for w in work)), "contigs_per_rank": len(work),
                       "min_base_quality": args.mbq, "percentages_stored": want_pc,
                       "parallelism": f"contig-sharded x{world}"},
            "gbases_piled_per_s": (world if not per_contig else 1) * events * args.steps / elapsed / 1e9,
            "device_us_per_step": dev_step * 1e6,
            "kernel_us": {kernel_names[n]: v * 1e6 for n, v in kern_s.items()},
            "kernels": ("k_pileup (kernel 1 and kernel 2 fused), one launch per contig per step"
                        if dom == "pileup" else "k_rc (kernel 1, into a zeroed scratch) + k_stats (kernel 2, moves the counts out and re-zeroes) per contig per step")
                       + (", the K timed steps replayed from one hipGraph" if graph is not None else ", eager launches"),
            "parity_vs_oracle": parity,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": kernel_names[dom], "algorithmic_bytes": kbytes},
            "cpu_baseline": cpu,
            "gather_ms": gather_ms,
        }
        if cpu:
            line["speedup_vs_cpu"] = value / cpu["value"]
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()
    if not parity:
        sys.exit(3)


if __name__ == "__main__":
    main()
