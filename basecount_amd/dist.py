"""Multi-GPU (one process per GPU) plumbing for the CLI and the bench: contig sharding, the
reference order every rank follows, and the gather to rank 0.

The counting path needs no communication: references are independent, so each
rank owns whole references (LPT on an estimate of their cost) and runs the single-GPU path on
them.  The only exchanges are
  * the reference order: main.py:92 iterates ``set(references)``, whose order depends on each
    process's hash seed, so rank 0's order is broadcast and every rank follows it (sharding,
    error exchange, output order);
  * the per-reference first out-of-range read (all ranks raise the same first error, in the
    reference's order: main.py's error timeline);
  * the output: summary numbers are gathered to rank 0; per-position rows are written by their
    owner in reference order (barrier per reference), so hundreds of GB of TSV never travel.

Two interchangeable groups implement these exchanges:
  * ``RcclGroup`` (the product's, default): RCCL over xGMI through the C-ABI of
    libbasecount_hip.so (bc_comm_*, bc_allgather_i64, bc_broadcast_bytes, bc_gather_bytes), on
    the rank's own GPU and stream.  No PyTorch anywhere: one HIP runtime per process.  The RCCL
    unique id is handed from rank 0 to the others over a TCP socket at MASTER_ADDR, port
    ``BASECOUNT_RDZV_PORT`` (default MASTER_PORT + 1: torchrun's own store holds MASTER_PORT).
  * ``GlooGroup``: torch.distributed's gloo backend on the CPU (``BASECOUNT_DIST_BACKEND=gloo``),
    for multi-process tests without one GPU per rank (RCCL refuses two ranks on one GPU).

Launch: ``python -m torch.distributed.run --nproc-per-node N -m basecount_amd BAM ...`` (each
rank reads RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT).
"""
from __future__ import annotations

import contextlib
import ctypes as C
import json
import os
import socket
import struct
import sys
import time


def env() -> tuple[int, int, int]:
    """(world_size, rank, local_rank) from the torchrun environment."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def Group(backend: str | None = None, ctx=None):
    """The process group of this job: RCCL (default) or gloo (BASECOUNT_DIST_BACKEND)."""
    backend = backend or os.environ.get("BASECOUNT_DIST_BACKEND") or "rccl"
    if backend in ("rccl", "nccl"):
        return RcclGroup(ctx)
    if backend == "gloo":
        return GlooGroup()
    raise ValueError(f"unknown BASECOUNT_DIST_BACKEND {backend!r} (rccl or gloo)")


class _GroupOps:
    """Operations built on the three primitives every group provides: all_gather_ints,
    broadcast_bytes and gather_bytes."""

    def broadcast_obj(self, obj):
        """Rank 0's JSON-serialisable object on every rank."""
        data = json.dumps(obj).encode() if self.rank == 0 else b""
        return json.loads(self.broadcast_bytes(data).decode())


def agree_order(group, order: list) -> list:
    """The reference order of rank 0 on every rank (main.py:92's set order is per process)."""
    mine = list(order)
    theirs = group.broadcast_obj(mine)
    if sorted(theirs) != sorted(mine):
        raise RuntimeError("ranks disagree on the set of references")
    return theirs


class _stdout_to_stderr:
    """fd-level redirect of stdout to stderr (native libraries write to fd 1 directly)."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        os.dup2(self.saved, 1)
        os.close(self.saved)


def _rdzv_port() -> int:
    v = os.environ.get("BASECOUNT_RDZV_PORT")
    if v:
        return int(v)
    return int(os.environ.get("MASTER_PORT", "29500")) + 1


def _recv_exact(s: socket.socket, n: int) -> bytes:
    buf = b""
    while len(buf) < n:
        part = s.recv(n - len(buf))
        if not part:
            raise ConnectionError("rendezvous peer closed the connection")
        buf += part
    return buf


def _rdzv_timeout() -> float:
    v = os.environ.get("BASECOUNT_RDZV_TIMEOUT")
    return float(v) if v else 120.0


class CommInitError(RuntimeError):
    """The job's communicator could not be created on every rank.  Raised on EVERY rank (the ranks
    vote, see rendezvous_init) after every init call has returned and the communicators that did
    come up were destroyed, so a caller that falls back (bench.py: gloo) does so on all ranks alike,
    with no library state left behind, and no rank is left waiting in a collective the others never
    join."""


class CommInitAbandoned(RuntimeError):
    """Some rank's init call was still blocked in the library (ncclCommInitRank) when the ranks
    voted.  Its thread is abandoned there and may hold runtime locks, so no rank may carry on in
    this process, on any backend: raised on EVERY rank instead of CommInitError, and the caller
    must end the process (bench.py: os._exit, non-zero)."""


def _init_timeout() -> float:
    v = os.environ.get("BASECOUNT_COMM_INIT_TIMEOUT")
    return float(v) if v else 120.0


def _run_with_timeout(fn, arg, timeout: float):
    """fn(arg) in a daemon thread: ("ok", result), ("fail", reason) or ("hang", reason).  A call
    still blocked at the timeout (a collective init whose peers never arrive) is abandoned with its
    thread: the process must not go on (CommInitAbandoned)."""
    import threading

    box = {}

    def target():
        try:
            box["v"] = ("ok", fn(arg))
        except Exception as e:  # noqa: BLE001 - reported to the other ranks, re-raised by the caller
            box["v"] = ("fail", f"{type(e).__name__}: {e}")

    t = threading.Thread(target=target, daemon=True)
    t.start()
    t.join(timeout)
    return box.get("v", ("hang", f"no result within {timeout:.0f} s (BASECOUNT_COMM_INIT_TIMEOUT)"))


_STATES = ("ok", "fail", "hang")


def _send_msg(conn, state: str, text: str) -> None:
    b = text.encode()
    conn.sendall(struct.pack("<II", _STATES.index(state), len(b)) + b)


def _recv_msg(conn) -> tuple:
    code, n = struct.unpack("<II", _recv_exact(conn, 8))
    return _STATES[code] if code < len(_STATES) else "fail", _recv_exact(conn, n).decode(errors="replace")


def rendezvous_init(rank: int, world: int, make_id, init, timeout: float | None = None,
                    init_timeout: float | None = None, destroy=None):
    """A communicator created by agreement of all ranks, over one TCP connection per peer to rank
    0 (port ``BASECOUNT_RDZV_PORT``, default MASTER_PORT + 1):

      1. rank 0 binds the port (failing at once, with the port in the message, if it is taken),
         calls make_id(), waits until every peer has connected and only then sends the id's
         bytes to all of them (an empty id if make_id failed: every rank then raises at once), so
         no rank starts its init clock before the last one has arrived;
      2. every rank calls init(id) (the collective bc_comm_init) in a thread bounded by
         ``init_timeout`` (``BASECOUNT_COMM_INIT_TIMEOUT``, default 120 s);
      3. every rank reports ok / failed / still blocked to rank 0, which answers all of them
         with the verdict.  Unless every rank succeeded, the ranks whose init succeeded call
         destroy(result), and then every rank raises: CommInitAbandoned if some init was still
         blocked (no rank may go on in the process), CommInitError otherwise (a fallback is safe).

    The peers retry the connection for ``timeout`` seconds (``BASECOUNT_RDZV_TIMEOUT``, default
    120).  Returns init's result."""
    addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
    port = _rdzv_port()
    timeout = _rdzv_timeout() if timeout is None else float(timeout)
    init_timeout = _init_timeout() if init_timeout is None else float(init_timeout)
    deadline = time.monotonic() + timeout

    def verdict_of(statuses: list) -> tuple:
        bad = [f"rank {r}: {w}" for r, (st, w) in enumerate(statuses) if st != "ok"]
        state = ("hang" if any(st == "hang" for st, _ in statuses) else
                 "fail" if bad else "ok")
        return state, "; ".join(bad)

    def conclude(state: str, why: str, mine: tuple):
        if state == "ok":
            return mine[1]
        # no communicator is left behind -- except on a 'hang' verdict: the process ends right
        # after (os._exit), and destroying a communicator whose peers are stuck in init could
        # block and keep it from ever getting there
        if mine[0] == "ok" and destroy is not None and state != "hang":
            with contextlib.suppress(Exception):
                destroy(mine[1])
        if state == "hang":
            raise CommInitAbandoned(f"communicator init still blocked on some rank ({why}): ending the process")
        raise CommInitError(f"communicator not created on every rank: {why}")

    if rank == 0:
        srv = None
        if world > 1:
            srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            try:
                srv.bind((addr, port))
            except OSError as e:
                srv.close()
                raise RuntimeError(f"rank 0 cannot bind the rendezvous port {addr}:{port} ({e}); set "
                                   "BASECOUNT_RDZV_PORT to a free port") from e
            srv.listen(max(1, world))
            srv.settimeout(timeout)
        conns = []
        try:
            try:
                uid, id_err = make_id(), None
            except Exception as e:  # noqa: BLE001 - every peer is told, then it is re-raised
                uid, id_err = b"", e
            while srv is not None and len(conns) < world - 1:
                try:
                    conn, _ = srv.accept()
                except socket.timeout as e:
                    raise CommInitError(f"rank 0: only {len(conns)} of {world - 1} peers reached the "
                                        f"rendezvous at {addr}:{port} within {timeout:.0f} s") from e
                conn.settimeout(init_timeout + timeout)
                peer = struct.unpack("<I", _recv_exact(conn, 4))[0]
                conns.append((peer, conn))
            try:  # every peer is here: the id goes out to all of them together
                for _, conn in conns:
                    conn.sendall(struct.pack("<I", len(uid)) + uid)
            except OSError as e:
                # the peers that already have the id fail at once when their report or the verdict
                # finds the connection closed (finally, below), instead of waiting out init_timeout
                raise CommInitError(f"rank 0: sending the communicator id failed ({e})") from e
            if id_err is not None:
                raise CommInitError(f"rank 0 could not create the communicator id: {id_err}") from id_err
            mine = _run_with_timeout(init, uid, init_timeout)
            statuses = [(mine[0], mine[1] if mine[0] != "ok" else "")] + [("fail", "no report")] * (world - 1)
            for peer, conn in conns:
                try:
                    st, msg = _recv_msg(conn)
                    if 0 < peer < world:
                        statuses[peer] = (st, msg)
                except (OSError, ConnectionError) as e:
                    if 0 < peer < world:
                        statuses[peer] = ("fail", f"lost ({e})")
            state, why = verdict_of(statuses)
            for _, conn in conns:
                with contextlib.suppress(OSError):
                    _send_msg(conn, state, why)
        finally:
            for _, conn in conns:
                conn.close()
            if srv is not None:
                srv.close()
        return conclude(state, why, mine)
    while True:
        try:
            s = socket.create_connection((addr, port), timeout=10)
            break
        except (ConnectionRefusedError, socket.timeout, OSError) as e:
            if time.monotonic() > deadline:
                raise CommInitError(f"rank {rank}: no rendezvous from rank 0 at {addr}:{port} within "
                                    f"{timeout:.0f} s (BASECOUNT_RDZV_TIMEOUT)") from e
            time.sleep(0.05)
    with s:
        s.settimeout(init_timeout + timeout)
        try:
            s.sendall(struct.pack("<I", rank))
            (n,) = struct.unpack("<I", _recv_exact(s, 4))
            uid = _recv_exact(s, n)
        except (OSError, ConnectionError) as e:
            raise CommInitError(f"rank {rank}: the rendezvous with rank 0 failed ({e})") from e
        if not uid:
            raise CommInitError(f"rank {rank}: rank 0 could not create the communicator id")
        mine = _run_with_timeout(init, uid, init_timeout)
        try:
            _send_msg(s, mine[0], "" if mine[0] == "ok" else (mine[1] or "failed"))
            state, why = _recv_msg(s)
        except (OSError, ConnectionError) as e:
            # no verdict: rank 0 is gone.  An init still blocked here forbids going on.
            state, why = ("hang" if mine[0] == "hang" else "fail"), f"rank {rank}: no verdict from rank 0 ({e})"
    return conclude(state, why, mine)


class RcclGroup(_GroupOps):
    """RCCL over xGMI through libbasecount_hip.so's bc_comm (one GPU per rank)."""

    backend = "rccl"

    def __init__(self, ctx=None):
        from . import device as D

        self.D = D
        world, rank, _ = env()
        if ctx is None:
            from .main import context

            ctx = context()
        self.ctx = ctx
        L = D.lib()

        def make_id():
            buf = (C.c_uint8 * D.COMM_ID_BYTES)()
            D.check(L.bc_comm_unique_id(buf))
            return bytes(buf)

        def init(uid):
            h = C.c_void_p()
            ubuf = (C.c_uint8 * len(uid)).from_buffer_copy(uid)
            D.check(L.bc_comm_init(ctx.h, ubuf, rank, world, C.byref(h)))
            return h.value

        self.world, self.rank = world, rank
        # RCCL prints a version banner on fd 1 when a communicator comes up: keep stdout for the
        # TSV output (the first collective runs inside the redirect too).  The ranks agree on the
        # outcome (rendezvous_init): either every rank has the communicator or every rank raises.
        with _stdout_to_stderr():
            self.h = rendezvous_init(rank, world, make_id, init,
                                     destroy=lambda h: L.bc_comm_destroy(C.c_void_p(h)))
            self.barrier()

    def barrier(self):
        self.D.check(self.D.lib().bc_comm_barrier(self.h))

    def all_gather_ints(self, vals: list[int]) -> list[list[int]]:
        import numpy as np

        a = np.ascontiguousarray(vals, np.int64)
        out = np.zeros(self.world * a.size, np.int64)
        self.D.check(self.D.lib().bc_allgather_i64(self.h, a.ctypes.data, a.size, out.ctypes.data))
        return out.reshape(self.world, a.size).tolist()

    def reduce_i32(self, buf, n: int, root: int) -> None:
        """Sum every rank's int32 device buffer [n] into root's, in place (RCCL reduce on the
        rank's stream, after the kernels that filled it)."""
        self.D.check(self.D.lib().bc_reduce_i32_dev(self.h, buf.ptr, buf.ptr, int(n), int(root)))

    def broadcast_bytes(self, data: bytes) -> bytes:
        n = self.all_gather_ints([len(data)])[0][0]
        buf = (C.c_uint8 * max(1, n))()
        if self.rank == 0 and n:
            C.memmove(buf, data, n)
        self.D.check(self.D.lib().bc_broadcast_bytes(self.h, buf, n, 0))
        return bytes(buf)[:n]

    def gather_bytes(self, data: bytes) -> list[bytes] | None:
        """Rank 0 receives every rank's bytes (ragged sizes, bc_gather_layout offsets)."""
        import numpy as np

        sizes = np.ascontiguousarray([s[0] for s in self.all_gather_ints([len(data)])], np.int64)
        offs = gather_layout(sizes)
        src = (C.c_uint8 * max(1, len(data)))()
        if data:
            C.memmove(src, data, len(data))
        dst = (C.c_uint8 * max(1, int(offs[-1])))() if self.rank == 0 else None
        self.D.check(self.D.lib().bc_gather_bytes(self.h, src, len(data), dst, sizes.ctypes.data, 0))
        if self.rank != 0:
            return None
        raw = bytes(dst)
        return [raw[offs[r]: offs[r + 1]] for r in range(self.world)]

    def close(self):
        if getattr(self, "h", None):
            self.D.lib().bc_comm_destroy(self.h)
            self.h = None


def gather_layout(sizes) -> list[int]:
    """bc_gather_layout: offsets [world + 1] of a ragged gather (host arithmetic, no GPU)."""
    import numpy as np

    from . import device as D

    s = np.ascontiguousarray(sizes, np.int64)
    out = np.zeros(s.size + 1, np.int64)
    D.check(D.lib().bc_gather_layout(s.ctypes.data, int(s.size), out.ctypes.data))
    return out.tolist()


class GlooGroup(_GroupOps):
    """torch.distributed gloo on the CPU: multi-process tests without one GPU per rank."""

    backend = "gloo"

    def __init__(self):
        import torch
        import torch.distributed as td

        self.td, self.torch = td, torch
        if not td.is_initialized():
            # the backend logs connection messages on fd 1: keep stdout for the TSV output
            with _stdout_to_stderr():
                td.init_process_group("gloo")
        self.world, self.rank = td.get_world_size(), td.get_rank()

    def barrier(self):
        self.td.barrier()

    def all_gather_ints(self, vals: list[int]) -> list[list[int]]:
        t = self.torch.tensor(vals, dtype=self.torch.int64)
        out = [self.torch.empty_like(t) for _ in range(self.world)]
        self.td.all_gather(out, t)
        return [o.tolist() for o in out]

    def reduce_i32(self, buf, n: int, root: int) -> None:
        """reduce_i32 through the host (gloo tests: several ranks share one GPU)."""
        import numpy as np

        t = self.torch.from_numpy(np.ascontiguousarray(buf.download(np.int32, int(n))))
        self.td.reduce(t, dst=int(root), op=self.td.ReduceOp.SUM)
        if self.rank == root:
            buf.upload(t.numpy())

    def broadcast_bytes(self, data: bytes) -> bytes:
        n = self.all_gather_ints([len(data)])[0][0]
        buf = self.torch.zeros(max(1, n), dtype=self.torch.uint8)
        if self.rank == 0 and n:
            buf[:n] = self.torch.frombuffer(bytearray(data), dtype=self.torch.uint8)
        self.td.broadcast(buf, 0)
        return bytes(buf.numpy()[:n])

    def gather_bytes(self, data: bytes) -> list[bytes] | None:
        sizes = [s[0] for s in self.all_gather_ints([len(data)])]
        offs = gather_layout(sizes)
        n = max(sizes) if sizes else 0
        buf = self.torch.zeros(max(1, n), dtype=self.torch.uint8)
        if data:
            buf[: len(data)] = self.torch.frombuffer(bytearray(data), dtype=self.torch.uint8)
        outs = [self.torch.empty_like(buf) for _ in range(self.world)]
        self.td.all_gather(outs, buf)
        if self.rank != 0:
            return None
        assert offs[-1] == sum(sizes)
        return [bytes(o.numpy()[: sizes[i]]) for i, o in enumerate(outs)]

    def close(self):
        if self.td.is_initialized():
            self.td.destroy_process_group()


def shard(refs: list[str], weights: dict, world: int) -> dict:
    """ref -> owning rank: longest-processing-time-first on `weights` (deterministic ties)."""
    load = [0.0] * world
    owner = {}
    for ref in sorted(refs, key=lambda r: (-float(weights[r]), r)):
        r = min(range(world), key=lambda i: (load[i], i))
        owner[ref] = r
        load[r] += float(weights[ref])
    return owner


def shard_contiguous(weights: list, world: int) -> list[int]:
    """Cuts b[0] = 0 <= b[1] <= ... <= b[world] = n of items 0..n-1 (references in file order)
    into `world` contiguous runs, rank r owning [b[r], b[r + 1]): the smallest largest-run weight
    (binary search on it, runs filled greedily), then the runs spread so that no rank is left
    empty while another holds two or more items."""
    n = len(weights)
    w = [max(0, int(x)) + 1 for x in weights]  # +1: unrequested / empty references still cost a little

    def runs(cap):
        cuts, load = [0], 0
        for i, x in enumerate(w):
            if load + x > cap and load > 0:
                cuts.append(i)
                load = 0
            load += x
        return cuts

    lo, hi = max(w, default=1), max(1, sum(w))
    while lo < hi:
        mid = (lo + hi) // 2
        if len(runs(mid)) <= world:
            hi = mid
        else:
            lo = mid + 1
    cuts = runs(lo)
    # more ranks than runs: split the runs with several items (largest first) while they last
    while len(cuts) < world:
        bounds = cuts + [n]
        best = max(range(len(cuts)), key=lambda i: (bounds[i + 1] - bounds[i] > 1,
                                                      sum(w[bounds[i]:bounds[i + 1]]), -i))
        a, b = bounds[best], bounds[best + 1]
        if b - a < 2:
            break
        half, acc, m = sum(w[a:b]) / 2, 0, a + 1
        for i in range(a, b - 1):
            acc += w[i]
            m = i + 1
            if acc >= half:
                break
        cuts.insert(best + 1, m)
    cuts += [n] * (world + 1 - len(cuts))
    return cuts


BOUND = -(2 ** 31)  # a cut at a reference's start (before any of its reads)


def plan_ranges(lengths: list, wanted: list, world: int, split_max: int):
    """The sharded decode's ranges: cut points [(refID, pos)] * (world + 1) of a coordinate-
    sorted file, rank r holding the records in [cut[r], cut[r + 1]) (coordinate order; pos BOUND:
    the reference's start; cut[world] = (n_refs, BOUND), the last rank also holds the unmapped
    reads).  When every requested reference is at most `split_max` positions long (C2-C4-like
    files), the requested references' concatenated positions are cut into `world` equal parts,
    so one reference's reads can be split over ranks (their histograms are then summed into the
    reference's owner); otherwise whole references (shard_contiguous).
    Returns (cuts, owner_of_tid, split_tids)."""
    n = len(lengths)
    wl = [int(L) if w else 0 for L, w in zip(lengths, wanted)]
    total = sum(wl)
    if world > 1 and total > 0 and all(int(L) <= split_max for L, w in zip(lengths, wanted) if w):
        cuts = [(0, BOUND)]
        starts = [0]
        for x in wl:
            starts.append(starts[-1] + x)
        for r in range(1, world):
            x = total * r // world
            t = next(u for u in range(n) if wl[u] > 0 and starts[u] <= x < starts[u + 1])
            pos = x - starts[t]
            cuts.append((t, BOUND) if pos == 0 else (t, pos))
        cuts.append((n, BOUND))
    else:
        cuts = [(t, BOUND) for t in shard_contiguous(wl, world)]
    split = {t for t, p in cuts[1:-1] if p != BOUND}
    owner = {}
    for t in range(n):
        owner[t] = max(r for r in range(world) if cuts[r] <= (t, BOUND))
    return cuts, owner, split


def _stdout_bytes(data: bytes) -> None:
    sys.stdout.flush()
    sys.stdout.buffer.write(data)
    sys.stdout.buffer.flush()


def ordered_write(group, order: list[str], owner: dict, blocks: dict, write=None) -> None:
    """Write each reference's bytes in `order` (rank 0's, agree_order), by its owning rank, one
    reference at a time (all ranks share the launcher's stdout; the barrier after each reference
    keeps the order)."""
    write = write or _stdout_bytes
    for ref in order:
        if owner[ref] == group.rank and ref in blocks:
            write(blocks[ref])
        group.barrier()
