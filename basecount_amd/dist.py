"""Multi-GPU (one process per GPU) plumbing for the CLI: contig sharding + gather to rank 0.

The counting path needs no communication: references are independent, so each
rank owns whole references (LPT on an estimate of their cost) and runs the single-GPU path on
them.  The only exchanges are
  * the per-reference range-error indices (all ranks must raise the same first error, in the
    reference's order: main.py's error timeline), and
  * the output: summary text is gathered to rank 0 over the process group (RCCL with the
    "nccl" backend, GPU-resident byte tensors), per-position rows are written by their owner in
    reference order (barrier per reference), so hundreds of GB of TSV never travel.

Launch: ``python -m torch.distributed.run --nproc-per-node N -m basecount_amd BAM ...`` (each
rank reads RANK / LOCAL_RANK / WORLD_SIZE; MASTER_ADDR=127.0.0.1).  Torch's bundled HIP runtime
must initialise before libbasecount_hip's, so ``init()`` runs first in ``run()``.
"""
from __future__ import annotations

import os
import sys


def env() -> tuple[int, int, int]:
    """(world_size, rank, local_rank) from the torchrun environment."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


class Group:
    """A torch.distributed process group plus the device its byte tensors live on."""

    def __init__(self, backend: str | None = None):
        import torch
        import torch.distributed as td

        self.td, self.torch = td, torch
        world, rank, local = env()
        if backend is None:
            backend = os.environ.get("BASECOUNT_DIST_BACKEND") or (
                "nccl" if torch.cuda.is_available() else "gloo")
        self.backend = backend
        if backend == "nccl":
            torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
            self.dev = torch.device("cuda", torch.cuda.current_device())
        else:
            self.dev = torch.device("cpu")
        if not td.is_initialized():
            kw = {"device_id": self.dev} if backend == "nccl" else {}
            # the backends log connection messages on fd 1: keep stdout for the TSV output
            sys.stdout.flush()
            saved = os.dup(1)
            try:
                os.dup2(2, 1)
                td.init_process_group(backend, **kw)
            finally:
                os.dup2(saved, 1)
                os.close(saved)
        self.world, self.rank = td.get_world_size(), td.get_rank()

    def barrier(self):
        if self.backend == "nccl":
            self.td.barrier(device_ids=[self.dev.index])
        else:
            self.td.barrier()

    def all_gather_ints(self, vals: list[int]) -> list[list[int]]:
        """Every rank's list of int64 (same length on all ranks)."""
        t = self.torch.tensor(vals, dtype=self.torch.int64, device=self.dev)
        out = [self.torch.empty_like(t) for _ in range(self.world)]
        self.td.all_gather(out, t)
        return [o.cpu().tolist() for o in out]

    def gather_bytes(self, data: bytes) -> list[bytes] | None:
        """Rank 0 receives every rank's bytes (ragged: sizes first, then padded payloads)."""
        sizes = [s[0] for s in self.all_gather_ints([len(data)])]
        n = max(sizes) if sizes else 0
        buf = self.torch.zeros(max(1, n), dtype=self.torch.uint8)
        if data:
            buf[: len(data)] = self.torch.frombuffer(bytearray(data), dtype=self.torch.uint8)
        buf = buf.to(self.dev)
        outs = [self.torch.empty_like(buf) for _ in range(self.world)]
        self.td.all_gather(outs, buf)
        if self.rank != 0:
            return None
        return [bytes(o.cpu().numpy()[: sizes[i]]) for i, o in enumerate(outs)]

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


def _stdout_bytes(data: bytes) -> None:
    sys.stdout.flush()
    sys.stdout.buffer.write(data)
    sys.stdout.buffer.flush()


def ordered_write(group: Group, order: list[str], owner: dict, blocks: dict, write=None) -> None:
    """Write each reference's bytes in `order`, by its owning rank, one reference at a time
    (all ranks share the launcher's stdout; the barrier after each reference keeps the order)."""
    write = write or _stdout_bytes
    for ref in order:
        if owner[ref] == group.rank and ref in blocks:
            write(blocks[ref])
        group.barrier()
