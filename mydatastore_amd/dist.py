"""Partition sharding across GPUs and the per-build root gather.

Partitions are independent (main/merkle_tree.go:86-116 reads only one partition's records), so
partition p lives on rank p % world and each rank builds its partitions with no data exchange.
The single exchange step is the gather of the per-partition roots: every rank contributes one
fixed-size slab of ceil(P / world) x 32 bytes and `all_gather_into_tensor` (RCCL over xGMI with
the "nccl" backend; gloo on CPU for tests) delivers all roots to every rank. That is the in-node
analogue of the reference's gRPC fan-out of epoch trees (main/manager.go:729-771).
"""
from __future__ import annotations

import numpy as np


def weak_totals(n_keys: int, n_partitions: int, world: int) -> tuple[int, int]:
    """Weak scaling (bench.py default): every rank holds a workload of the per-GPU shape
    (n_partitions partitions, n_keys keys), so the job has world x both. With partition p on rank
    p % world and round-robin (p = gid % P) or block (p = gid // keys_per_partition) tagging, each
    rank's shard has exactly the single-GPU per-partition record counts."""
    return n_keys * world, n_partitions * world


def partition_rank(p: int, world: int) -> int:
    return p % world


def local_partitions(n_partitions: int, rank: int, world: int) -> np.ndarray:
    """Global ids of the partitions rank `rank` holds, in local slot order (slot i = p // world)."""
    return np.arange(rank, n_partitions, world, dtype=np.int64)


def shard_gids(n_keys: int, n_partitions: int, part_mode: str, keys_per_partition: int,
               rank: int = 0, world: int = 1) -> np.ndarray:
    """Global record ids whose partition lands on `rank`."""
    g = np.arange(n_keys, dtype=np.uint64)
    if world == 1:
        return g
    if part_mode == "block":
        p = g // np.uint64(keys_per_partition)
    elif part_mode == "mod":
        p = g % np.uint64(n_partitions)
    else:
        raise ValueError("hash partitioning is sharded after tagging; use world == 1")
    return g[(p % np.uint64(world)) == np.uint64(rank)]


class RootGather:
    """Fixed-size slab all-gather of per-partition 32-byte roots, double-buffered so a caller can
    keep the gather of build i in flight while build i+1 computes. `batch` > 1 buckets the roots
    of that many builds into one collective (slab [batch][ceil(P/world)][width] per rank): on a
    node each collective costs the same few tens of microseconds whatever its size (32 KiB per
    build at C4), and each cross-stream hand-off to the collective's stream costs ~10 us, so a
    run of builds gathers once per bucket."""

    def __init__(self, n_partitions: int, world: int, device, nbuf: int = 2, width: int = 32,
                 batch: int = 1):
        """width: bytes per partition (32 = one root; 64 = the roots of two replicas)."""
        import torch
        self.P, self.world, self.width, self.batch = n_partitions, world, width, batch
        self.slab = -(-n_partitions // world)
        per_rank = batch * self.slab * width
        self.send = [torch.zeros(per_rank, dtype=torch.uint8, device=device) for _ in range(nbuf)]
        self.recv = [torch.zeros(world * per_rank, dtype=torch.uint8, device=device) for _ in range(nbuf)]

    def gather(self, roots, buf: int = 0):
        """roots: this rank's [n_local * width] uint8 tensor, or a list of up to `batch` of them
        (one per build). Enqueued on the current stream."""
        import torch
        import torch.distributed as dist
        if not isinstance(roots, (list, tuple)):
            roots = [roots]
        if len(roots) > self.batch:
            raise ValueError(f"{len(roots)} builds exceed the gather bucket of {self.batch}")
        stride = self.slab * self.width
        for j, r in enumerate(roots):
            self.send[buf][j * stride:j * stride + r.numel()].copy_(r.reshape(-1), non_blocking=True)
        if dist.get_backend() == "gloo":  # CPU tests / single-GPU rehearsal: stage through host
            send = self.send[buf].cpu()
            parts = [t.cpu() for t in self.recv[buf].view(self.world, -1).unbind(0)]
            dist.all_gather(parts, send)
            self.recv[buf].copy_(torch.cat(parts))
        else:
            dist.all_gather_into_tensor(self.recv[buf], self.send[buf])
        return self.recv[buf]

    def assemble(self, buf: int = 0, build: int = 0) -> np.ndarray:
        """All roots of the bucket's `build`-th build in global partition order: [P, width] uint8
        (slot i of rank r = partition r + i * world)."""
        g = self.recv[buf].view(self.world, self.batch, self.slab, self.width)[:, build].cpu().numpy()
        out = np.zeros((self.P, self.width), np.uint8)
        for r in range(self.world):
            pids = local_partitions(self.P, r, self.world)
            out[pids] = g[r, :len(pids)]
        return out
