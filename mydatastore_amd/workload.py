"""Device-resident synthetic KV workloads in layout A.

Records are generated directly in HBM by the engine's own kernels: the key of record ``gid`` is
``"k%016x" % gid``; its bucket is ``BE64(SHA256(key)[:8]) % B`` (main/manager.go:773-778); its
partition is ``gid // keys_per_partition`` ("block"), ``gid % P`` ("mod", round-robin) or
``FindPartitionID(key)`` ("hash"). Records are ordered by (partition, bucket) -- the order the
reference's per-bucket LSM range scans yield -- and the value bytes are splitmix64 words.
torch is used only to allocate HBM and to sort the tags (plumbing); hashing and value generation
run in the engine's HIP kernels.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

import mydatastore_amd as mde
from mydatastore_amd.dist import local_partitions, shard_gids

SYNTH_SEED = 0x4D445354
_MODES = {"block": 0, "mod": 1, "hash": 2}


@dataclass
class Workload:
    engine: "mde.Engine"
    values: "object"        # torch.uint8 [n * value_len] on device
    seg_rec: "object"       # torch.int64 [P*B + 1] on device (u64 bit pattern)
    n_partitions: int       # partitions held here (local)
    n_buckets: int
    n_records: int
    value_len: int
    partition_ids: np.ndarray  # global partition id of each local partition
    bucket_tag: "object" = None  # layout B: torch.int16 [n] bucket of each record
    part_rec: "object" = None    # layout B: torch.int64 [P+1]

    def __post_init__(self):
        import torch
        P, B, dev = self.n_partitions, self.n_buckets, self.values.device
        self.n_int = mde.tree_internal_nodes(B)
        if self.bucket_tag is not None:
            self.rec = mde.Records(self.values.data_ptr() if self.values.numel() else 0,
                                   self.values.numel(), self.value_len, mde.LAYOUT_TAGGED, 0,
                                   self.n_records, P, B, 0, self.bucket_tag.data_ptr(),
                                   self.part_rec.data_ptr())
        else:
            self.rec = mde.Records(self.values.data_ptr() if self.values.numel() else 0,
                                   self.values.numel(), self.value_len, mde.LAYOUT_SORTED, 0,
                                   self.n_records, P, B, self.seg_rec.data_ptr())

        def outs():
            o = {"digest": torch.zeros(P * B, dtype=torch.int64, device=dev),
                 "size": torch.zeros(P * B, dtype=torch.int32, device=dev),
                 "items": torch.zeros(P, dtype=torch.int32, device=dev),
                 "root": torch.zeros(P * 32, dtype=torch.uint8, device=dev),
                 "nodes": torch.zeros(P * self.n_int * 32, dtype=torch.uint8, device=dev)}
            return o, mde.TreeOut(*(o[k].data_ptr() for k in ("digest", "size", "items", "root", "nodes")))

        self.out, self.tree_out = outs()
        self._outs = outs

    @property
    def value_bytes(self) -> int:
        return self.n_records * self.value_len

    def build_async(self, out=None):
        """One Merkle build of every local partition, enqueued on the engine stream."""
        self.engine.build_async(self.rec, out if out is not None else self.tree_out)

    def digest_async(self):
        self.engine.digest_async(self.rec)

    def tree_async(self, out=None):
        self.engine.tree_async(self.rec, out if out is not None else self.tree_out)

    def build(self):
        """Synchronous build into fresh output tensors (for tests)."""
        o, to = self._outs()
        self.engine.build_async(self.rec, to)
        self.engine.synchronize()
        return o

    def diff(self, a, b):
        """DifferentMerkleTreeBuckets for every local partition between two builds."""
        import torch
        P, B = self.n_partitions, self.n_buckets
        cap = mde.diff_capacity(B, B)
        ids = torch.zeros(P * cap, dtype=torch.int32, device=self.values.device)
        cnt = torch.zeros(P, dtype=torch.int32, device=self.values.device)
        self.engine.diff_async(P, B, a["digest"], a["nodes"], B, b["digest"], b["nodes"], ids, cap, cnt)
        self.engine.synchronize()
        ids, cnt = ids.cpu().numpy(), cnt.cpu().numpy()
        return [int(c) if c < 0 else ids[p * cap:p * cap + c].tolist() for p, c in enumerate(cnt)]


def perturb_replica(w: Workload):
    """Replica B of BASELINE config 5: replica A's values with one record
    per partition changed -- the first record of bucket (p * 37) % B (p = global partition id)
    gets its first value byte + 1 mod 256, which always changes that bucket's digest (the sum moves
    by +1 or -255, never a multiple of 999999). Returns (values B on device, {local partition:
    bucket}) for the partitions whose bucket is non-empty."""
    import torch
    B, V = w.n_buckets, w.value_len
    vb = w.values.clone()
    seg = w.seg_rec.cpu().numpy()
    touched, idx = {}, []
    for lp, gp in enumerate(w.partition_ids):
        b = int(gp * 37) % B
        r0, r1 = int(seg[lp * B + b]), int(seg[lp * B + b + 1])
        if r1 > r0:
            touched[lp] = b
            idx.append(r0 * V)
    if idx:
        ii = torch.tensor(idx, dtype=torch.int64, device=vb.device)
        vb[ii] = ((vb[ii].to(torch.int32) + 1) % 256).to(torch.uint8)
    return vb, touched


def make_workload(engine: "mde.Engine", n_partitions: int, n_buckets: int, value_len: int,
                  part_mode: str = "block", keys_per_partition: int = 0, n_keys: int = 0,
                  rank: int = 0, world: int = 1, seed: int = SYNTH_SEED,
                  device: str = "cuda", layout: str = "a") -> Workload:
    """layout "a": records sorted by (partition, bucket) + seg_rec; layout "b": records grouped by
    partition in arrival (gid) order + per-record bucket tags + part_rec."""
    import torch
    if not n_keys:
        n_keys = n_partitions * keys_per_partition
    if part_mode == "block" and not keys_per_partition:
        keys_per_partition = -(-n_keys // n_partitions)
    dev = torch.device(f"{device}:{engine.device}") if device == "cuda" else torch.device(device)
    gids_np = shard_gids(n_keys, n_partitions, part_mode, keys_per_partition, rank, world)
    n = int(gids_np.size)
    pids = local_partitions(n_partitions, rank, world)
    P = int(pids.size)
    gids = torch.from_numpy(gids_np.view(np.int64)).to(dev)
    part = torch.empty(n, dtype=torch.int32, device=dev)
    bkt = torch.empty(n, dtype=torch.int32, device=dev)
    engine.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    engine.synth_tags_async(gids, n, n_partitions, n_buckets, _MODES[part_mode],
                            max(keys_per_partition, 1), part, bkt)
    local = part.to(torch.int64) // world   # partition p lives on rank p % world at slot p // world
    if layout == "b":
        comp = local
    else:
        comp = local * n_buckets + bkt.to(torch.int64)
    del part
    comp_sorted, order = torch.sort(comp, stable=True)
    nseg = P if layout == "b" else P * n_buckets
    counts = torch.bincount(comp_sorted, minlength=nseg)
    del comp, comp_sorted
    seg_rec = torch.zeros(nseg + 1, dtype=torch.int64, device=dev)
    seg_rec[1:] = torch.cumsum(counts, 0)
    sorted_gids = gids[order].contiguous()
    tags = bkt[order].to(torch.int16).contiguous() if layout == "b" else None
    del order, gids, counts, bkt
    values = torch.empty(n * value_len, dtype=torch.uint8, device=dev)
    engine.synth_values_async(values, sorted_gids, n, value_len, seed)
    torch.cuda.synchronize(dev)
    del sorted_gids
    if layout == "b":
        return Workload(engine, values, None, P, n_buckets, n, value_len, pids, tags, seg_rec)
    return Workload(engine, values, seg_rec, P, n_buckets, n, value_len, pids)
