"""Host-side oracle samples of the BASELINE workloads -- test infrastructure only.

The records of a few partitions of a synthetic workload, regenerated on
the host by the C restatement's own generator (oracle/mde_oracle.c: `"k%016x"` keys, SHA-256
bucket tags, splitmix64 values) -- independent of the device generator -- and laid out in the
LSM order (layout A) over exactly those partitions. Used by the `-m gpu` parity tests of the
full-size configs and by bench.py's `cpu_baseline` leg (its checker and its timed sample).
"""
from __future__ import annotations

import numpy as np

SYNTH_SEED = 0x4D445354
_MODES = {"block": 0, "mod": 1}


def sample_gids(n_keys: int, n_partitions: int, mode: str, part_ids) -> np.ndarray:
    """Global record ids of the listed partitions, ascending (the order make_workload and the
    oracle's stable layout both keep inside a bucket)."""
    P = n_partitions
    sample = np.asarray(part_ids, dtype=np.int64)
    kpp = -(-n_keys // P)
    if mode == "mod":  # p = gid % P
        g = (np.arange(kpp, dtype=np.uint64)[None, :] * np.uint64(P) + sample.astype(np.uint64)[:, None]).reshape(-1)
        return np.sort(g[g < n_keys])
    return np.concatenate([np.arange(p * kpp, min((p + 1) * kpp, n_keys), dtype=np.uint64) for p in sample])


def host_sample(co, n_keys: int, n_partitions: int, value_len: int, n_buckets: int, mode: str, part_ids,
                seed: int = SYNTH_SEED):
    """(values, seg_rec, n_sample, gids_in_layout_order) of the listed partitions, regenerated on
    the host; slot i of the sample is part_ids[i]."""
    P, B = n_partitions, n_buckets
    sample = np.asarray(part_ids, dtype=np.int64)
    g = sample_gids(n_keys, P, mode, sample)
    kpp = -(-n_keys // P)
    part, bk = co.synth_tags(g, P, B, _MODES[mode], kpp)
    slot = np.full(P, -1, np.int64)
    slot[sample] = np.arange(sample.size)
    order, seg = co.layout_a(slot[part].astype(np.uint32), bk, int(sample.size), B)
    gl = g[order]
    values = co.synth_values(gl, value_len, seed)
    return values, seg, int(sample.size), gl


def perturb_first_record(values: np.ndarray, seg: np.ndarray, value_len: int, n_buckets: int, part_ids):
    """Replica B of config 5 on a host sample: the first record of bucket
    (p * 37) % B of every listed partition p gets its first value byte + 1 mod 256. Returns the
    perturbed copy and {slot: bucket} of the partitions whose bucket was non-empty."""
    vb = values.copy()
    touched = {}
    for i, p in enumerate(part_ids):
        b = int(p * 37) % n_buckets
        r0, r1 = int(seg[i * n_buckets + b]), int(seg[i * n_buckets + b + 1])
        if r1 > r0:
            touched[i] = b
            vb[r0 * value_len] = (int(vb[r0 * value_len]) + 1) % 256
    return vb, touched
