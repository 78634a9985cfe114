"""Test-input builders: reconstruct a golden synth case's arrays (layout A) on the host."""
import numpy as np

from oracle import oracle as O

MODES = {"block": 0, "mod": 1, "hash": 2}


def synth_arrays(case, coracle):
    """values (u8), value_off (u64 or None), stride, seg_rec for a tests/golden synth case."""
    n, P, B = case["n"], case["P"], case["B"]
    gids = np.arange(n, dtype=np.uint64)
    part, bk = coracle.synth_tags(gids, P, B, MODES[case["part_mode"]], case["keys_per_partition"])
    order, seg = coracle.layout_a(part, bk, P, B)
    assert seg.tolist() == case["seg_rec"], case["name"]
    sg = gids[order]
    seed = case["seed"]
    if case["var_len"]:
        lens = (O.synth_value_words(sg, 1, seed)[:, 0] % np.uint64(300) + np.uint64(1)).astype(np.uint64)
        value_off = np.zeros(n + 1, np.uint64)
        np.cumsum(lens, out=value_off[1:])
        values = np.concatenate([coracle.synth_values(sg[i:i + 1], int(lens[i]), seed)
                                 for i in range(n)]) if n else np.zeros(0, np.uint8)
        return values, value_off, 0, seg
    values = coracle.synth_values(sg, case["value_len"], seed)
    return values, None, case["value_len"], seg


def mtr_arena(fix, lo, hi):
    """TestMerkleTreeRaw: the epoch-index values (LE64 timestamps) of epochs [lo, hi), grouped by
    bucket in LSM order (main/merkle_tree.go:90-113, main/manager.go:780-818)."""
    B = fix["n_buckets"]
    rows = [(fix["bucket_of"][k], f"{e:010d}", k, ts) for k, e, ts in fix["writes"] if lo <= e < hi]
    rows.sort(key=lambda r: (r[0], r[1], r[2]))  # key order within a bucket: epoch_p_b_EEEE_key
    vals = np.array([r[3] for r in rows], dtype="<i8").view(np.uint8)
    counts = np.bincount([r[0] for r in rows], minlength=B) if rows else np.zeros(B, np.int64)
    seg = np.zeros(B + 1, np.uint64)
    np.cumsum(counts, out=seg[1:])
    return vals, seg
