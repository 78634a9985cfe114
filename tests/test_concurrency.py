"""Concurrent host calls on ONE shared context: the reference runs VerifyEpoch on any of 100
worker goroutines with up to 10 partition verifications in flight (main/manager.go:166-170,
main/consistency_controller.go:79-81), and the cgo shim shares one mde_ctx (INTEGRATION.md
section 2). Every entry point locks the context, so concurrent calls must serialize on it and
return exactly what the same calls return one at a time. ctypes releases the GIL for the foreign
call, so the host threads below really do enter the C ABI concurrently.
"""
import threading

import numpy as np
import pytest

from oracle import wire_pb


def _partition(rng, n, B):
    """One partition in the production shape: n records of 8-byte LE timestamps in B buckets."""
    ts = rng.integers(1, 2**40, n, dtype=np.uint64)
    values = ts.view(np.uint8)
    cuts = np.sort(rng.integers(0, n + 1, B - 1))
    seg = np.concatenate([[0], cuts, [n]]).astype(np.uint64)
    return values, seg


def _verify_call(engine, B, values, seg, peers_seed, E):
    out = engine.build(values, seg, 1, B, value_stride=8)
    dg, sz = out["digest"], out["size"]
    rng = np.random.default_rng(peers_seed)
    d2 = dg.copy()
    b = int(rng.integers(0, B))
    d2[b] = (int(d2[b]) + 1) % 999999
    peers = [[wire_pb.marshal(0, E, E + 1, [int(x) for x in dg], [int(x) for x in sz]),
              wire_pb.marshal(0, E, E + 1, [int(x) for x in d2], [int(x) for x in sz], valid=True)]]
    v = engine.verify_epochs(B, dg, sz, out["nodes"], peers, 2, E)
    return out["root"].tobytes(), v


@pytest.mark.gpu
def test_shared_context_concurrent_build_and_verify(engine):
    B, E, n_threads, per_thread = 64, 11, 8, 12
    rng = np.random.default_rng(99)
    work = [_partition(rng, int(rng.integers(500, 20000)), B) for _ in range(n_threads * per_thread)]
    serial = [_verify_call(engine, B, v, s, k, E) for k, (v, s) in enumerate(work)]
    got = [None] * len(work)
    errors = []

    def worker(t):
        try:
            for j in range(per_thread):
                k = t * per_thread + j
                got[k] = _verify_call(engine, B, *work[k], k, E)
        except Exception as e:  # surfaced below
            errors.append(e)

    threads = [threading.Thread(target=worker, args=(t,)) for t in range(n_threads)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=90)
    assert not any(th.is_alive() for th in threads), "a worker is stuck"
    assert not errors, errors[:3]
    assert got == serial
    # the verdicts themselves: one agreeing peer, one Valid peer differing in one bucket
    for root, v in got:
        assert v["valid"] == [True] and v["valid_count"] == [1] and len(v["diff"][0]) == 1


@pytest.mark.gpu
def test_shared_context_errors_stay_with_their_call(engine):
    """Threads sharing one context each get the message of THEIR failed call (the binding pairs
    the call and mde_last_error_copy in one critical section, as the Go shim's mdeCall does)."""
    import mydatastore_amd as mde
    values = np.zeros(64, np.uint8)
    bad_seg = np.array([0, 5, 3, 8], np.uint64)   # decreasing -> "nondecreasing" message
    long_seg = np.array([0, 100], np.uint64)      # 8 records only -> "exceeds n_records"
    errors, wrong = [], []

    def worker(t):
        try:
            for _ in range(40):
                try:
                    if t % 2:
                        engine.build(values, bad_seg, 1, 3, value_stride=8)
                    else:
                        engine.build(values, long_seg, 1, 1, value_stride=8)
                    wrong.append((t, "no error"))
                except mde.MdeError as e:
                    want = "nondecreasing" if t % 2 else "exceeds n_records"
                    if want not in str(e):
                        wrong.append((t, str(e)))
        except Exception as e:  # surfaced below
            errors.append(e)

    threads = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=60)
    assert not errors, errors[:3]
    assert not wrong, wrong[:5]
