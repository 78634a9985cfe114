"""CPU, gloo world_size 2 (and 3): partition sharding p % world and the root gather used by
bench.py reassemble exactly the single-process roots. The C oracle stands in for the per-rank
build (no GPU here); the device path of the same code is exercised by bench.py at N > 1."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from tests.conftest import ROOT

P, B, N_KEYS, V = 12, 16, 3000, 40


def _oracle_roots(co, gids, n_parts_global, rank, world, mode, n_keys=N_KEYS):
    from mydatastore_amd.dist import local_partitions
    kpp = -(-n_keys // n_parts_global)
    part, bk = co.synth_tags(gids, n_parts_global, B, {"block": 0, "mod": 1}[mode], kpp)
    local = (part // world).astype(np.uint32)
    pl = len(local_partitions(n_parts_global, rank, world))
    order, seg = co.layout_a(local, bk, pl, B)
    vals = co.synth_values(gids[order], V, 0x4D445354)
    out = co.build(vals, seg, pl, B, V)
    return out["root"]


def _worker(rank, world, port, mode, q, batch=1, weak=False):
    import torch
    import torch.distributed as dist
    import sys
    sys.path.insert(0, str(ROOT))
    from mydatastore_amd.dist import RootGather, shard_gids
    from tests.oracle_c import COracle
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        co = COracle()
        from mydatastore_amd.dist import weak_totals
        n_keys, n_parts = weak_totals(N_KEYS, P, world) if weak else (N_KEYS, P)
        kpp = -(-n_keys // n_parts)
        gids = shard_gids(n_keys, n_parts, mode, kpp, rank, world)
        roots = _oracle_roots(co, gids, n_parts, rank, world, mode, n_keys)
        g = RootGather(n_parts, world, torch.device("cpu"), batch=batch)
        if batch == 1:
            g.gather(torch.from_numpy(roots.copy()), 0)
            allr = g.assemble(0)
        else:  # a bucket of builds: build j's roots are the real roots with every byte + j
            g.gather([torch.from_numpy((roots + j).astype(np.uint8)) for j in range(batch)], 1)
            allr = np.stack([g.assemble(1, j) for j in range(batch)])
        if rank == 0:
            q.put(allr)
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize("world,mode,batch,weak", [(2, "mod", 1, False), (2, "block", 1, False), (3, "mod", 1, False),
                                                  (2, "mod", 3, False), (2, "mod", 1, True), (3, "block", 1, True)])
def test_sharded_gather_matches_single_process(world, mode, batch, weak, coracle):
    """Strong (the config's total split over the ranks) and weak (bench.py's default: world x
    the partitions and keys): the ranks' sharded builds, gathered, equal one process's build of
    the whole job."""
    from mydatastore_amd.dist import weak_totals
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, mode, q, batch, weak)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n_keys, n_parts = weak_totals(N_KEYS, P, world) if weak else (N_KEYS, P)
    full = _oracle_roots(coracle, np.arange(n_keys, dtype=np.uint64), n_parts, 0, 1, mode, n_keys).reshape(n_parts, 32)
    if batch == 1:
        assert np.array_equal(got, full)
    else:
        for j in range(batch):
            assert np.array_equal(got[j], (full + j).astype(np.uint8)), j


def test_shard_partitions_cover_everything():
    from mydatastore_amd.dist import local_partitions, shard_gids
    for world in (1, 2, 4, 8):
        parts = np.concatenate([local_partitions(1024, r, world) for r in range(world)])
        assert sorted(parts.tolist()) == list(range(1024))
        gids = np.concatenate([shard_gids(10_000, 1024, "mod", 10, r, world) for r in range(world)])
        assert sorted(gids.tolist()) == list(range(10_000))


@pytest.mark.parametrize("mode,n_keys,P", [("mod", 10_000_000, 1024), ("block", 64_000_000, 64), ("mod", 3000, 12)])
def test_weak_shards_have_the_single_gpu_shape(mode, n_keys, P):
    """Weak scaling: every rank's shard of the world x workload holds P partitions with exactly
    the per-partition record counts of the single-GPU workload (so each GPU streams the same
    bytes as at N = 1)."""
    from mydatastore_amd.dist import local_partitions, weak_totals
    kpp = -(-n_keys // P)

    def counts(nk, np_, rank, world):
        # records per local slot without materialising the ids: round-robin p = gid % np_ has
        # ceil((nk - p) / np_) records, block tagging min(kpp, nk - p * kpp)
        pids = local_partitions(np_, rank, world)
        if mode == "mod":
            return -(-(nk - pids) // np_)
        return np.minimum(kpp, nk - pids * kpp)

    one = counts(n_keys, P, 0, 1)
    for world in (2, 4, 8):
        nk, np_ = weak_totals(n_keys, P, world)
        for rank in range(world):
            assert np.array_equal(counts(nk, np_, rank, world), one), (world, rank)
