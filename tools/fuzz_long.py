#!/usr/bin/env python3
"""Long seeded fuzz runs of the decoder and the verify step (device vs oracle), beyond the test
suite's sizes. Not a test: run on the GPU box, prints one JSON line per run.
    python tools/fuzz_long.py [seeds] [decode_objects_per_seed] [verify_trials_per_seed]
"""
import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main(seeds=4, n_dec=20000, n_ver=300):
    import mydatastore_amd as mde
    from oracle import wire_pb
    from tests.test_wire import GO_RULE_CASES, _expect_decode, _group_walk, _mutate
    from tests.test_verify import STATUS, _oracle_verify
    eng = mde.Engine(0)
    for seed in range(seeds):
        rng = np.random.default_rng(10_000 + seed)
        base = []
        for B in (1, 2, 3, 7, 30, 63, 64, 65, 128, 300):
            d = rng.integers(0, 999999, B).tolist()
            s = rng.integers(-2**31, 2**31, B).tolist() if B % 3 else rng.integers(0, 300, B).tolist()
            base.append(wire_pb.marshal(int(rng.integers(-9, 9)), int(rng.integers(0, 2**40)), 7, d, s,
                                        bool(B % 2)))
        # unknown groups nested past the decoder's 64-level ring (rescans) ahead of valid objects
        for t in ([70, 0], [130, 20, 200, 0], [65, 64, 66, 0]):
            base.append(_group_walk(rng, t)[0] + base[int(rng.integers(0, 10))])
        objs = [_mutate(rng, base[int(rng.integers(0, len(base)))]) for _ in range(n_dec)]
        objs += [b for b, _ in GO_RULE_CASES.values()]
        for cap in (64, 512):
            got = eng.decode_objects(objs, cap=cap)
            bad = [i for i, (g, o) in enumerate(zip(got, objs)) if g != _expect_decode(o, cap)]
            print(json.dumps({"fuzz": "decode", "seed": seed, "cap": cap, "objects": len(objs),
                              "errors_expected": sum(1 for g in got if not isinstance(g, dict)),
                              "mismatches": len(bad), "first": [objs[i].hex() for i in bad[:3]]}), flush=True)
        mism = 0
        for trial in range(n_ver):
            # B > 64 takes the fused kernel's kDeep instantiation (batched diff, block encode,
            # 256-entry decode window); up to the fused capacity of 1,024
            B = int(rng.integers(1, 130)) if trial % 4 else int(rng.integers(130, 1025))
            E, replica = int(rng.integers(0, 50)), int(rng.integers(1, 4))
            digests = rng.integers(0, 999999, size=B, dtype=np.uint64)
            sizes = rng.integers(0, 3000, size=B).astype(np.int32)
            _, nodes = eng.tree_from_digests(digests, B)
            d, s = [int(x) for x in digests], [int(x) for x in sizes]
            peers = []
            for _ in range(int(rng.integers(1, 9))):
                kind = int(rng.integers(0, 6))
                if kind == 0:
                    peers.append(None)
                    continue
                dd, ss = list(d), list(s)
                if kind in (1, 5):
                    for b in rng.choice(B, size=int(rng.integers(1, B + 1)), replace=False):
                        dd[b] = (dd[b] + 1 + int(rng.integers(0, 999997))) % 999999
                elif kind == 2:
                    nb = max(1, int(rng.integers(1, 2 * B + 2)))
                    dd = [int(x) for x in rng.integers(0, 999999, nb)] if nb > B else dd[:nb]
                    ss = [int(x) for x in rng.integers(0, 3000, len(dd))]
                obj = wire_pb.marshal(trial, E, E + 1, dd, ss, valid=bool(rng.integers(0, 2)))
                if kind == 5:
                    obj = _mutate(rng, obj)
                peers.append(obj)
            res = []
            for mode in (0, 1):
                eng.set_verify_mode(mode)
                res.append(eng.verify_epochs(B, digests, sizes, nodes, [peers], replica, E,
                                             partition=np.array([trial], np.int32)))
            eng.set_verify_mode(0)
            w = _oracle_verify(B, digests, sizes, [peers], replica, E, np.array([trial], np.int32))[0]
            g = res[0]
            ok = (res[0] == res[1] and g["valid"][0] == w["valid"] and g["valid_count"][0] == w["valid_count"]
                  and g["diff"][0] == w["diff"] and g["objects"][0] == w["object"]
                  and g["peer_status"][0] == [STATUS.get(x, x) for x in w["status"]])
            mism += not ok
        print(json.dumps({"fuzz": "verify", "seed": seed, "trials": n_ver, "mismatches": mism}), flush=True)


if __name__ == "__main__":
    main(*(int(x) for x in sys.argv[1:4]))
