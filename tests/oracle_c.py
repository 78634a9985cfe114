"""ctypes binding of oracle/build/liboracle.so (the C restatement) -- test infrastructure only."""
import ctypes as C
import subprocess
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
LIB = ROOT / "oracle" / "build" / "liboracle.so"


def _p(a):
    return None if a is None else a.ctypes.data


class COracle:
    def __init__(self):
        if not LIB.exists():
            subprocess.run([sys.executable, "-m", "mydatastore_amd._build", "-q"], cwd=ROOT, check=True)
        L = C.CDLL(str(LIB))
        u8p = C.c_void_p
        L.oracle_sha256.argtypes = [u8p, C.c_uint64, u8p]
        L.oracle_xxh64.argtypes = [u8p, C.c_uint64, C.c_uint64]
        L.oracle_xxh64.restype = C.c_uint64
        L.oracle_key_bucket.argtypes = [u8p, C.c_uint64, C.c_uint32]
        L.oracle_key_bucket.restype = C.c_uint32
        L.oracle_find_partition.argtypes = [u8p, C.c_uint64, C.c_uint32]
        L.oracle_find_partition.restype = C.c_uint32
        L.oracle_synth_values.argtypes = [u8p, u8p, C.c_uint64, C.c_uint32, C.c_uint64]
        L.oracle_synth_tags.argtypes = [u8p, C.c_uint64, C.c_uint32, C.c_uint32, C.c_int, C.c_uint64, u8p, u8p]
        L.oracle_layout_a.argtypes = [u8p, u8p, C.c_uint64, C.c_uint32, C.c_uint32, u8p, u8p]
        L.oracle_layout_a.restype = C.c_int
        L.oracle_n_internal.argtypes = [C.c_uint32]
        L.oracle_n_internal.restype = C.c_uint64
        L.oracle_tree.argtypes = [u8p, C.c_uint32, u8p, u8p]
        L.oracle_build.argtypes = [u8p, C.c_uint32, u8p, u8p, C.c_uint32, C.c_uint32, u8p, u8p, u8p, u8p, u8p, C.c_int]
        L.oracle_diff.argtypes = [u8p, C.c_uint32, u8p, C.c_uint32, u8p, C.c_int32]
        L.oracle_diff.restype = C.c_int32
        self.L = L

    def sha256(self, m: bytes) -> bytes:
        buf = np.frombuffer(m or b"\0", np.uint8).copy()
        out = np.zeros(32, np.uint8)
        self.L.oracle_sha256(_p(buf), len(m), _p(out))
        return out.tobytes()

    def xxh64(self, m: bytes, seed=0) -> int:
        buf = np.frombuffer(m or b"\0", np.uint8).copy()
        return int(self.L.oracle_xxh64(_p(buf), len(m), seed))

    def synth_values(self, gids, value_len, seed):
        gids = np.ascontiguousarray(gids, np.uint64)
        out = np.zeros(len(gids) * value_len, np.uint8)
        self.L.oracle_synth_values(_p(out), _p(gids), len(gids), value_len, seed)
        return out

    def synth_tags(self, gids, P, B, mode, kpp):
        gids = np.ascontiguousarray(gids, np.uint64)
        part = np.zeros(len(gids), np.uint32)
        bk = np.zeros(len(gids), np.uint32)
        self.L.oracle_synth_tags(_p(gids), len(gids), P, B, mode, kpp, _p(part), _p(bk))
        return part, bk

    def layout_a(self, part, bk, P, B):
        part = np.ascontiguousarray(part, np.uint32)
        bk = np.ascontiguousarray(bk, np.uint32)
        order = np.zeros(len(part), np.uint64)
        seg = np.zeros(P * B + 1, np.uint64)
        assert self.L.oracle_layout_a(_p(part), _p(bk), len(part), P, B, _p(order), _p(seg)) == 0
        return order, seg

    def build(self, values, seg_rec, P, B, stride=0, value_off=None, threads=1, want_nodes=True):
        values = np.ascontiguousarray(values, np.uint8)
        seg_rec = np.ascontiguousarray(seg_rec, np.uint64)
        vo = None if value_off is None else np.ascontiguousarray(value_off, np.uint64)
        ni = int(self.L.oracle_n_internal(B))
        out = {"digest": np.zeros(P * B, np.uint64), "size": np.zeros(P * B, np.int32),
               "items": np.zeros(P, np.int32), "root": np.zeros(P * 32, np.uint8),
               "nodes": np.zeros(P * ni * 32, np.uint8) if want_nodes else None}
        self.L.oracle_build(_p(values), stride, _p(vo), _p(seg_rec), P, B, _p(out["digest"]),
                            _p(out["size"]), _p(out["items"]), _p(out["root"]), _p(out["nodes"]), threads)
        return out

    def tree(self, digests, B):
        d = np.ascontiguousarray(digests, np.uint64)
        ni = int(self.L.oracle_n_internal(B))
        nodes = np.zeros(ni * 32, np.uint8)
        root = np.zeros(32, np.uint8)
        self.L.oracle_tree(_p(d), B, _p(nodes), _p(root))
        return root.tobytes(), nodes.tobytes()

    def diff(self, d1, d2):
        d1 = np.ascontiguousarray(d1, np.uint64)
        d2 = np.ascontiguousarray(d2, np.uint64)
        cap = 4 * (len(d1) + len(d2)) + 16
        out = np.zeros(cap, np.int32)
        n = int(self.L.oracle_diff(_p(d1), len(d1), _p(d2), len(d2), _p(out), cap))
        return n if n < 0 else out[:n].tolist()
