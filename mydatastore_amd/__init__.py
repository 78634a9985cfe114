"""mydatastore_amd -- MI355X anti-entropy Merkle engine (drop-in for main/merkle_tree.go).

The product is ``libmde.so`` (C ABI, ``include/mde.h``; gfx950 HIP kernels). This module is a
thin ctypes binding over that ABI for tests and benches; there is no Python or CPU fallback:
every call goes to the device and raises :class:`MdeError` when the library, the device or a
kernel fails.
"""
from __future__ import annotations

import ctypes as C
import os
import threading
from pathlib import Path

import numpy as np

_PKG = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("MDE_LIB", _PKG / "libmde.so"))

MDE_OK = 0
MDE_E_INVAL = -1
MDE_E_NOMEM = -2
MDE_E_DEVICE = -3
MDE_E_TREE = -4
MDE_E_CAPACITY = -5
MDE_E_DECODE = -6
HASH_MOD = 999999
LAYOUT_SORTED = 0  # layout A: sorted by (partition, bucket), seg_rec
LAYOUT_TAGGED = 1  # layout B: grouped by partition, per-record bucket tags

# Every symbol include/mde.h declares (checked by tests/test_abi.py).
EXPORTED_SYMBOLS = (
    "mde_abi_version", "mde_strerror", "mde_create", "mde_destroy", "mde_last_error",
    "mde_last_error_copy", "mde_group_last_error_copy",
    "mde_set_stream", "mde_use_own_stream", "mde_set_tuning", "mde_set_digest_piece_bytes", "mde_set_verify_mode", "mde_get_stream", "mde_synchronize", "mde_device_info", "mde_tree_depth",
    "mde_tree_internal_nodes", "mde_diff_capacity", "mde_build", "mde_build_async",
    "mde_build_streamed",
    "mde_digest_async", "mde_tree_async", "mde_build_pipelined_async", "mde_build_pipeline_drain_async",
    "mde_tree_from_digests", "mde_tree_from_digests_async",
    "mde_decode_bucket_hashes", "mde_diff", "mde_diff_async", "mde_diff_digests", "mde_tag_keys_async", "mde_tag_keys",
    "mde_extract", "mde_extract_async", "mde_stream_buckets", "mde_stream_buckets_async",
    "mde_epoch_tree_object_max_bytes",
    "mde_encode_epoch_tree_objects", "mde_encode_epoch_tree_objects_async",
    "mde_decode_epoch_tree_objects", "mde_decode_epoch_tree_objects_async", "mde_synth_tags_async", "mde_synth_values_async", "mde_dev_alloc", "mde_dev_free",
    "mde_memcpy_h2d", "mde_memcpy_d2h", "mde_verify_peer_capacity", "mde_verify_epochs",
    "mde_verify_epochs_async", "mde_group_create", "mde_group_destroy", "mde_group_size",
    "mde_group_ctx", "mde_group_last_error", "mde_multi_build", "mde_multi_build_streamed",
    "mde_group_gather_kind", "mde_group_partitions", "mde_group_build_async", "mde_group_build_pipelined_async",
    "mde_group_build_pipeline_drain_async", "mde_group_gather_async", "mde_group_synchronize", "mde_device_count",
    "mde_batcher_create", "mde_batcher_destroy", "mde_batcher_ctx", "mde_batcher_contexts", "mde_batcher_stats",
    "mde_batch_build", "mde_batch_verify", "mde_reserve_decode_scratch",
    "mde_server_create", "mde_server_destroy", "mde_server_slots", "mde_server_build", "mde_server_build_levels", "mde_server_verify", "mde_server_stats",
    "mde_tree_prefix_nodes", "mde_group_gather_overlapped_async", "mde_group_gather_wait_async",
    "mde_group_diff_async", "mde_group_extract_async", "mde_device_list", "mde_server_usable",
    "mde_server_disable", "mde_ctx_stats",
)


class MdeError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"mde error {code}: {msg}")
        self.code = code


class Records(C.Structure):
    """struct mde_records (include/mde.h)."""
    _fields_ = [
        ("values", C.c_void_p), ("values_bytes", C.c_uint64), ("value_stride", C.c_uint32),
        ("layout", C.c_uint32), ("value_off", C.c_void_p), ("n_records", C.c_uint64),
        ("n_partitions", C.c_uint32), ("n_buckets", C.c_uint32), ("seg_rec", C.c_void_p),
        ("bucket_tag", C.c_void_p), ("part_rec", C.c_void_p),
    ]


class TreeOut(C.Structure):
    """struct mde_tree_out (include/mde.h)."""
    _fields_ = [("digest", C.c_void_p), ("size", C.c_void_p), ("items", C.c_void_p),
                ("root", C.c_void_p), ("nodes", C.c_void_p)]


class DiffArgs(C.Structure):
    """struct mde_diff_args (include/mde.h): one device's mde_diff_async arguments."""
    _fields_ = [("n_pairs", C.c_uint32), ("n_buckets_a", C.c_uint32), ("n_buckets_b", C.c_uint32),
                ("digest_a", C.c_void_p), ("nodes_a", C.c_void_p), ("digest_b", C.c_void_p),
                ("nodes_b", C.c_void_p), ("out_ids", C.c_void_p), ("out_stride", C.c_uint64),
                ("out_count", C.c_void_p)]


class ExtractArgs(C.Structure):
    """struct mde_extract_args (include/mde.h): one device's mde_extract_async arguments."""
    _fields_ = [("ids", C.c_void_p), ("ids_stride", C.c_uint64), ("counts", C.c_void_p),
                ("part_off", C.c_void_p), ("out_rec", C.c_void_p), ("rec_cap", C.c_uint64),
                ("out_values", C.c_void_p), ("out_value_off", C.c_void_p), ("bytes_cap", C.c_uint64),
                ("status", C.c_void_p)]


_lib = None


def load_library() -> C.CDLL:
    """Load libmde.so (raises if it has not been built -- there is no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    path = Path(os.environ.get("MDE_LIBRARY", LIB_PATH))  # override: A/B of two builds
    if not path.exists():
        raise ImportError(f"{path} not built: run `python -m mydatastore_amd._build`")
    # One HIP runtime per process. torch ships its own libamdhip64 (SONAME libamdhip64.so.7, the
    # same SONAME as /opt/rocm's) but its libc10_hip asks for the unversioned file name, so if
    # libmde.so loaded /opt/rocm's runtime first, torch would load a second one and fail to find
    # the GPU. Loading torch first makes libmde.so bind to torch's runtime by SONAME.
    try:
        import torch  # noqa: F401
    except ImportError:  # standalone use: libmde.so binds /opt/rocm's runtime
        pass
    lib = C.CDLL(str(path))
    u32, u64, i32, vp = C.c_uint32, C.c_uint64, C.c_int32, C.c_void_p
    sig = {
        "mde_abi_version": (C.c_int, []),
        "mde_strerror": (C.c_char_p, [C.c_int]),
        "mde_create": (C.c_int, [C.c_int, C.POINTER(vp)]),
        "mde_destroy": (None, [vp]),
        "mde_last_error": (C.c_char_p, [vp]),
        "mde_last_error_copy": (C.c_uint64, [vp, C.c_char_p, C.c_uint64]),
        "mde_set_stream": (C.c_int, [vp, vp]),
        "mde_use_own_stream": (C.c_int, [vp]),
        "mde_set_tuning": (C.c_int, [vp, C.c_int, C.c_int, C.c_int]),
        "mde_ctx_stats": (C.c_int, [vp, vp, vp, vp]),
        "mde_set_digest_piece_bytes": (C.c_int, [vp, u64]),
        "mde_set_verify_mode": (C.c_int, [vp, C.c_int]),
        "mde_get_stream": (vp, [vp]),
        "mde_synchronize": (C.c_int, [vp]),
        "mde_device_info": (C.c_int, [vp, C.POINTER(C.c_int), C.c_char_p, C.c_int]),
        "mde_tree_depth": (u32, [u32]),
        "mde_tree_internal_nodes": (u64, [u32]),
        "mde_diff_capacity": (u64, [u32, u32]),
        "mde_build": (C.c_int, [vp, C.POINTER(Records), C.POINTER(TreeOut)]),
        "mde_build_async": (C.c_int, [vp, C.POINTER(Records), C.POINTER(TreeOut)]),
        "mde_build_streamed": (C.c_int, [vp, C.POINTER(Records), C.POINTER(TreeOut), u64]),
        "mde_digest_async": (C.c_int, [vp, C.POINTER(Records)]),
        "mde_tree_async": (C.c_int, [vp, C.POINTER(Records), C.POINTER(TreeOut)]),
        "mde_build_pipelined_async": (C.c_int, [vp, C.POINTER(Records), C.POINTER(TreeOut)]),
        "mde_build_pipeline_drain_async": (C.c_int, [vp]),
        "mde_tree_from_digests": (C.c_int, [vp, u32, u32, vp, vp, vp]),
        "mde_tree_from_digests_async": (C.c_int, [vp, u32, u32, vp, vp, vp]),
        "mde_decode_bucket_hashes": (C.c_int, [vp, vp, u32, vp]),
        "mde_diff": (C.c_int, [vp, u32, u32, vp, vp, u32, vp, vp, vp, u64, vp]),
        "mde_diff_async": (C.c_int, [vp, u32, u32, vp, vp, u32, vp, vp, vp, u64, vp]),
        "mde_diff_digests": (C.c_int, [vp, u32, u32, vp, u32, vp, vp, u64, vp]),
        "mde_tag_keys_async": (C.c_int, [vp, vp, vp, u64, u32, u32, vp, vp]),
        "mde_tag_keys": (C.c_int, [vp, vp, vp, u64, u32, u32, vp, vp]),
        "mde_extract": (C.c_int, [vp, C.POINTER(Records), vp, u64, vp, vp, vp, u64, vp, vp, u64]),
        "mde_extract_async": (C.c_int, [vp, C.POINTER(Records), vp, u64, vp, vp, vp, u64, vp, vp, u64, vp]),
        "mde_stream_buckets": (C.c_int, [vp, C.POINTER(Records), vp, u64, vp, vp, vp, u64, vp, vp, u64]),
        "mde_stream_buckets_async": (C.c_int, [vp, C.POINTER(Records), vp, u64, vp, vp, vp, u64, vp, vp, u64, vp]),
        "mde_epoch_tree_object_max_bytes": (u64, [u32]),
        "mde_encode_epoch_tree_objects": (C.c_int, [vp, u32, u32, vp, C.c_int64, C.c_int64, vp, vp, vp, vp, vp, u64, vp]),
        "mde_encode_epoch_tree_objects_async": (C.c_int, [vp, u32, u32, vp, C.c_int64, C.c_int64, vp, vp, vp, vp, vp, u64, vp]),
        "mde_decode_epoch_tree_objects": (C.c_int, [vp, u32, vp, vp, u32, vp, vp, vp, vp, vp, vp, vp, vp]),
        "mde_decode_epoch_tree_objects_async": (C.c_int, [vp, u32, vp, vp, u32, vp, vp, vp, vp, vp, vp, vp, vp]),
        "mde_verify_peer_capacity": (u32, [u32]),
        "mde_reserve_decode_scratch": (C.c_int, [vp, u64, u64]),
        "mde_verify_epochs": (C.c_int, [vp, u32, u32, vp, C.c_int64, vp, vp, vp, u32, vp, vp, u32,
                                        vp, vp, vp, vp, vp, vp, u64, vp]),
        "mde_verify_epochs_async": (C.c_int, [vp, u32, u32, vp, C.c_int64, vp, vp, vp, u32, vp, vp,
                                              u32, vp, vp, vp, vp, vp, vp, u64, vp]),
        "mde_group_create": (C.c_int, [vp, u32, C.POINTER(vp)]),
        "mde_group_destroy": (None, [vp]),
        "mde_group_size": (u32, [vp]),
        "mde_group_ctx": (vp, [vp, u32]),
        "mde_group_last_error": (C.c_char_p, [vp]),
        "mde_group_last_error_copy": (C.c_uint64, [vp, C.c_char_p, C.c_uint64]),
        "mde_multi_build": (C.c_int, [vp, C.POINTER(Records), C.POINTER(TreeOut)]),
        "mde_multi_build_streamed": (C.c_int, [vp, C.POINTER(Records), C.POINTER(TreeOut), C.c_uint64]),
        "mde_group_gather_kind": (C.c_char_p, [vp]),
        "mde_group_partitions": (u32, [vp, u32, u32]),
        "mde_group_build_async": (C.c_int, [vp, C.POINTER(Records), C.POINTER(TreeOut)]),
        "mde_group_build_pipelined_async": (C.c_int, [vp, C.POINTER(Records), C.POINTER(TreeOut)]),
        "mde_group_build_pipeline_drain_async": (C.c_int, [vp]),
        "mde_group_gather_async": (C.c_int, [vp, C.POINTER(vp), C.POINTER(vp), C.c_uint64]),
        "mde_group_synchronize": (C.c_int, [vp]),
        "mde_group_gather_overlapped_async": (C.c_int, [vp, C.POINTER(vp), C.POINTER(vp), C.c_uint64,
                                                        C.POINTER(C.c_uint64)]),
        "mde_group_gather_wait_async": (C.c_int, [vp, C.c_uint64]),
        "mde_group_diff_async": (C.c_int, [vp, C.POINTER(DiffArgs)]),
        "mde_group_extract_async": (C.c_int, [vp, C.POINTER(Records), C.POINTER(ExtractArgs)]),
        "mde_device_count": (C.c_int, []),
        "mde_batcher_create": (C.c_int, [C.c_int, u32, u32, C.POINTER(vp)]),
        "mde_batcher_destroy": (None, [vp]),
        "mde_batcher_ctx": (vp, [vp, u32]),
        "mde_batcher_contexts": (u32, [vp]),
        "mde_batcher_stats": (C.c_int, [vp, vp, vp, vp]),
        "mde_batch_build": (C.c_int, [vp, C.POINTER(Records), C.POINTER(TreeOut), C.c_char_p, u64]),
        "mde_server_create": (C.c_int, [C.c_int, u32, u32, C.POINTER(vp)]),
        "mde_server_destroy": (None, [vp]),
        "mde_server_slots": (u32, [vp]),
        "mde_server_build": (C.c_int, [vp, C.POINTER(Records), C.POINTER(TreeOut), C.c_char_p, u64]),
        "mde_server_stats": (C.c_int, [vp, vp, vp, vp]),
        "mde_server_usable": (C.c_int, [vp]),
        "mde_server_disable": (C.c_int, [vp, C.c_char_p]),
        "mde_device_list": (C.c_int, [vp, C.c_int]),
        "mde_server_build_levels": (C.c_int, [vp, C.POINTER(Records), C.POINTER(TreeOut), u32, C.c_char_p, u64]),
        "mde_tree_prefix_nodes": (u64, [u32, u32]),
        "mde_server_verify": (C.c_int, [vp, u32, C.c_int32, C.c_int64, vp, vp, u32, vp, vp, u32, vp, vp, vp, vp,
                                        vp, vp, u64, vp, C.c_char_p, u64]),
        "mde_batch_verify": (C.c_int, [vp, u32, i32, C.c_int64, vp, vp, u32, vp, vp, u32, vp, vp, vp, vp,
                                       vp, vp, u64, vp, C.c_char_p, u64]),
        "mde_synth_tags_async": (C.c_int, [vp, vp, u64, u32, u32, C.c_int, u64, vp, vp]),
        "mde_synth_values_async": (C.c_int, [vp, vp, vp, u64, u32, u64]),
        "mde_dev_alloc": (C.c_int, [vp, u64, C.POINTER(vp)]),
        "mde_dev_free": (C.c_int, [vp, vp]),
        "mde_memcpy_h2d": (C.c_int, [vp, vp, vp, u64]),
        "mde_memcpy_d2h": (C.c_int, [vp, vp, vp, u64]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def tree_internal_nodes(n_buckets: int) -> int:
    return int(load_library().mde_tree_internal_nodes(n_buckets))


def tree_depth(n_buckets: int) -> int:
    return int(load_library().mde_tree_depth(n_buckets))


def diff_capacity(b1: int, b2: int) -> int:
    return int(load_library().mde_diff_capacity(b1, b2))


def _build_outputs(P: int, B: int, want_nodes: bool, want_tree: bool) -> dict:
    """Host output arrays of a build; a digest-only build (want_tree False) has no root / nodes."""
    return {
        "digest": np.zeros(P * B, np.uint64), "size": np.zeros(P * B, np.int32),
        "items": np.zeros(P, np.int32), "root": np.zeros(P * 32, np.uint8) if want_tree else None,
        "nodes": np.zeros(P * tree_internal_nodes(B) * 32, np.uint8) if want_nodes and want_tree else None,
    }


def _ptr(a) -> int:
    """Address of a numpy array or a torch tensor (None -> NULL)."""
    if a is None:
        return 0
    if isinstance(a, np.ndarray):
        if not a.flags["C_CONTIGUOUS"]:
            raise ValueError("array must be C-contiguous")
        return a.ctypes.data
    if hasattr(a, "data_ptr"):
        if not a.is_contiguous():
            raise ValueError("tensor must be contiguous")
        return a.data_ptr()
    raise TypeError(f"unsupported buffer type {type(a)}")


def _nbytes(a) -> int:
    if isinstance(a, np.ndarray):
        return a.nbytes
    return a.numel() * a.element_size()


class Engine:
    """One mde_ctx (device, stream, scratch). Host-array methods are synchronous; ``*_async``
    methods take device tensors and enqueue on the context stream (see :meth:`set_stream`)."""

    def __init__(self, device: int = 0):
        self._mu = threading.Lock()
        self.lib = load_library()
        h = C.c_void_p()
        rc = self.lib.mde_create(device, C.byref(h))
        if rc != MDE_OK:
            raise MdeError(rc, f"mde_create(device={device}) failed: "
                               f"{self.lib.mde_strerror(rc).decode()} (needs a gfx950 GPU)")
        self.ctx = h
        self.device = device

    def close(self):
        if getattr(self, "ctx", None):
            self.lib.mde_destroy(self.ctx)
            self.ctx = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def _call(self, name: str, *args):
        """Call entry point `name` on this context and raise MdeError with ITS message: the call
        and the message copy are one critical section, so threads sharing the Engine cannot
        swap messages (the context lock serialises the calls anyway)."""
        with self._mu:
            rc = getattr(self.lib, name)(self.ctx, *args)
            if rc == MDE_OK:
                return
            buf = C.create_string_buffer(512)
            self.lib.mde_last_error_copy(self.ctx, buf, len(buf))
        raise MdeError(rc, buf.value.decode(errors="replace") or self.lib.mde_strerror(rc).decode())

    # -- context ------------------------------------------------------------------------------
    def set_stream(self, stream_handle: int):
        """Launch on a HIP stream handle (0 = the null stream = torch's default stream)."""
        self._call("mde_set_stream", C.c_void_p(int(stream_handle)))

    def set_tuning(self, digest_variant: int = -1, digest_blocks_per_cu: int = -1, digest_oversub: int = -1):
        self._call("mde_set_tuning", digest_variant, digest_blocks_per_cu, digest_oversub)

    def set_digest_piece_bytes(self, piece_bytes: int = -1):
        """Layout-A digest work split: 0 = one range per wave, N = interleaved ~N-byte pieces,
        -1 = the built-in default."""
        self._call("mde_set_digest_piece_bytes", (1 << 64) - 1 if piece_bytes < 0 else piece_bytes)

    def set_verify_mode(self, mode: int):
        """0 = fused one-launch verify when it fits (default), 1 = the five-launch chain."""
        self._call("mde_set_verify_mode", mode)

    def use_own_stream(self):
        self._call("mde_use_own_stream")

    def synchronize(self):
        self._call("mde_synchronize")

    def device_info(self):
        cus = C.c_int()
        arch = C.create_string_buffer(64)
        self._call("mde_device_info", C.byref(cus), arch, 64)
        return cus.value, arch.value.decode()

    # -- build --------------------------------------------------------------------------------
    @staticmethod
    def records(values, n_partitions, n_buckets, seg_rec, value_stride=0, value_off=None,
                n_records=None) -> Records:
        if n_records is None:
            n_records = int(seg_rec[-1]) if isinstance(seg_rec, np.ndarray) else None
        if n_records is None:
            raise ValueError("n_records required for device seg_rec")
        return Records(_ptr(values), _nbytes(values) if values is not None else 0, value_stride, 0,
                       _ptr(value_off), n_records, n_partitions, n_buckets, _ptr(seg_rec))

    def build(self, values: np.ndarray, seg_rec: np.ndarray, n_partitions: int, n_buckets: int,
              value_stride: int = 0, value_off: np.ndarray | None = None, want_nodes=True, want_tree=True):
        """RawPartitionMerkleTree for P partitions from host arrays (H2D, build, D2H).
        want_tree=False: a digest-only build (root and nodes None: digests, sizes, items)."""
        P, B = n_partitions, n_buckets
        seg_rec = np.ascontiguousarray(seg_rec, dtype=np.uint64)
        values = np.ascontiguousarray(values, dtype=np.uint8).reshape(-1)
        if value_off is not None:
            value_off = np.ascontiguousarray(value_off, dtype=np.uint64)
        n_rec = (value_off.size - 1) if value_off is not None else (
            values.size // value_stride if value_stride else 0)
        rec = Records(_ptr(values), values.nbytes, value_stride, 0, _ptr(value_off), n_rec, P, B,
                      _ptr(seg_rec))
        out = _build_outputs(P, B, want_nodes, want_tree)
        to = TreeOut(*(_ptr(out[k]) for k in ("digest", "size", "items", "root", "nodes")))
        self._call("mde_build", C.byref(rec), C.byref(to))
        return out

    def build_streamed(self, values, seg_rec, n_partitions, n_buckets, value_stride=0,
                       value_off=None, chunk_bytes=0, want_nodes=True, part_rec=None, bucket_tag=None,
                       want_tree=True):
        """mde_build_streamed: host arena streamed through a two-slot device ring. `values` may
        be a numpy array or a (pinned) CPU torch tensor. Layout B: pass part_rec + bucket_tag
        (seg_rec None)."""
        P, B = n_partitions, n_buckets
        if value_off is not None:
            value_off = np.ascontiguousarray(value_off, dtype=np.uint64)
        nbytes = _nbytes(values)
        n_rec = (value_off.size - 1) if value_off is not None else (nbytes // value_stride if value_stride else 0)
        if part_rec is not None:
            part_rec = np.ascontiguousarray(part_rec, dtype=np.uint64)
            bucket_tag = np.ascontiguousarray(bucket_tag, dtype=np.uint16)
            rec = Records(_ptr(values), nbytes, value_stride, LAYOUT_TAGGED, 0, n_rec, P, B, 0,
                          _ptr(bucket_tag), _ptr(part_rec))
        else:
            seg_rec = np.ascontiguousarray(seg_rec, dtype=np.uint64)
            rec = Records(_ptr(values), nbytes, value_stride, 0, _ptr(value_off), n_rec, P, B, _ptr(seg_rec))
        out = _build_outputs(P, B, want_nodes, want_tree)
        to = TreeOut(*(_ptr(out[k]) for k in ("digest", "size", "items", "root", "nodes")))
        self._call("mde_build_streamed", C.byref(rec), C.byref(to), chunk_bytes)
        return out

    def build_tagged(self, values: np.ndarray, part_rec: np.ndarray, bucket_tag: np.ndarray,
                     n_partitions: int, n_buckets: int, value_stride: int, want_nodes=True, want_tree=True):
        """Layout B build: records grouped by partition in arrival order + bucket tags."""
        P, B = n_partitions, n_buckets
        values = np.ascontiguousarray(values, dtype=np.uint8).reshape(-1)
        part_rec = np.ascontiguousarray(part_rec, dtype=np.uint64)
        tags = np.ascontiguousarray(bucket_tag, dtype=np.uint16)
        rec = Records(_ptr(values), values.nbytes, value_stride, LAYOUT_TAGGED, 0,
                      values.size // value_stride, P, B, 0, _ptr(tags), _ptr(part_rec))
        out = _build_outputs(P, B, want_nodes, want_tree)
        to = TreeOut(*(_ptr(out[k]) for k in ("digest", "size", "items", "root", "nodes")))
        self._call("mde_build", C.byref(rec), C.byref(to))
        return out

    def build_async(self, rec: Records, out: TreeOut):
        self._call("mde_build_async", C.byref(rec), C.byref(out))

    def digest_async(self, rec: Records):
        self._call("mde_digest_async", C.byref(rec))

    def tree_async(self, rec: Records, out: TreeOut):
        self._call("mde_tree_async", C.byref(rec), C.byref(out))

    def build_pipelined_async(self, rec: Records, out: TreeOut):
        """One software-pipelined build (mde_build_pipelined_async): this call's digest and the
        previous call's trees in one launch; `out` is complete after the next call or a drain."""
        self._call("mde_build_pipelined_async", C.byref(rec), C.byref(out))

    def build_pipeline_drain_async(self):
        self._call("mde_build_pipeline_drain_async")

    # -- tree from digests (EpochTreeObjectToMerkleTree) --------------------------------------
    def tree_from_digests(self, digests: np.ndarray, n_buckets: int, want_nodes=True):
        d = np.ascontiguousarray(digests, dtype=np.uint64).reshape(-1)
        T = d.size // n_buckets
        root = np.zeros(T * 32, np.uint8)
        nodes = np.zeros(T * tree_internal_nodes(n_buckets) * 32, np.uint8) if want_nodes else None
        self._call("mde_tree_from_digests", T, n_buckets, _ptr(d), _ptr(root),
                                                   _ptr(nodes))
        return root, nodes

    def tree_from_digests_async(self, n_trees, n_buckets, digest, root, nodes=None):
        self._call("mde_tree_from_digests_async", n_trees, n_buckets, _ptr(digest),
                                                         _ptr(root), _ptr(nodes))

    # -- diff (DifferentMerkleTreeBuckets) ----------------------------------------------------
    def diff(self, ba: int, da: np.ndarray, na: np.ndarray, bb: int, db: np.ndarray,
             nb: np.ndarray, n_pairs: int = 1):
        """Returns a list (per pair) of bucket-id lists, or MDE_E_TREE where the reference errors."""
        cap = diff_capacity(ba, bb)
        ids = np.zeros(n_pairs * cap, np.int32)
        cnt = np.zeros(n_pairs, np.int32)
        da, db = (np.ascontiguousarray(x, dtype=np.uint64) for x in (da, db))
        na, nb = (np.ascontiguousarray(x, dtype=np.uint8) for x in (na, nb))
        self._call("mde_diff", n_pairs, ba, _ptr(da), _ptr(na), bb, _ptr(db),
                                      _ptr(nb), _ptr(ids), cap, _ptr(cnt))
        res = []
        for i in range(n_pairs):
            c = int(cnt[i])
            res.append(c if c < 0 else ids[i * cap:i * cap + c].tolist())
        return res

    def diff_digests(self, ba: int, da: np.ndarray, bb: int, db: np.ndarray, n_pairs: int = 1):
        """mde_diff_digests: trees built on device from the two digest vectors, then diffed."""
        cap = diff_capacity(ba, bb)
        ids = np.zeros(n_pairs * cap, np.int32)
        cnt = np.zeros(n_pairs, np.int32)
        da, db = (np.ascontiguousarray(x, dtype=np.uint64) for x in (da, db))
        self._call("mde_diff_digests", n_pairs, ba, _ptr(da), bb, _ptr(db),
                                              _ptr(ids), cap, _ptr(cnt))
        return [int(c) if c < 0 else ids[i * cap:i * cap + int(c)].tolist() for i, c in enumerate(cnt)]

    def diff_async(self, n_pairs, ba, da, na, bb, db, nb, out_ids, out_stride, out_count):
        self._call("mde_diff_async", n_pairs, ba, _ptr(da), _ptr(na), bb, _ptr(db),
                                            _ptr(nb), _ptr(out_ids), out_stride, _ptr(out_count))

    # -- out-of-sync range extract (StreamBucketsTask) ----------------------------------------
    def extract(self, values, seg_rec, n_partitions, n_buckets, ids, ids_stride, counts,
                value_stride=0, value_off=None, want_values=True, part_rec=None, bucket_tag=None):
        """Records of the listed buckets per partition (dedup; layout A: ascending bucket, LSM
        order; layout B -- part_rec + bucket_tag instead of seg_rec -- arrival order).
        Returns (part_off, rec_idx, values_bytes, value_off)."""
        values = np.ascontiguousarray(values, dtype=np.uint8).reshape(-1)
        if value_off is not None:
            value_off = np.ascontiguousarray(value_off, dtype=np.uint64)
        n_rec = (value_off.size - 1) if value_off is not None else (
            values.size // value_stride if value_stride else 0)
        if part_rec is not None:
            part_rec = np.ascontiguousarray(part_rec, dtype=np.uint64)
            bucket_tag = np.ascontiguousarray(bucket_tag, dtype=np.uint16)
            rec = Records(_ptr(values), values.nbytes, value_stride, LAYOUT_TAGGED, 0, n_rec,
                          n_partitions, n_buckets, 0, _ptr(bucket_tag), _ptr(part_rec))
        else:
            seg_rec = np.ascontiguousarray(seg_rec, dtype=np.uint64)
            rec = Records(_ptr(values), values.nbytes, value_stride, 0, _ptr(value_off), n_rec,
                          n_partitions, n_buckets, _ptr(seg_rec))
        ids = np.ascontiguousarray(ids, dtype=np.int32)
        counts = np.ascontiguousarray(counts, dtype=np.int32)
        rec_cap = max(int(n_rec), 1)
        bytes_cap = max(values.nbytes, 1)
        part_off = np.zeros(n_partitions + 1, np.uint64)
        out_rec = np.zeros(rec_cap, np.uint64)
        out_vals = np.zeros(bytes_cap, np.uint8) if want_values else None
        out_voff = np.zeros(rec_cap + 1, np.uint64) if want_values else None
        self._call("mde_extract", C.byref(rec), _ptr(ids), ids_stride, _ptr(counts),
                                         _ptr(part_off), _ptr(out_rec), rec_cap, _ptr(out_vals),
                                         _ptr(out_voff), bytes_cap)
        n = int(part_off[-1])
        if not want_values:
            return part_off, out_rec[:n], None, None
        return part_off, out_rec[:n], out_vals[:int(out_voff[n])], out_voff[:n + 1]

    def stream_buckets(self, values, seg_rec, n_partitions, n_buckets, ids, ids_stride, counts,
                       value_stride=0, value_off=None, want_values=True):
        """mde_stream_buckets: StreamBucketsTask's request-order contract (main/manager.go:447-485)
        -- ids walked as given, repeats streamed again, ids outside [0, B) stream nothing,
        counts[p] == 0 streams every bucket. Layout A. Returns (part_off, rec_idx, values_bytes,
        value_off); the output capacities are the requests' record and byte totals."""
        values = np.ascontiguousarray(values, dtype=np.uint8).reshape(-1)
        if value_off is not None:
            value_off = np.ascontiguousarray(value_off, dtype=np.uint64)
        n_rec = (value_off.size - 1) if value_off is not None else (
            values.size // value_stride if value_stride else 0)
        seg_rec = np.ascontiguousarray(seg_rec, dtype=np.uint64)
        rec = Records(_ptr(values), values.nbytes, value_stride, 0, _ptr(value_off), n_rec,
                      n_partitions, n_buckets, _ptr(seg_rec))
        ids = np.ascontiguousarray(ids, dtype=np.int32)
        counts = np.ascontiguousarray(counts, dtype=np.int32)
        # capacities: every request's run (repeats included)
        nrec = seg_rec[1:].astype(np.int64) - seg_rec[:-1].astype(np.int64)
        segb = (value_off[seg_rec.astype(np.int64)] if value_off is not None
                else seg_rec * np.uint64(value_stride)).astype(np.int64)
        nbyt = segb[1:] - segb[:-1]
        need_r = need_b = 0
        for p in range(n_partitions):
            c = int(counts[p])
            req = (np.arange(n_buckets) if c == 0 else
                   ids[p * ids_stride: p * ids_stride + max(c, 0)].astype(np.int64))
            req = req[(req >= 0) & (req < n_buckets)] + p * n_buckets
            need_r += int(nrec[req].sum())
            need_b += int(nbyt[req].sum())
        rec_cap, bytes_cap = max(need_r, 1), max(need_b, 1)
        part_off = np.zeros(n_partitions + 1, np.uint64)
        out_rec = np.zeros(rec_cap, np.uint64)
        out_vals = np.zeros(bytes_cap, np.uint8) if want_values else None
        out_voff = np.zeros(rec_cap + 1, np.uint64) if want_values else None
        self._call("mde_stream_buckets", C.byref(rec), _ptr(ids), ids_stride, _ptr(counts),
                   _ptr(part_off), _ptr(out_rec), rec_cap, _ptr(out_vals), _ptr(out_voff), bytes_cap)
        n = int(part_off[-1])
        if not want_values:
            return part_off, out_rec[:n], None, None
        return part_off, out_rec[:n], out_vals[:int(out_voff[n])], out_voff[:n + 1]

    def stream_buckets_async(self, rec: Records, ids, ids_stride, counts, part_off, out_rec, rec_cap,
                             out_values, out_value_off, bytes_cap, status):
        self._call("mde_stream_buckets_async", C.byref(rec), _ptr(ids), ids_stride,
                   _ptr(counts), _ptr(part_off), _ptr(out_rec), rec_cap,
                   _ptr(out_values), _ptr(out_value_off), bytes_cap, _ptr(status))

    def extract_async(self, rec: Records, ids, ids_stride, counts, part_off, out_rec, rec_cap,
                      out_values, out_value_off, bytes_cap, status):
        self._call("mde_extract_async", C.byref(rec), _ptr(ids), ids_stride,
                                               _ptr(counts), _ptr(part_off), _ptr(out_rec), rec_cap,
                                               _ptr(out_values), _ptr(out_value_off), bytes_cap,
                                               _ptr(status))

    # -- EpochTreeObject wire bytes -----------------------------------------------------------
    def encode_objects(self, n_buckets, digest, size, partition=None, lower=0, upper=0, valid=None,
                       items=None, n_objects=None):
        """proto.Marshal(EpochTreeObject) for each of the n trees: list of bytes objects
        (n_buckets = 0: objects without buckets; pass n_objects)."""
        B = n_buckets
        digest = np.ascontiguousarray(digest, dtype=np.uint64)
        size = np.ascontiguousarray(size, dtype=np.int32)
        n = n_objects if n_objects is not None else digest.size // B
        stride = int(self.lib.mde_epoch_tree_object_max_bytes(B))
        out = np.zeros(n * stride, np.uint8)
        ln = np.zeros(n, np.uint32)
        part = None if partition is None else np.ascontiguousarray(partition, dtype=np.int32)
        val = None if valid is None else np.ascontiguousarray(valid, dtype=np.uint8)
        it = None if items is None else np.ascontiguousarray(items, dtype=np.int32)
        self._call("mde_encode_epoch_tree_objects", n, B, _ptr(part), lower, upper,
                                                           _ptr(digest), _ptr(size), _ptr(val), _ptr(it),
                                                           _ptr(out), stride, _ptr(ln))
        return [out[i * stride:i * stride + int(ln[i])].tobytes() for i in range(n)]

    def decode_objects(self, objs, cap):
        """Decode EpochTreeObject bytes: list of dicts (or an MDE_E_* code per object)."""
        n = len(objs)
        off = np.zeros(n + 1, np.uint64)
        off[1:] = np.cumsum([len(o) for o in objs])
        blob = np.frombuffer(b"".join(objs) or b"\0", dtype=np.uint8).copy()
        o = {"partition": np.zeros(n, np.int32), "lower": np.zeros(n, np.int64),
             "upper": np.zeros(n, np.int64), "digest": np.zeros(n * cap, np.uint64),
             "size": np.zeros(n * cap, np.int32), "valid": np.zeros(n, np.uint8),
             "items": np.zeros(n, np.int32), "n_buckets": np.zeros(n, np.int32)}
        self._call("mde_decode_epoch_tree_objects",
            n, _ptr(blob), _ptr(off), cap, *(_ptr(o[k]) for k in (
                "partition", "lower", "upper", "digest", "size", "valid", "items", "n_buckets")))
        res = []
        for i in range(n):
            nb = int(o["n_buckets"][i])
            if nb < 0:
                res.append(nb)
                continue
            res.append({"partition": int(o["partition"][i]), "lower": int(o["lower"][i]),
                        "upper": int(o["upper"][i]), "valid": bool(o["valid"][i]),
                        "items": int(o["items"][i]),
                        "digest": o["digest"][i * cap:i * cap + nb].tolist(),
                        "size": o["size"][i * cap:i * cap + nb].tolist()})
        return res

    # -- VerifyEpoch decision step ------------------------------------------------------------
    def verify_epochs(self, n_buckets, digest, size, nodes, peer_objects, replica_count, epoch,
                      partition=None, want_objects=True):
        """Manager.VerifyEpoch over P partitions (mde_verify_epochs). ``peer_objects[p]`` is the
        list of peer EpochTreeObject wire bytes for partition p (None = absent peer); every
        partition must list the same number of peers. Returns a dict with valid, valid_count,
        diff (ascending Int32Set per partition), peer_status ([P][R]) and objects (the persisted
        EpochTreeObject bytes per partition)."""
        B = n_buckets
        digest = np.ascontiguousarray(digest, dtype=np.uint64).reshape(-1)
        size = np.ascontiguousarray(size, dtype=np.int32).reshape(-1)
        if nodes is not None:  # None: each partition builds its tree on the device if a peer needs it
            nodes = np.ascontiguousarray(nodes, dtype=np.uint8).reshape(-1)
        P = digest.size // B
        R = len(peer_objects[0]) if P else 0
        if any(len(x) != R for x in peer_objects):
            raise ValueError("every partition needs the same number of peer slots")
        flat = [o or b"" for row in peer_objects for o in row]
        off = np.zeros(len(flat) + 1, np.uint64)
        off[1:] = np.cumsum([len(o) for o in flat])
        blob = np.frombuffer(b"".join(flat) or b"\0", dtype=np.uint8).copy()
        part = None if partition is None else np.ascontiguousarray(partition, dtype=np.int32)
        valid = np.zeros(P, np.uint8)
        vcount = np.zeros(P, np.int32)
        ids = np.zeros(P * B, np.int32)
        dcount = np.zeros(P, np.int32)
        status = np.zeros(max(P * R, 1), np.int32)
        stride = int(self.lib.mde_epoch_tree_object_max_bytes(B)) if want_objects else 0
        objs = np.zeros(max(P * stride, 1), np.uint8) if want_objects else None
        olen = np.zeros(P, np.uint32) if want_objects else None
        self._call("mde_verify_epochs",
            P, B, _ptr(part), epoch, _ptr(digest), _ptr(size), _ptr(nodes), R, _ptr(blob),
            _ptr(off), replica_count, _ptr(valid), _ptr(vcount), _ptr(ids), _ptr(dcount),
            _ptr(status), _ptr(objs), stride, _ptr(olen))
        return {
            "valid": [bool(v) for v in valid], "valid_count": vcount.tolist(),
            "diff": [ids[p * B:p * B + int(dcount[p])].tolist() for p in range(P)],
            "peer_status": [status[p * R:(p + 1) * R].tolist() for p in range(P)],
            "objects": ([objs[p * stride:p * stride + int(olen[p])].tobytes() for p in range(P)]
                        if want_objects else None),
        }

    def verify_epochs_async(self, n_partitions, n_buckets, partition, epoch, digest, size, nodes,
                            n_peers, peer_bytes, peer_off, replica_count, valid, valid_count,
                            diff_ids, diff_count, peer_status=None, object_out=None,
                            object_stride=0, object_len=None):
        self._call("mde_verify_epochs_async",
            n_partitions, n_buckets, _ptr(partition), epoch, _ptr(digest), _ptr(size),
            _ptr(nodes), n_peers, _ptr(peer_bytes), _ptr(peer_off), replica_count, _ptr(valid),
            _ptr(valid_count), _ptr(diff_ids), _ptr(diff_count), _ptr(peer_status),
            _ptr(object_out), object_stride, _ptr(object_len))

    # -- tagging / synthetic workload ---------------------------------------------------------
    def tag_keys(self, keys, n_buckets: int, n_partitions: int):
        """(bucket, partition) for a list of byte keys (getKeyBucket / FindPartitionID)."""
        offs = np.zeros(len(keys) + 1, np.uint64)
        offs[1:] = np.cumsum([len(k) for k in keys])
        blob = np.frombuffer(b"".join(keys) or b"\0", dtype=np.uint8).copy()
        bk = np.zeros(len(keys), np.uint32)
        pt = np.zeros(len(keys), np.uint32)
        self._call("mde_tag_keys", _ptr(blob), _ptr(offs), len(keys), n_buckets,
                                          n_partitions, _ptr(bk), _ptr(pt))
        return bk, pt

    def tag_keys_async(self, keys, key_off, n, n_buckets, n_partitions, bucket, partition):
        self._call("mde_tag_keys_async", _ptr(keys), _ptr(key_off), n, n_buckets,
                                                n_partitions, _ptr(bucket), _ptr(partition))

    def synth_tags_async(self, gids, n, n_partitions, n_buckets, part_mode, kpp, part, bucket):
        self._call("mde_synth_tags_async", _ptr(gids), n, n_partitions, n_buckets,
                                                  part_mode, kpp, _ptr(part), _ptr(bucket))

    def synth_values_async(self, dst, gids, n, value_len, seed):
        self._call("mde_synth_values_async", _ptr(dst), _ptr(gids), n, value_len,
                                                    seed)


class Group:
    """mde_group: one process driving several GPUs; partition p on device p % G, the roots
    all-gathered over RCCL (or device copies when a device is listed twice)."""

    def __init__(self, devices):
        self._mu = threading.Lock()
        self.lib = load_library()
        devs = (C.c_int * len(devices))(*devices)
        h = C.c_void_p()
        rc = self.lib.mde_group_create(devs, len(devices), C.byref(h))
        if rc != MDE_OK:
            raise MdeError(rc, f"mde_group_create({list(devices)}) failed: {self.lib.mde_strerror(rc).decode()}")
        self.g = h

    def close(self):
        if getattr(self, "g", None):
            self.lib.mde_group_destroy(self.g)
            self.g = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def __len__(self):
        return int(self.lib.mde_group_size(self.g))

    @property
    def gather_kind(self) -> str:
        return self.lib.mde_group_gather_kind(self.g).decode()

    def partitions(self, n_partitions: int, i: int) -> int:
        """Partitions on device i (i, i + G, ...)."""
        return int(self.lib.mde_group_partitions(self.g, n_partitions, i))

    def ctx(self, i: int):
        return self.lib.mde_group_ctx(self.g, i)

    def ctx_stats(self, i: int):
        """mde_ctx_stats of device i's context: {"builds", "partitions", "value_bytes"}."""
        v = [C.c_uint64() for _ in range(3)]
        self._check(self.lib.mde_ctx_stats(self.ctx(i), *[C.byref(x) for x in v]))
        return dict(zip(("builds", "partitions", "value_bytes"), (int(x.value) for x in v)))

    def _check(self, rc):
        if rc != MDE_OK:
            buf = C.create_string_buffer(512)
            self.lib.mde_group_last_error_copy(self.g, buf, len(buf))
            raise MdeError(rc, buf.value.decode(errors="replace"))

    def build_async(self, shards, outs, pipelined=False):
        """mde_group_build[_pipelined]_async: shards / outs = one Records / TreeOut per device
        (device-i pointers)."""
        n = len(self)
        recs = (Records * n)(*shards)
        tos = (TreeOut * n)(*outs)
        fn = self.lib.mde_group_build_pipelined_async if pipelined else self.lib.mde_group_build_async
        self._check(fn(self.g, recs, tos))

    def drain_async(self):
        self._check(self.lib.mde_group_build_pipeline_drain_async(self.g))

    def gather_async(self, send, recv, nbytes: int):
        """mde_group_gather_async: send[i] / recv[i] device-i tensors (or pointers)."""
        n = len(self)
        s = (C.c_void_p * n)(*[_ptr(x) if not isinstance(x, int) else x for x in send])
        r = (C.c_void_p * n)(*[_ptr(x) if not isinstance(x, int) else x for x in recv])
        self._check(self.lib.mde_group_gather_async(self.g, s, r, nbytes))

    def gather_overlapped_async(self, send, recv, nbytes: int) -> int:
        """mde_group_gather_overlapped_async: the gather on each device's side stream; returns its
        ticket for gather_wait_async."""
        n = len(self)
        s = (C.c_void_p * n)(*[_ptr(x) if not isinstance(x, int) else x for x in send])
        r = (C.c_void_p * n)(*[_ptr(x) if not isinstance(x, int) else x for x in recv])
        t = C.c_uint64()
        self._check(self.lib.mde_group_gather_overlapped_async(self.g, s, r, nbytes, C.byref(t)))
        return int(t.value)

    def gather_wait_async(self, ticket: int):
        self._check(self.lib.mde_group_gather_wait_async(self.g, ticket))

    def diff_async(self, args):
        """mde_group_diff_async: one DiffArgs per device (device-i pointers)."""
        self._check(self.lib.mde_group_diff_async(self.g, (DiffArgs * len(self))(*args)))

    def extract_async(self, shards, args):
        """mde_group_extract_async: one Records + ExtractArgs per device."""
        n = len(self)
        self._check(self.lib.mde_group_extract_async(self.g, (Records * n)(*shards), (ExtractArgs * n)(*args)))

    def synchronize(self):
        self._check(self.lib.mde_group_synchronize(self.g))

    def build(self, values, n_partitions, n_buckets, value_stride=0, value_off=None, seg_rec=None,
              part_rec=None, bucket_tag=None, want_nodes=True, streamed=False, chunk_bytes=0, want_tree=True):
        """mde_multi_build (or mde_multi_build_streamed) from host arrays (layout A with seg_rec,
        or layout B with part_rec + bucket_tag); same outputs as Engine.build."""
        P, B = n_partitions, n_buckets
        values = np.ascontiguousarray(values, dtype=np.uint8).reshape(-1)
        if value_off is not None:
            value_off = np.ascontiguousarray(value_off, dtype=np.uint64)
        n_rec = (value_off.size - 1) if value_off is not None else (values.size // value_stride if value_stride else 0)
        if part_rec is not None:
            part_rec = np.ascontiguousarray(part_rec, dtype=np.uint64)
            bucket_tag = np.ascontiguousarray(bucket_tag, dtype=np.uint16)
            rec = Records(_ptr(values), values.nbytes, value_stride, LAYOUT_TAGGED, 0, n_rec, P, B, 0,
                          _ptr(bucket_tag), _ptr(part_rec))
        else:
            seg_rec = np.ascontiguousarray(seg_rec, dtype=np.uint64)
            rec = Records(_ptr(values), values.nbytes, value_stride, LAYOUT_SORTED, _ptr(value_off), n_rec, P, B,
                          _ptr(seg_rec))
        out = _build_outputs(P, B, want_nodes, want_tree)
        to = TreeOut(*(_ptr(out[k]) for k in ("digest", "size", "items", "root", "nodes")))
        # the call and the copy of ITS message are one critical section (threads sharing a Group
        # cannot swap messages; the group lock serialises the builds anyway)
        with self._mu:
            if streamed:
                rc = self.lib.mde_multi_build_streamed(self.g, C.byref(rec), C.byref(to), chunk_bytes)
            else:
                rc = self.lib.mde_multi_build(self.g, C.byref(rec), C.byref(to))
            if rc != MDE_OK:
                buf = C.create_string_buffer(512)
                self.lib.mde_group_last_error_copy(self.g, buf, len(buf))
        if rc != MDE_OK:
            raise MdeError(rc, buf.value.decode(errors="replace"))
        return out


class Batcher:
    """mde_batcher: concurrent one-partition calls coalesced into one device build / verify (group
    commit). Thread-safe; ctypes releases the GIL, so Python threads really call concurrently."""

    def __init__(self, device: int = 0, max_partitions: int = 256, max_wait_us: int = 0):
        self.lib = load_library()
        h = C.c_void_p()
        rc = self.lib.mde_batcher_create(device, max_partitions, max_wait_us, C.byref(h))
        if rc != MDE_OK:
            raise MdeError(rc, f"mde_batcher_create(device={device}) failed: {self.lib.mde_strerror(rc).decode()}")
        self.b = h

    def close(self):
        if getattr(self, "b", None):
            self.lib.mde_batcher_destroy(self.b)
            self.b = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def stats(self):
        v = [C.c_uint64() for _ in range(3)]
        self.lib.mde_batcher_stats(self.b, *(C.byref(x) for x in v))
        return {"batches": v[0].value, "requests": v[1].value, "partitions": v[2].value}

    def build(self, values, seg_rec, n_partitions, n_buckets, value_stride=0, value_off=None, want_nodes=True,
              want_tree=True):
        """mde_batch_build: RawPartitionMerkleTree for this caller's partitions; same outputs as
        Engine.build (want_tree=False: digest-only)."""
        P, B = n_partitions, n_buckets
        seg_rec = np.ascontiguousarray(seg_rec, dtype=np.uint64)
        values = np.ascontiguousarray(values, dtype=np.uint8).reshape(-1)
        if value_off is not None:
            value_off = np.ascontiguousarray(value_off, dtype=np.uint64)
        n_rec = (value_off.size - 1) if value_off is not None else (values.size // value_stride if value_stride else 0)
        rec = Records(_ptr(values), values.nbytes, value_stride, 0, _ptr(value_off), n_rec, P, B, _ptr(seg_rec))
        out = _build_outputs(P, B, want_nodes, want_tree)
        to = TreeOut(*(_ptr(out[k]) for k in ("digest", "size", "items", "root", "nodes")))
        err = C.create_string_buffer(512)
        rc = self.lib.mde_batch_build(self.b, C.byref(rec), C.byref(to), err, len(err))
        if rc != MDE_OK:
            raise MdeError(rc, err.value.decode(errors="replace"))
        return out

    def verify(self, n_buckets, digest, size, peer_objects, replica_count, epoch, partition=0, want_object=True):
        """mde_batch_verify for one partition: peer_objects = list of wire bytes (None = absent)."""
        B = n_buckets
        digest = np.ascontiguousarray(digest, dtype=np.uint64).reshape(-1)
        size = np.ascontiguousarray(size, dtype=np.int32).reshape(-1)
        R = len(peer_objects)
        flat = [o or b"" for o in peer_objects]
        off = np.zeros(R + 1, np.uint64)
        off[1:] = np.cumsum([len(o) for o in flat])
        blob = np.frombuffer(b"".join(flat) or b"\0", dtype=np.uint8).copy()
        valid = np.zeros(1, np.uint8)
        vc = np.zeros(1, np.int32)
        ids = np.zeros(B, np.int32)
        dc = np.zeros(1, np.int32)
        st = np.zeros(max(R, 1), np.int32)
        stride = int(self.lib.mde_epoch_tree_object_max_bytes(B)) if want_object else 0
        obj = np.zeros(max(stride, 1), np.uint8) if want_object else None
        olen = np.zeros(1, np.uint32) if want_object else None
        err = C.create_string_buffer(512)
        rc = self.lib.mde_batch_verify(self.b, B, int(partition), epoch, _ptr(digest), _ptr(size), R, _ptr(blob),
                                       _ptr(off), replica_count, _ptr(valid), _ptr(vc), _ptr(ids), _ptr(dc),
                                       _ptr(st), _ptr(obj), stride, _ptr(olen), err, len(err))
        if rc != MDE_OK:
            raise MdeError(rc, err.value.decode(errors="replace"))
        return {"valid": bool(valid[0]), "valid_count": int(vc[0]), "diff": ids[:int(dc[0])].tolist(),
                "peer_status": st[:R].tolist(),
                "object": obj[:int(olen[0])].tobytes() if want_object else None}


class Server:
    """mde_server: the resident build service -- one-partition builds served by a persistent
    launch polling request slots in pinned host memory (no launch, copy or event per call).
    Thread-safe; ctypes releases the GIL."""

    def __init__(self, device: int = 0, n_slots: int = 0, max_buckets: int = 0):
        self.lib = load_library()
        h = C.c_void_p()
        rc = self.lib.mde_server_create(device, n_slots, max_buckets, C.byref(h))
        if rc != MDE_OK:
            raise MdeError(rc, f"mde_server_create(device={device}) failed: {self.lib.mde_strerror(rc).decode()}")
        self.s = h

    def close(self):
        if getattr(self, "s", None):
            self.lib.mde_server_destroy(self.s)
            self.s = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def stats(self):
        v = [C.c_uint64() for _ in range(3)]
        self.lib.mde_server_stats(self.s, *(C.byref(x) for x in v))
        return {"requests": v[0].value, "launches": v[1].value, "on_context": v[2].value}

    @property
    def usable(self) -> bool:
        """mde_server_usable: the resident launch serves calls (else they run on its context)."""
        return bool(self.lib.mde_server_usable(self.s))

    def disable(self, why: str = ""):
        """mde_server_disable: take the resident launch out of service; later calls run on the
        service's context."""
        rc = self.lib.mde_server_disable(self.s, why.encode())
        if rc != MDE_OK:
            raise MdeError(rc, "mde_server_disable failed")

    def build(self, values, seg_rec, n_partitions, n_buckets, value_stride=0, value_off=None, want_nodes=True,
              want_tree=True):
        """mde_server_build: same outputs as Engine.build / Batcher.build."""
        P, B = n_partitions, n_buckets
        seg_rec = np.ascontiguousarray(seg_rec, dtype=np.uint64)
        values = np.ascontiguousarray(values, dtype=np.uint8).reshape(-1)
        if value_off is not None:
            value_off = np.ascontiguousarray(value_off, dtype=np.uint64)
        n_rec = (value_off.size - 1) if value_off is not None else (values.size // value_stride if value_stride else 0)
        rec = Records(_ptr(values), values.nbytes, value_stride, 0, _ptr(value_off), n_rec, P, B, _ptr(seg_rec))
        out = _build_outputs(P, B, want_nodes, want_tree)
        to = TreeOut(*(_ptr(out[k]) for k in ("digest", "size", "items", "root", "nodes")))
        err = C.create_string_buffer(512)
        rc = self.lib.mde_server_build(self.s, C.byref(rec), C.byref(to), err, len(err))
        if rc != MDE_OK:
            raise MdeError(rc, err.value.decode(errors="replace"))
        return out

    def build_levels(self, values, seg_rec, n_partitions, n_buckets, top_nodes, value_stride=0, value_off=None):
        """mde_server_build_levels: digests, sizes, items and the tree's levels 1 .. the first of at
        most top_nodes nodes (the first mde_tree_prefix_nodes(B, top_nodes) of every partition's
        nodes; the nodes past that prefix are unspecified -- a call the service runs on its context
        writes every level -- and the caller hashes them)."""
        P, B = n_partitions, n_buckets
        seg_rec = np.ascontiguousarray(seg_rec, dtype=np.uint64)
        values = np.ascontiguousarray(values, dtype=np.uint8).reshape(-1)
        if value_off is not None:
            value_off = np.ascontiguousarray(value_off, dtype=np.uint64)
        n_rec = (value_off.size - 1) if value_off is not None else (values.size // value_stride if value_stride else 0)
        rec = Records(_ptr(values), values.nbytes, value_stride, 0, _ptr(value_off), n_rec, P, B, _ptr(seg_rec))
        out = _build_outputs(P, B, True, True)
        out["root"] = None
        to = TreeOut(*(_ptr(out[k]) for k in ("digest", "size", "items", "root", "nodes")))
        err = C.create_string_buffer(512)
        rc = self.lib.mde_server_build_levels(self.s, C.byref(rec), C.byref(to), top_nodes, err, len(err))
        if rc != MDE_OK:
            raise MdeError(rc, err.value.decode(errors="replace"))
        out["prefix_nodes"] = int(self.lib.mde_tree_prefix_nodes(B, top_nodes))
        return out

    def verify(self, n_buckets, digest, size, peer_objects, replica_count, epoch, partition=0, want_object=True):
        """mde_server_verify: Batcher.verify's contract, served by the resident launch."""
        B = n_buckets
        digest = np.ascontiguousarray(digest, dtype=np.uint64).reshape(-1)
        size = np.ascontiguousarray(size, dtype=np.int32).reshape(-1)
        R = len(peer_objects)
        flat = [o or b"" for o in peer_objects]
        off = np.zeros(R + 1, np.uint64)
        off[1:] = np.cumsum([len(o) for o in flat])
        blob = np.frombuffer(b"".join(flat) or b"\0", dtype=np.uint8).copy()
        valid = np.zeros(1, np.uint8)
        vc = np.zeros(1, np.int32)
        ids = np.zeros(B, np.int32)
        dc = np.zeros(1, np.int32)
        st = np.zeros(max(R, 1), np.int32)
        stride = int(self.lib.mde_epoch_tree_object_max_bytes(B)) if want_object else 0
        obj = np.zeros(max(stride, 1), np.uint8) if want_object else None
        olen = np.zeros(1, np.uint32) if want_object else None
        err = C.create_string_buffer(512)
        rc = self.lib.mde_server_verify(self.s, B, int(partition), epoch, _ptr(digest), _ptr(size), R, _ptr(blob),
                                        _ptr(off), replica_count, _ptr(valid), _ptr(vc), _ptr(ids), _ptr(dc),
                                        _ptr(st), _ptr(obj), stride, _ptr(olen), err, len(err))
        if rc != MDE_OK:
            raise MdeError(rc, err.value.decode(errors="replace"))
        return {"valid": bool(valid[0]), "valid_count": int(vc[0]), "diff": ids[:int(dc[0])].tolist(),
                "peer_status": st[:R].tolist(),
                "object": obj[:int(olen[0])].tobytes() if want_object else None}

