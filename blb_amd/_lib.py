"""ctypes binding of libblbrs.so (include/blb_rs.h).

There is no CPU fallback: if the HIP library is missing, importing the engine fails loudly.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("BLBRS_LIB_PATH") or os.path.join(HERE, "libblbrs.so")  # override: tuning builds

# Every symbol include/blb_rs.h declares, with its ctypes signature.
_P = ctypes.c_void_p
_SZ = ctypes.c_size_t
_I = ctypes.c_int
SIGNATURES = {
    "blbrs_new": (_I, [_I, _I, ctypes.POINTER(_P)]),
    "blbrs_free": (None, [_P]),
    "blbrs_data_shards": (_I, [_P]),
    "blbrs_parity_shards": (_I, [_P]),
    "blbrs_matrix": (_I, [_P, _P, _SZ]),
    "blbrs_encoder_compiled_network": (_I, [_P]),
    "blbrs_encode": (_I, [_P, _P, _P]),
    "blbrs_verify": (_I, [_P, _P, _P, ctypes.POINTER(_I)]),
    "blbrs_reconstruct": (_I, [_P, _P, _P]),
    "blbrs_reconstruct_data": (_I, [_P, _P, _P]),
    "blbrs_reconstruct_verify": (_I, [_P, _P, _P, ctypes.POINTER(_I)]),
    "blbrs_encode_dev": (_I, [_P, _P, _SZ, _SZ, _SZ, _SZ, _P]),
    "blbrs_encode_dev_ptrs": (_I, [_P, _P, _SZ, _SZ, _P]),
    "blbrs_reconstruct_dev": (_I, [_P, _P, _SZ, _SZ, _SZ, _SZ, _P, _I, _P]),
    "blbrs_reconstruct_dev_ptrs": (_I, [_P, _P, _SZ, _SZ, _P, _I, _P]),
    "blbrs_verify_dev": (_I, [_P, _P, _SZ, _SZ, _SZ, _SZ, _P, _P]),
    "blbrs_verify_dev_ptrs": (_I, [_P, _P, _SZ, _SZ, _P, _P]),
    "blbrs_reconstruct_verify_dev": (_I, [_P, _P, _SZ, _SZ, _SZ, _SZ, _P, _P, _P]),
    "blbrs_encode_host_batch": (_I, [_P, _P, _SZ, _SZ, _I]),
    "blbrs_crc32c_dev": (_I, [_P, _SZ, _SZ, _SZ, _SZ, _P, _P]),
    "blbrs_crc32c": (_I, [_P, _SZ, _SZ, _P]),
    "blbrs_encode_crc_dev": (_I, [_P, _P, _SZ, _SZ, _SZ, _SZ, _SZ, _P, _P]),
    "blbrs_crc32c_dev_at": (_I, [_P, _SZ, _SZ, _SZ, _SZ, _SZ, _P, _P, _P]),
    "blbrs_encode_crc_dev_at": (_I, [_P, _P, _SZ, _SZ, _SZ, _SZ, _SZ, _SZ, _P, _P, _P]),
    "blbrs_reconstruct_crc_dev_at": (_I, [_P, _P, _SZ, _SZ, _SZ, _SZ, _P, _I, _SZ, _SZ, _P, _P, _P]),
    "blbrs_pack_dev": (_I, [_P, _SZ, _SZ, _SZ, _P, _SZ, _P]),
    "blbrs_pack_encode_dev": (_I, [_P, _P, _SZ, _SZ, _SZ, _SZ, _P, _SZ, _P]),
    "blbrs_batcher_new": (_I, [_I, _I, ctypes.POINTER(_P)]),
    "blbrs_batcher_free": (None, [_P]),
    "blbrs_encoder_set_batcher": (_I, [_P, _P]),
    "blbrs_batcher_stats": (_I, [_P, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]),
    "blbrs_new_on": (_I, [_I, _I, _P, _I, ctypes.POINTER(_P)]),
    "blbrs_encoder_devices": (_I, [_P, _P, _I, ctypes.POINTER(_I)]),
    "blbrs_set_default_devices": (_I, [_P, _I]),
    "blbrs_encode_parts": (_I, [_P, _P, _SZ, _SZ]),
    "blbrs_reconstruct_parts": (_I, [_P, _P, _SZ, _SZ, _P, _I]),
    "blbrs_verify_parts": (_I, [_P, _P, _SZ, _SZ, _P]),
    "blbrs_batcher_new_on": (_I, [_I, _I, _P, _I, ctypes.POINTER(_P)]),
    "blbrs_buffer_get": (_I, [_SZ, ctypes.POINTER(_P), ctypes.POINTER(_SZ)]),
    "blbrs_buffer_put": (_I, [_P]),
    "blbrs_pool_set_idle_limit": (_I, [_SZ]),
    "blbrs_buffer_register": (_I, [_P, _SZ]),
    "blbrs_buffer_unregister": (_I, [_P]),
    "blbrs_pool_set_live_limit": (_I, [_SZ]),
    "blbrs_encoder_lane_stats": (_I, [_P, _I, _P]),
    "blbrs_get_pool_stats": (_I, [_P]),
    "blbrs_host_alloc": (_I, [_SZ, ctypes.POINTER(_P)]),
    "blbrs_host_free": (_I, [_P]),
    "blbrs_host_register": (_I, [_P, _SZ]),
    "blbrs_host_unregister": (_I, [_P]),
    "blbrs_set_worker_limit": (_I, [_I]),
    "blbrs_get_device_stats": (_I, [_I, _P]),
    "blbrs_trim": (_I, []),
    "blbrs_plan_stats": (_I, [ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]),
    "blbrs_debug_watch_faults": (_I, []),
    "blbrs_table_fault_take": (_I, [_I, _P, ctypes.POINTER(_I)]),
    "blbrs_debug_corrupt_next_table": (_I, [_I]),
    "blbrs_set_device": (_I, [_I]),
    "blbrs_device_count": (_I, [ctypes.POINTER(_I)]),
    "blbrs_device_numa_node": (_I, [_I, ctypes.POINTER(_I)]),
    "blbrs_set_device_numa_node": (_I, [_I, _I]),
    "blbrs_host_numa_node": (_I, [_P, ctypes.POINTER(_I)]),
    "blbrs_lane_policy": (_I, [_P, _P, _SZ, _SZ, _I, ctypes.POINTER(_SZ)]),
    "blbrs_set_tuning": (_I, [ctypes.c_char_p, ctypes.c_long]),
    "blbrs_get_tuning": (_I, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_long)]),
    "blbrs_rtc_get_stats": (_I, [_P]),
    "blbrs_rtc_compile": (_I, [_I, _I, _P, _I, _I, _P, _SZ, ctypes.POINTER(_SZ)]),
    "blbrs_rtc_wait": (_I, [ctypes.c_long]),
    "blbrs_rtc_network_source": (_I, [_I, _I, _P, _P, _SZ, ctypes.POINTER(_I)]),
    "blbrs_last_error": (ctypes.c_char_p, []),
    "blbrs_version": (ctypes.c_char_p, []),
    "blbrs_strerror": (ctypes.c_char_p, [_I]),
}



class DeviceStats(ctypes.Structure):
    """blbrs_device_stats"""
    _fields_ = [("workers", ctypes.c_uint64), ("idle", ctypes.c_uint64), ("waits", ctypes.c_uint64),
                ("staging_bytes", ctypes.c_uint64), ("calls", ctypes.c_uint64), ("inflight", ctypes.c_int64),
                ("done_waits", ctypes.c_uint64), ("done_fallbacks", ctypes.c_uint64)]


class PoolStats(ctypes.Structure):
    """blbrs_pool_stats"""
    _fields_ = [("gets", ctypes.c_uint64), ("puts", ctypes.c_uint64), ("allocs", ctypes.c_uint64),
                ("frees", ctypes.c_uint64), ("live_bytes", ctypes.c_uint64), ("idle_bytes", ctypes.c_uint64),
                ("registered_bytes", ctypes.c_uint64), ("registrations", ctypes.c_uint64),
                ("live_limit", ctypes.c_uint64), ("limit_rejects", ctypes.c_uint64)]


class LaneStats(ctypes.Structure):
    """blbrs_lane_stats"""
    _fields_ = [("calls", ctypes.c_uint64), ("bytes", ctypes.c_uint64), ("inflight_calls", ctypes.c_int64),
                ("inflight_bytes", ctypes.c_int64)]


class RtcStats(ctypes.Structure):
    """blbrs_rtc_stats"""
    _fields_ = [("requested", ctypes.c_uint64), ("compiled", ctypes.c_uint64), ("loaded", ctypes.c_uint64),
                ("failed", ctypes.c_uint64), ("pending", ctypes.c_uint64), ("compile_ms", ctypes.c_double)]


class TableFault(ctypes.Structure):
    """blbrs_table_fault"""
    _fields_ = [("stripe", ctypes.c_uint32), ("slot", ctypes.c_uint32), ("launch_tag", ctypes.c_uint32),
                ("entry_tag", ctypes.c_uint32), ("address", ctypes.c_uint64)]


class DevPart(ctypes.Structure):
    """blbrs_dev_part"""
    _fields_ = [("stripes", _P), ("shard_stride", _SZ), ("stripe_stride", _SZ), ("batch", _SZ),
                ("stream", _P)]


_lib = None


def _one_hip_runtime() -> None:
    """Make the process's HIP runtime the one torch brings, before libblbrs.so is mapped.

    torch's wheel ships its own libamdhip64 / libhsa-runtime64 (torch/lib, ROCm 7.0) with the
    same SONAMEs as /opt/rocm's (7.2), which libblbrs.so links.  Loaded after torch, the
    library's DT_NEEDED entries resolve to torch's copies: one runtime.  Loaded before torch,
    /opt/rocm's copies are mapped first, torch then maps its own by path, and the process holds
    two HIP and two HSA runtimes over one /dev/kfd (seen: the second one finds no device).  So
    import torch first when it is installed; C / C++ / Go callers are not affected (one runtime,
    /opt/rocm's).  BLBRS_NO_TORCH=1: a ctypes-only process that never imports torch (it then
    runs on /opt/rocm's runtime alone)."""
    if os.environ.get("BLBRS_NO_TORCH") == "1":
        return
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def load() -> ctypes.CDLL:
    """Load libblbrs.so (built by `make -C blb_amd` / __graft_entry__.build())."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"blb_amd: HIP engine library not built ({LIB_PATH} missing); run "
                "`python -c 'import __graft_entry__ as g; g.build()'` or `make -C blb_amd`")
        _one_hip_runtime()
        lib = ctypes.CDLL(LIB_PATH)
        # An older build loaded through $BLBRS_LIB_PATH for an A/B run (tools/) may lack the
        # newest entry points; the shipped library must export them all (tests/test_capi.py).
        lenient = "BLBRS_LIB_PATH" in os.environ
        for name, (res, args) in SIGNATURES.items():
            if lenient and not hasattr(lib, name):
                continue
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib
