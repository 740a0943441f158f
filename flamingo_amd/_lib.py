"""ctypes binding of libflamingo_hip.so (include/flamingo_hip.h).

There is no fallback: if the library is missing or cannot load, importing the
engine raises.  The product path never computes on the CPU.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# FLM_LIB_PATH: load another build of the same sources (tools/sanitize.sh's ASan/UBSan host build)
LIB_PATH = os.environ.get("FLM_LIB_PATH") or os.path.join(HERE, "lib", "libflamingo_hip.so")

_u8p = ctypes.POINTER(ctypes.c_uint8)
_i8p = ctypes.POINTER(ctypes.c_int8)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_i64p = ctypes.POINTER(ctypes.c_int64)
_vp = ctypes.c_void_p
_sz = ctypes.c_size_t
_u64 = ctypes.c_uint64
_int = ctypes.c_int

# name -> (restype, argtypes); every symbol declared in include/flamingo_hip.h
SIGNATURES = {
    "flm_device_count": (_int, []),
    "flm_init": (_int, [ctypes.POINTER(_vp), _int]),
    "flm_free": (None, [_vp]),
    "flm_last_error": (ctypes.c_char_p, [_vp]),
    "flm_version": (ctypes.c_char_p, []),
    "flm_ctx_stream": (_vp, [_vp]),
    "flm_aggregate_unmask": (_int, [_vp, ctypes.POINTER(_u32p), _int, _u8p, _i8p, _int, _sz, _u32p]),
    "flm_client_mask": (_int, [_vp, _u32p, _int, _i64p, _u8p, _i8p, _sz, _u32p]),
    "flm_prg_expand": (_int, [_vp, _u8p, _int, _sz, _u64, _u32p]),
    "flm_mask_accumulate": (_int, [_vp, _u8p, _i8p, _int, _u32p, _sz, _u64]),
    "flm_chacha20_xor": (_int, [_vp, _u8p, _u8p, _u64, _u8p, _u8p, _sz]),
    "flm_aggregate_unmask_dev": (_int, [_vp, _vp, _sz, _int, _vp, _vp, _int, _sz, _sz, _sz, _u64, _vp, _vp]),
    "flm_seed_table_dev": (_int, [_vp, _vp, _vp, _int, _vp]),
    "flm_aggregate_dev": (_int, [_vp, _vp, _sz, _int, _int, _sz, _sz, _sz, _u64, _vp, _vp]),
    "flm_client_mask_dev": (_int, [_vp, _vp, _sz, _int, _i64p, _vp, _i8p, _sz, _vp, _vp]),
    "flm_prg_expand_dev": (_int, [_vp, _vp, _int, _sz, _u64, _vp, _sz, _vp]),
    "flm_check_signs": (_int, [_vp, ctypes.POINTER(_int)]),
    "flm_last_plan": (_int, [_vp, ctypes.POINTER(_int), ctypes.POINTER(_int), ctypes.POINTER(_int),
                             ctypes.POINTER(_int)]),
    "flm_set_tuning": (_int, [_vp, ctypes.c_char_p, _int]),
    "flm_get_tuning": (_int, [_vp, ctypes.c_char_p, ctypes.POINTER(_int)]),
    "flm_plan_aggregate": (_int, [_int, _int, _sz, _int, _int, _sz, _sz, _sz, _u64, _vp, _int,
                                  ctypes.POINTER(_int), ctypes.POINTER(_int)]),
    "flm_ec_combine": (_int, [_vp, _u8p, _u8p, _u8p, _int, _int, _int, _u8p, _u8p, _u32p]),
    "flm_ec_combine_dev": (_int, [_vp, _vp, _vp, _vp, _int, _int, _int, _vp, _vp, _vp, _vp]),
    "flm_ec_mul": (_int, [_vp, _u8p, _u8p, _int, _u8p, _u32p]),
    "flm_hash_to_curve": (_int, [_vp, _u8p, _u32p, _int, _u8p, _u32p]),
    "flm_hash_to_curve_decimal": (_int, [_vp, ctypes.c_uint32, _int, _u8p, _u32p]),
    "flm_hash_to_curve_decimal_dev": (_int, [_vp, ctypes.c_uint32, _int, _vp, _vp, _vp]),
    "flm_shamir_combine": (_int, [_vp, _u8p, _u8p, _int, _int, _u8p]),
    "flm_shamir_combine_dev": (_int, [_vp, _vp, _vp, _int, _int, _vp, _vp]),
    "flm_pair_units_dev": (_int, [_vp, _vp, _vp, _int, _vp, _vp, _vp, _sz, _vp, _int, _int, _vp]),
    "flm_flag_set_dev": (_int, [_vp, _vp, _vp]),
    "flm_cu_count": (_int, [_vp, _vp]),
    "flm_stream_create_cu_mask": (_int, [_vp, _vp, _int, _vp]),
    "flm_stream_destroy": (_int, [_vp, _vp]),
    "flm_shard_bounds": (_int, [_sz, _int, _int, ctypes.POINTER(_sz), ctypes.POINTER(_sz), ctypes.POINTER(_sz)]),
    "flm_client_bounds": (_int, [_int, _int, _int, ctypes.POINTER(_int), ctypes.POINTER(_int)]),
    "flm_rccl_available": (_int, []),
    "flm_comm_unique_id": (_int, [_vp]),
    "flm_comm_init_rank": (_int, [_vp, _int, _int, _vp]),
    "flm_comm_size": (_int, [_vp, ctypes.POINTER(_int), ctypes.POINTER(_int)]),
    "flm_comm_destroy": (_int, [_vp]),
    "flm_reduce_scatter_dev": (_int, [_vp, _vp, _vp, _sz, _vp]),
    "flm_all_gather_dev": (_int, [_vp, _vp, _vp, _sz, _vp]),
    "flm_group_init": (_int, [ctypes.POINTER(_vp), _int, ctypes.POINTER(_int)]),
    "flm_group_free": (None, [_vp]),
    "flm_group_last_error": (ctypes.c_char_p, [_vp]),
    "flm_group_size": (_int, [_vp]),
    "flm_group_is_loopback": (_int, [_vp]),
    "flm_group_init_flags": (_int, [ctypes.POINTER(_vp), _int, ctypes.POINTER(_int), ctypes.c_uint]),
    "flm_group_has_rccl": (_int, [_vp]),
    "flm_group_ctx": (_vp, [_vp, _int]),
    "flm_group_sync": (_int, [_vp]),
    "flm_group_aggregate_unmask": (_int, [_vp, ctypes.POINTER(_u32p), _int, _u8p, _i8p, _int, _sz, _u32p]),
    "flm_group_aggregate_unmask_dev": (_int, [_vp, ctypes.POINTER(_vp), _sz, ctypes.POINTER(_int),
                                              ctypes.POINTER(_vp), ctypes.POINTER(_vp), _int, _sz,
                                              ctypes.POINTER(_vp)]),
    "flm_store_create": (_int, [ctypes.POINTER(_vp), _vp, _vp, _sz, _int]),
    "flm_store_free": (None, [_vp]),
    "flm_store_last_error": (ctypes.c_char_p, [_vp]),
    "flm_store_count": (_int, [_vp]),
    "flm_store_add": (_int, [_vp, ctypes.c_int64, _vp, _sz]),
    "flm_store_partial": (_int, [_vp]),
    "flm_store_partial_wait": (_int, [_vp, ctypes.POINTER(ctypes.c_float)]),
    "flm_store_partial_host": (_int, [_vp, _u32p]),
    "flm_store_unmask": (_int, [_vp, _u8p, _i8p, _int, _u32p]),
    "flm_store_unmask_ms": (_int, [_vp, ctypes.POINTER(ctypes.c_float)]),
    "flm_store_reset": (_int, [_vp]),
    "flm_host_alloc": (_vp, [_sz]),
    "flm_host_free": (None, [_vp]),
}

_lib = None


def load(path: str = LIB_PATH):
    """Load the HIP library (raises OSError/RuntimeError if it is missing)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(
            f"libflamingo_hip.so not found at {path}: build it with `python -m flamingo_amd.build` "
            "(hipcc --offload-arch=gfx950); there is no CPU fallback")
    # One HIP runtime per process: torch ships its own libamdhip64.so.7 (same
    # soname as /opt/rocm's).  Whichever loads first is used by both, and torch
    # only initialises on its own, so let torch load it first when present.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def p_u8(a):
    return a.ctypes.data_as(_u8p)


def p_i8(a):
    return a.ctypes.data_as(_i8p)


def p_u32(a):
    return a.ctypes.data_as(_u32p)


def p_i64(a):
    return a.ctypes.data_as(_i64p)
