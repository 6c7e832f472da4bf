"""ctypes binding of libjylis_gpu.so (include/jylis_gpu.h).

The product path has no CPU fallback: if the HIP library is missing or no
GPU is present, loading fails loudly.
"""
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# JY_LIB: an alternative build of the same library (kernel A/B experiments)
LIB_PATH = os.environ.get("JY_LIB") or os.path.join(_HERE, "libjylis_gpu.so")

JY_OK, JY_EINVAL, JY_ENOMEM, JY_EHIP, JY_ERANGE, JY_ETYPE = 0, -1, -2, -3, -4, -5
JY_NO_SLOT = 0xFFFFFFFF
GCOUNT, PNCOUNT, TREG, TLOG, UJSON = 0, 1, 2, 3, 4
TYPE_NAMES = {"GCOUNT": GCOUNT, "PNCOUNT": PNCOUNT, "TREG": TREG, "TLOG": TLOG, "UJSON": UJSON}
HOST, DEVICE = 0, 1
CFG_TREG_WHOLE_LINES = 1
CFG_TREG_DUP_TEST = 2
TLOG_INS, TLOG_TRIMAT, TLOG_TRIM, TLOG_CLR = 0, 1, 2, 3
UJSON_INS, UJSON_RM, UJSON_CLR = 0, 1, 2


class JyConfig(C.Structure):
    _fields_ = [
        ("device", C.c_int32),
        ("counter_columns", C.c_uint32),
        ("ujson_columns", C.c_uint32),
        ("flags", C.c_uint32),
        ("key_capacity", C.c_uint64 * 5),
        ("entry_capacity", C.c_uint64 * 5),
        ("arena_capacity", C.c_uint64 * 5),
    ]


NODE_MAX_SHARDS = 64
FABRIC_RCCL, FABRIC_COPY = 0, 1


class JyNodeConfig(C.Structure):
    _fields_ = [
        ("nshards", C.c_uint32),
        ("nlocal", C.c_uint32),
        ("rank0", C.c_uint32),
        ("fabric", C.c_uint32),
        ("devices", C.c_int32 * NODE_MAX_SHARDS),
        ("unique_id", C.c_uint8 * 128),
        ("engine", JyConfig),
    ]


P = C.c_void_p
U64 = C.c_uint64
U32 = C.c_uint32
I32 = C.c_int32

# name -> (restype, argtypes); every symbol include/jylis_gpu.h declares
SIGNATURES = {
    "jy_config_default": (None, [P]),
    "jy_engine_create": (I32, [P, P]),
    "jy_engine_destroy": (None, [P]),
    "jy_last_error": (C.c_char_p, [P]),
    "jy_skipped": (U64, [P]),
    "jy_set_stream": (I32, [P, P]),
    "jy_get_stream": (P, [P]),
    "jy_sync": (I32, [P]),
    "jy_timing_enable": (I32, [P, I32]),
    "jy_timing_read": (I32, [P, U64, P, P]),
    "jy_replica_col": (I32, [P, U64, P]),
    "jy_replica_id": (I32, [P, U32, P]),
    "jy_replica_count": (U32, [P]),
    "jy_keys_intern": (I32, [P, I32, U64, P, P, P]),
    "jy_keys_lookup": (I32, [P, I32, U64, P, P, P]),
    "jy_keys_intern_mem": (I32, [P, I32, U64, P, P, P, I32]),
    "jy_keys_lookup_mem": (I32, [P, I32, U64, P, P, P, I32]),
    "jy_keys_count": (U64, [P, I32]),
    "jy_keys_reserve": (I32, [P, I32, U64]),
    "jy_keys_export": (I32, [P, I32, U64, U64, P, P, U64]),
    "jy_key_owner": (U32, [P, U64, U32]),
    "jy_values_pack": (I32, [P, I32, U64, P, P, P, P]),
    "jy_gcount_converge": (I32, [P, U64, P, P, P, I32]),
    "jy_gcount_converge_block": (I32, [P, U32, P, U32, U32, P, I32]),
    "jy_gcount_get": (I32, [P, U64, P, P, I32]),
    "jy_pncount_converge": (I32, [P, U64, P, P, P, U64, P, P, P, I32]),
    "jy_pncount_converge_block": (I32, [P, U32, P, U32, U32, P, P, I32]),
    "jy_pncount_get": (I32, [P, U64, P, P, I32]),
    "jy_counter_converge_keys": (I32, [P, I32, U64, P, P, U64, P, P, P, P, I32]),
    "jy_counter_export": (I32, [P, I32, U32, U32, U32, P]),
    "jy_counter_write": (I32, [P, I32, I32, U32, U64, P, P, I32]),
    "jy_counter_deltas_size": (I32, [P, I32, P]),
    "jy_counter_flush": (I32, [P, I32, U64, P, P, P, P, I32]),
    "jy_treg_converge": (I32, [P, U64, P, P, P, P, I32]),
    "jy_treg_converge_block": (I32, [P, U32, U64, P, P, P, I32]),
    "jy_treg_read": (I32, [P, U64, P, P, P, P]),
    "jy_treg_set": (I32, [P, U64, P, P, P, P, I32]),
    "jy_treg_deltas_size": (I32, [P, P]),
    "jy_treg_flush": (I32, [P, U64, P, P, P, P, P, I32]),
    "jy_arena_read": (I32, [P, I32, U64, U64, P]),
    "jy_tlog_converge": (I32, [P, U64, P, P, P, U64, P, P, P, I32]),
    "jy_tlog_read_sizes": (I32, [P, U64, P, P, P]),
    "jy_tlog_read": (I32, [P, U64, P, P, P, P, P]),
    "jy_ujson_converge": (I32, [P, U64, P, P, U64, P, P, P, U64, P, P, U64, P, I32]),
    "jy_ujson_read_sizes": (I32, [P, U64, P, P, P]),
    "jy_ujson_read": (I32, [P, U64, P, P, P, P, P, P, P]),
    "jy_ujson_stats": (I32, [P, P]),
    "jy_ujson_stats_ext": (I32, [P, P]),
    "jy_ujson_set_inplace": (I32, [P, U32]),
    "jy_tlog_stats": (I32, [P, P]),
    "jy_arena_usage": (I32, [P, I32, P, P]),
    "jy_arena_collect": (I32, [P, I32, P]),
    "jy_tlog_write": (I32, [P, U64, P, P, P, P, P, P, I32]),
    "jy_ujson_write": (I32, [P, U64, P, P, P, U32, I32]),
    "jy_ujson_deltas_size": (I32, [P, P]),
    "jy_ujson_flush": (I32, [P, U64, U64, U64, P, P, P, P, P, P, P, P, P, P, I32]),
    "jy_tlog_deltas_size": (I32, [P, P]),
    "jy_tlog_flush": (I32, [P, U64, U64, P, P, P, P, P, P, P, P, I32]),
    "jy_keys_owner": (None, [U64, P, P, U32, P]),
    "jy_keys_route_part": (I32, [P, U64, P, P, U32, P, P, P, P, P]),
    "jy_keys_intern_lens": (I32, [P, I32, U64, P, P, P]),
    "jy_keys_route_back": (I32, [P, U64, P, P, P]),
    "jy_treg_route_part": (I32, [P, U64, P, P, P, P, P, U32, U64, U64, I32, P, P, P, P]),
    "jy_treg_route_part_self": (I32, [P, U64, P, P, P, P, P, U32, U32, U64, U64, I32, P, P, P, P]),
    "jy_treg_converge_routed": (I32, [P, U32, U64, U64, P, P, P]),
    "jy_arena_reserve": (I32, [P, I32, U64, P, P]),
    "jy_treg_converge_routed_at": (I32, [P, U32, U64, U64, P, P, U64]),
    "jy_route_words": (U64, [I32, U64, P]),
    "jy_tlog_route_part": (I32, [P, U64, P, P, P, P, U64, P, P, P, U32, U64, U64, U64, U64, I32, P, P, P, P]),
    "jy_tlog_converge_routed": (I32, [P, U32, U64, U64, U64, P, P]),
    "jy_ujson_route_part": (I32, [P, U64, P, P, P, U64, P, P, P, U64, P, P, U64, P, U32, U64, U64, U64, U64, U64,
                                  I32, P, P, P]),
    "jy_ujson_converge_routed": (I32, [P, U32, U64, U64, U64, U64, P]),
    "jy_node_unique_id": (I32, [P]),
    "jy_node_create": (I32, [P, P]),
    "jy_node_create_local": (I32, [U32, P, U32, P, P]),
    "jy_device_count": (I32, []),
    "jy_node_acquire_local": (I32, [P, P]),
    "jy_node_release": (None, [P]),
    "jy_node_destroy": (None, [P]),
    "jy_node_last_error": (C.c_char_p, [P]),
    "jy_node_nshards": (U32, [P]),
    "jy_node_engine": (P, [P, U32]),
    "jy_node_shard_of": (U32, [P, P, U64]),
    "jy_node_replica_col": (I32, [P, U64, P]),
    "jy_node_sync": (I32, [P]),
    "jy_node_fence": (I32, [P]),
    "jy_node_lock": (I32, [P]),
    "jy_node_unlock": (None, [P]),
    "jy_node_lock_type": (I32, [P, I32]),
    "jy_node_pending": (I32, [P, I32, P]),
    "jy_node_arena_gc": (I32, [P, U32]),
    "jy_node_exchange_plan": (I32, [U32, U32, U32, U32, P, P, P, P, U64, P, P]),
    "jy_node_counter_converge": (I32, [P, I32, U64, P, P, P, P, P, P, I32]),
    "jy_node_treg_converge": (I32, [P, U64, P, P, P, P, P, I32]),
    "jy_node_tlog_converge": (I32, [P, U64, P, P, P, P, P, P, P, I32]),
    "jy_node_ujson_converge": (I32, [P, U64, P, P, P, P, P, P, P, P, P, I32]),
    "jy_node_counter_converge_block": (I32, [P, I32, U32, P, U32, U32, P, P]),
    "jy_node_stats": (I32, [P, P]),
}

# include/jylis_host.h: the C++ host mirror (Database / RepoManagerCore / Repo*)
HOST_SIGNATURES = {
    "jyh_db_create": (I32, [I32, U64, P]),
    "jyh_db_destroy": (None, [P]),
    "jyh_db_error": (C.c_char_p, [P]),
    "jyh_db_apply": (I32, [P, U32, P, P, P, U64, P]),
    "jyh_db_flush": (I32, [P, P, P]),
    "jyh_db_converge": (I32, [P, P, U64]),
    "jyh_db_shutdown": (I32, [P]),
    "jyh_free": (None, [P]),
}

_lib = None


def load(path=LIB_PATH):
    """Load the engine library (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(
            f"{path} is missing: build it with `make -C jylis_amd` (hipcc, gfx950); "
            "there is no CPU fallback for the converge path")
    # PyTorch-ROCm ships its own libamdhip64 / libhsa-runtime64 under the same
    # sonames as /opt/rocm.  Whichever loads first serves the whole process;
    # if the engine's copy initialises first, torch sees no GPU.  Load torch's
    # runtime first (when torch is installed) so the engine and torch share
    # one HIP runtime and device pointers pass between them.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(path)
    for name, (res, args) in list(SIGNATURES.items()) + list(HOST_SIGNATURES.items()):
        fn = getattr(lib, name, None)
        if fn is None:
            if path == os.path.join(_HERE, "libjylis_gpu.so"):
                raise RuntimeError(f"{path} does not export {name}: rebuild it (make -C jylis_amd)")
            continue  # an older A/B build (JY_LIB) without a newer entry point
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib
