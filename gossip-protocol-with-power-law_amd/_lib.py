"""ctypes binding of libgossip_hip.so (include/gossip_capi.h).

The product path has no CPU fallback: if the HIP library is missing or fails to
load, every engine call raises GossipLibraryError.
"""
import ctypes
import os

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, "_build", "libgossip_hip.so")


class GossipLibraryError(RuntimeError):
    pass


class GossipError(RuntimeError):
    def __init__(self, status, msg):
        super().__init__(f"gossip status {status}: {msg}")
        self.status = status


GP_OK, GP_EINVAL, GP_EHIP, GP_ENOMEM, GP_ESTATE, GP_ERCCL, GP_ENOTRACK = 0, -1, -2, -3, -4, -5, -6

# gp_what
SEEN, FIRST, DIGEST, COVERAGE, FORWARDS, STATE, MISS, DEG_LIVE, ROW_PTR, COL, FRONTIER, FPOP, L2G = range(13)
JOB_DIGEST, JOB_COVERAGE, JOB_FORWARDS = 13, 14, 15   # after gp_shard_combine
# gp_shard_info transports
XPORT_NONE, XPORT_RCCL, XPORT_HOST = 0, 1, 2

# gp_allgather_fn: (user, send, bytes, recv[nranks * bytes]) -> 0 on success
AllGatherFn = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p)


class RoundStats(ctypes.Structure):
    _fields_ = [
        ("round", ctypes.c_int32),
        ("overflow", ctypes.c_int32),
        ("injected", ctypes.c_uint64),
        ("lost", ctypes.c_uint64),
        ("new_bits", ctypes.c_uint64),
        ("receivers", ctypes.c_uint64),
        ("sends", ctypes.c_uint64),
        ("active", ctypes.c_uint64),
        ("crashed", ctypes.c_uint64),
        ("reports", ctypes.c_uint64),
        ("removals", ctypes.c_uint64),
        ("dup_reports", ctypes.c_uint64),
        ("arcs_scanned", ctypes.c_uint64),
        ("rows_gathered", ctypes.c_uint64),
        ("seen_rows_read", ctypes.c_uint64),
        ("rows_written", ctypes.c_uint64),
        ("vertices_visited", ctypes.c_uint64),
        ("atomics", ctypes.c_uint64),
        ("next_arcs", ctypes.c_uint64),
        ("row_bytes", ctypes.c_uint64),
        ("mode", ctypes.c_int32),
        ("scan", ctypes.c_int32),
        ("expand_ms", ctypes.c_double),
        ("exchange_ms", ctypes.c_double),
        ("round_ms", ctypes.c_double),
        ("kernel_ms", ctypes.c_double),
        ("xchg_rows", ctypes.c_uint64),
        ("xchg_bytes", ctypes.c_uint64),
        ("done_nb", ctypes.c_uint64),
        ("lm_rows", ctypes.c_uint64),
        ("aliased", ctypes.c_uint64),
    ]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class Report(ctypes.Structure):
    _fields_ = [("dead", ctypes.c_int32), ("reporter", ctypes.c_int32), ("round", ctypes.c_int32)]


class Config(ctypes.Structure):
    _fields_ = [
        ("track_first", ctypes.c_int32),
        ("track_digest", ctypes.c_int32),
        ("track_msg_forwards", ctypes.c_int32),
        ("churn", ctypes.c_int32),
        ("p_fail", ctypes.c_double),
        ("churn_seed", ctypes.c_uint64),
        ("miss_threshold", ctypes.c_int32),
        ("hub_threshold", ctypes.c_int32),
        ("report_capacity", ctypes.c_int64),
        ("push_ratio", ctypes.c_double),
        ("early_exit", ctypes.c_int32),
        ("arc_mask_permille", ctypes.c_int32),
        ("prefilter_pct", ctypes.c_int32),
        ("compact_rows", ctypes.c_int32),
        ("unfiltered_pct", ctypes.c_int32),
        ("msg_word_base", ctypes.c_int32),
        ("flat_max_words", ctypes.c_int32),
        ("summary_min_n", ctypes.c_int64),
        ("partition_by_arcs", ctypes.c_int32),
        ("split_deg", ctypes.c_int32),
        ("split_max_permille", ctypes.c_int32),
    ]


# name -> (restype, argtypes): every symbol include/gossip_capi.h declares
_P = ctypes.c_void_p
_I32, _I64, _U64, _D = ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_double
_PI32, _PI64 = ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int64)
SIGNATURES = {
    "gp_abi_version": (ctypes.c_int, []),
    "gp_last_error": (ctypes.c_char_p, []),
    "gp_device_count": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
    "gp_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(_P)]),
    "gp_destroy": (None, [_P]),
    "gp_default_config": (None, [ctypes.POINTER(Config)]),
    "gp_configure": (ctypes.c_int, [_P, ctypes.POINTER(Config)]),
    "gp_load_graph": (ctypes.c_int, [_P, _I64, _I64, _P, _P, _I32, _P, _P]),
    "gp_build_chung_lu": (ctypes.c_int, [_P, _I64, _D, _D, _U64]),
    "gp_set_partition": (ctypes.c_int, [_P, _I32, _I32]),
    "gp_get_partition": (ctypes.c_int, [_P, _PI64, _PI64]),
    "gp_comm_unique_id": (ctypes.c_int, [_P]),
    "gp_comm_init": (ctypes.c_int, [_P, _P, _I32, _I32]),
    "gp_set_messages": (ctypes.c_int, [_P, _I32, _P, _P]),
    "gp_spread_keys": (ctypes.c_int, [_P, _I32, _I32, _P, _P]),
    "gp_crash": (ctypes.c_int, [_P, _I32, _P]),
    "gp_reset": (ctypes.c_int, [_P]),
    "gp_round": (ctypes.c_int, [_P, ctypes.POINTER(RoundStats)]),
    "gp_run": (ctypes.c_int, [_P, _I32, ctypes.POINTER(RoundStats), _PI32]),
    "gp_round_group": (ctypes.c_int, [ctypes.POINTER(_P), _I32, ctypes.POINTER(RoundStats)]),
    "gp_finalize_messages": (ctypes.c_int, [_P]),
    "gp_read": (ctypes.c_int, [_P, _I32, _P, _I64]),
    "gp_reports": (ctypes.c_int, [_P, ctypes.POINTER(Report), _I64, _PI64]),
    "gp_synchronize": (ctypes.c_int, [_P]),
    "gp_info": (ctypes.c_int, [_P, _PI64, _PI64, _PI32, _PI32]),
    "gp_local_info": (ctypes.c_int, [_P, _PI64, _PI64, _PI64, _PI64, _PI64]),
    "gp_shard_comm_init": (ctypes.c_int, [_P, _P, _I32, _I32]),
    "gp_shard_host_init": (ctypes.c_int, [_P, AllGatherFn, _P, _I32, _I32]),
    "gp_shard_info": (ctypes.c_int, [_P, _PI32, _PI32, _PI32]),
    "gp_shard_combine": (ctypes.c_int, [_P, ctypes.POINTER(RoundStats), _I32, _PI32, ctypes.POINTER(ctypes.c_double)]),
    "gp_checkpoint_size": (ctypes.c_int, [_P, _PI64]),
    "gp_checkpoint_save": (ctypes.c_int, [_P, _P, _I64]),
    "gp_checkpoint_load": (ctypes.c_int, [_P, _P, _I64]),
}

ABI_VERSION = 18   # include/gossip_capi.h GP_ABI_VERSION (struct layouts below)
_lib = None


def load(path=None):
    """Load (once) and type the HIP library; raise loudly if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get("GOSSIP_HIP_LIB", LIB_PATH)
    if not os.path.exists(path):
        raise GossipLibraryError(
            f"libgossip_hip.so not found at {path}; run __graft_entry__.build() "
            "(the engine has no CPU fallback)")
    try:
        # RTLD_LOCAL: the C-ABI is reached through ctypes only; nothing else in
        # the process binds to the library's (or its HIP runtime's) symbols.
        lib = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
    except OSError as e:
        raise GossipLibraryError(f"failed to load {path}: {e}") from e
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.gp_abi_version() != ABI_VERSION:
        raise GossipLibraryError(f"{path}: ABI {lib.gp_abi_version()} != expected {ABI_VERSION}; rebuild it")
    _lib = lib
    return lib


def check(status):
    if status != GP_OK:
        msg = load().gp_last_error()
        raise GossipError(status, msg.decode() if msg else "")
    return status


def device_count():
    n = ctypes.c_int(0)
    check(load().gp_device_count(ctypes.byref(n)))
    return n.value
