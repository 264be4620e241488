"""ctypes binding of libkhmer_hip.so (include/khmer_hip.h).

The product path has no CPU fallback: if the HIP library is missing this module
raises ImportError, and graph construction raises RuntimeError when no HIP
device is visible.
"""
import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("KHMER_AMD_LIB") or os.path.join(_HERE, "libkhmer_hip.so")   # override: development builds

KH_OK, KH_EVALUE, KH_EFILE, KH_EATTR, KH_ENOMEM, KH_EDEVICE, KH_ERUNTIME, KH_END = range(8)
STORAGE_BYTE, STORAGE_BIT, STORAGE_NIBBLE = 1, 2, 7
HASH_TWOBIT, HASH_MURMUR = 0, 1
GROUP_BROADCAST, GROUP_EXCHANGE, GROUP_DELTA = 0, 1, 2   # include/khmer_hip.h KH_GROUP_*
GROUP_MODES = {"broadcast": GROUP_BROADCAST, "exchange": GROUP_EXCHANGE, "delta": GROUP_DELTA}

if not os.path.exists(LIB_PATH):
    raise ImportError("khmer_amd: %s is not built; run `make -C khmer_amd/csrc` "
                      "(or __graft_entry__.build())" % LIB_PATH)

lib = ctypes.CDLL(LIB_PATH)

u64, u32, i32, sz = ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int, ctypes.c_size_t
P = ctypes.c_void_p
PU64 = ctypes.POINTER(u64)
PU32 = ctypes.POINTER(u32)
PI = ctypes.POINTER(i32)
PCHAR = ctypes.POINTER(ctypes.c_char_p)
PSZ = ctypes.POINTER(sz)

SIGNATURES = {
    "kh_last_error": (ctypes.c_char_p, []),
    "kh_abi_version": (i32, []),
    "kh_device_count": (i32, [PI]),
    "kh_hash_twobit": (i32, [ctypes.c_char_p, i32, PU64, PU64, PU64]),
    "kh_reverse_hash": (i32, [u64, i32, ctypes.c_char_p]),
    "kh_hash_murmur": (i32, [ctypes.c_char_p, i32, PU64, PU64]),
    "kh_reverse_complement": (i32, [ctypes.c_char_p, sz, ctypes.c_char_p]),
    "kh_kmer_hashes": (i32, [i32, i32, ctypes.c_char_p, sz, PU64, PU64]),
    "kh_is_prime": (i32, [u64, PI]),
    "kh_get_n_primes_near_x": (i32, [u32, u64, PU64, PU32]),
    "kh_parser_open": (i32, [ctypes.c_char_p, ctypes.POINTER(P)]),
    "kh_parser_next_read": (i32, [P, PCHAR, PSZ, PCHAR, PSZ, PCHAR, PSZ]),
    "kh_parser_num_reads": (i32, [P, PU64]),
    "kh_parser_is_complete": (i32, [P, PI]),
    "kh_parser_close": (None, [P]),
    "kh_graph_create": (i32, [i32, i32, i32, PU64, i32, i32, ctypes.POINTER(P)]),
    "kh_graph_destroy": (None, [P]),
    "kh_graph_info": (i32, [P, PI, PI, PI, PI]),
    "kh_graph_tablesizes": (i32, [P, PU64]),
    "kh_graph_set_use_bigcount": (i32, [P, i32]),
    "kh_graph_get_use_bigcount": (i32, [P, PI]),
    "kh_graph_n_unique_kmers": (i32, [P, PU64]),
    "kh_graph_n_occupied": (i32, [P, PU64]),
    "kh_graph_set_batch_kmers": (i32, [P, u64]),
    "kh_graph_clear": (i32, [P]),
    "kh_graph_get_bigcounts": (i32, [P, PU64, ctypes.POINTER(ctypes.c_uint16), u64, PU64]),
    "kh_group_unique_id": (i32, [ctypes.c_char_p, sz]),
    "kh_group_create": (i32, [i32, i32, i32, PU64, i32, i32, i32, i32, PI, ctypes.c_char_p, ctypes.POINTER(P)]),
    "kh_group_create_hosted": (i32, [i32, i32, i32, PU64, i32, i32, i32, i32, P, ctypes.POINTER(P)]),
    "kh_group_comm_info": (i32, [P, PI, PI]),
    "kh_group_destroy": (None, [P]),
    "kh_group_shard": (i32, [P, i32, ctypes.POINTER(P)]),
    "kh_group_info": (i32, [P, PI, PI, PI]),
    "kh_group_slice": (i32, [P, i32, i32, PU64, PU64]),
    "kh_group_consume_packed_fixed_device": (i32, [P, ctypes.POINTER(P), u64, u64]),
    "kh_group_counters": (i32, [P, PU64, PU64]),
    "kh_group_wire_stats": (i32, [P, PU64, PU64]),
    "kh_group_consume_bytes_fixed_device": (i32, [P, ctypes.POINTER(P), u64, u64]),
    "kh_group_median_fixed_device": (i32, [P, ctypes.POINTER(P), u64, u64, ctypes.POINTER(P), ctypes.POINTER(P),
                                           ctypes.POINTER(P)]),
    "kh_group_create_mode": (i32, [i32, i32, i32, PU64, i32, i32, i32, i32, PI, ctypes.c_char_p, i32,
                                   ctypes.POINTER(P)]),
    "kh_group_create_hosted_mode": (i32, [i32, i32, i32, PU64, i32, i32, i32, i32, P, i32, ctypes.POINTER(P)]),
    "kh_group_mode": (i32, [P, PI]),
    "kh_group_rank_slice": (i32, [P, i32, i32, PU64, PU64]),
    "kh_consume_parser": (i32, [P, P, i32, PU32, PU64]),
    "kh_consume_parser_filtered": (i32, [P, P, u32, u32, P, u32, i32, PU32, PU64]),
    "kh_consume_seqs": (i32, [P, ctypes.c_char_p, PU64, u64, i32, PU64]),
    "kh_consume_packed_device": (i32, [P, P, P, u64, u64]),
    "kh_consume_packed_fixed_device": (i32, [P, P, u64, u32]),
    "kh_consume_bytes_fixed_device": (i32, [P, P, u64, u32]),
    "kh_median_counts_fixed_device": (i32, [P, P, u64, u32, P, P, P]),
    "kh_add_hashes": (i32, [P, PU64, u64, ctypes.POINTER(ctypes.c_uint8)]),
    "kh_get_counts": (i32, [P, PU64, u64, ctypes.POINTER(ctypes.c_uint16)]),
    "kh_median_counts": (i32, [P, ctypes.c_char_p, PU64, u64, ctypes.POINTER(ctypes.c_uint16),
                               ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float),
                               ctypes.POINTER(ctypes.c_uint8)]),
    "kh_graph_kmer_hashes": (i32, [P, ctypes.c_char_p, PU64, u64, PU64, PU64]),
    "kh_graph_kmer_counts": (i32, [P, ctypes.c_char_p, PU64, u64, ctypes.POINTER(ctypes.c_uint16), PU64]),
    "kh_median_at_least": (i32, [P, ctypes.c_char_p, PU64, u64, u32, ctypes.POINTER(ctypes.c_uint8),
                                 ctypes.POINTER(ctypes.c_uint8)]),
    "kh_abundance_distribution": (i32, [P, P, P, PU64]),
    "kh_graph_table_nbytes": (i32, [P, i32, PU64]),
    "kh_graph_copy_table": (i32, [P, i32, ctypes.c_void_p]),
    "kh_graph_save": (i32, [P, ctypes.c_char_p]),
    "kh_graph_load": (i32, [ctypes.c_char_p, i32, i32, i32, ctypes.POINTER(P)]),
    "kh_file_header": (i32, [ctypes.c_char_p, i32, ctypes.POINTER(ctypes.c_int64)]),
    "kh_graph_n_tags": (i32, [P, PU64]),
    "kh_graph_get_tags": (i32, [P, PU64]),
    "kh_graph_add_tag": (i32, [P, u64]),
    "kh_graph_save_tagset": (i32, [P, ctypes.c_char_p]),
    "kh_graph_load_tagset": (i32, [P, ctypes.c_char_p, i32]),
    "kh_synth_packed_device": (i32, [i32, u64, u64, u64, i32, i32, P, P]),
    "kh_synth_genomic_device": (i32, [i32, u64, u64, u64, u64, i32, i32, P, P]),
    "kh_unpack_ascii_device": (i32, [i32, P, u64, P]),
    "kh_device_malloc": (i32, [i32, u64, ctypes.POINTER(P)]),
    "kh_device_copy": (i32, [i32, P, P, u64]),
    "kh_device_free": (i32, [i32, P]),
    "kh_device_synchronize": (i32, [i32]),
    "kh_graph_set_profiling": (i32, [P, i32]),
    "kh_graph_set_schedule": (i32, [P, i32, i32]),
    "kh_graph_kernel_stats": (i32, [P, ctypes.c_char_p, sz, PSZ]),
}

for _name, (_res, _args) in SIGNATURES.items():
    if os.environ.get("KHMER_AMD_LIB") and not hasattr(lib, _name):
        continue   # an older development build (A/B runs) may lack newer entry points
    _fn = getattr(lib, _name)
    _fn.restype = _res
    _fn.argtypes = _args

_EXC = {
    KH_EVALUE: ValueError,
    KH_EFILE: OSError,
    KH_EATTR: AttributeError,
    KH_ENOMEM: MemoryError,
    KH_EDEVICE: RuntimeError,
    KH_ERUNTIME: ValueError,
}


def last_error():
    return lib.kh_last_error().decode("utf-8", "replace")


def check(rc):
    """Raise the reference's Python exception class for a status code."""
    if rc == KH_OK:
        return rc
    raise _EXC.get(rc, RuntimeError)(last_error())


def device_count():
    n = ctypes.c_int(0)
    lib.kh_device_count(ctypes.byref(n))
    return n.value


_device_lock = threading.Lock()
_default_device = [None]


def default_device():
    """HIP device for new graphs: $KHMER_AMD_DEVICE, else LOCAL_RANK, else 0."""
    with _device_lock:
        if _default_device[0] is None:
            dev = os.environ.get("KHMER_AMD_DEVICE", os.environ.get("LOCAL_RANK", "0"))
            _default_device[0] = int(dev)
        return _default_device[0]


def set_default_device(dev):
    with _device_lock:
        _default_device[0] = int(dev)
