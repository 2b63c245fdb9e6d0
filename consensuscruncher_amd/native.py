"""ctypes bindings for libccio.so (host BAM I/O) and libccamd.so (HIP engine).

The libraries are built in-tree by ``__graft_entry__.build()`` into
``consensuscruncher_amd/lib/``.  Loading fails loudly: there is no CPU fallback
for the GPU engine (tests and bench rely on that).
"""
import ctypes as C
import os

import numpy as np

LIBDIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib")

CC_E = {
    -1: "CC_E_INVALID", -2: "CC_E_HIP", -3: "CC_E_N_HIGHQ", -4: "CC_E_BAD_BASE", -5: "CC_E_SHORT_READ",
    -6: "CC_E_NO_QUAL", -7: "CC_E_NO_CIGAR", -8: "CC_E_DUP_QNAME", -9: "CC_E_AMBIGUOUS",
    -10: "CC_E_COLLISION", -11: "CC_E_UNSUPPORTED", -12: "CC_E_KEYERROR",
    -13: "CC_E_REPLAY",
}
CC_E_N_HIGHQ = -3
CC_E_COLLISION = -10
CC_E_KEYERROR = -12
CC_E_REPLAY = -13

CNT = dict(COUNTER=0, UNMAPPED=1, UNMAPPED_MATE=2, MULTIPLE_MAPPING=3, BAD_SPACER=4, PAIRS=5, READ_ENDS=6,
           FAMILIES=7, ENTRIES=8, UNPAIRED=9, ORPHAN_TAGS=10, DROPPED=11, BAD_LISTED=12, FOREIGN=13)
NUM_COUNTERS = 16
REGION_MOVED = 1 << 30   # CC_REGION_MOVED: a stream entry moved to another shard (cc_read_bam)

OUT_RAW, OUT_RENAME, OUT_NEW = 0, 1, 2
W_SORT, W_INDEX, W_ASYNC = 1, 2, 4   # ccio writer flags (CCIO_W_SORT, CCIO_W_INDEX, CCIO_W_ASYNC)

RF_BAD_SPACER, RF_QUAL_MISSING, RF_RG_UNSUPPORTED = 1, 2, 4


class CCError(RuntimeError):
    def __init__(self, code, msg):
        RuntimeError.__init__(self, "%s (%d): %s" % (CC_E.get(code, "CC_E?"), code, msg))
        self.code = code


P = C.c_void_p
i32p = C.POINTER(C.c_int32)
i64p = C.POINTER(C.c_int64)


class cc_records(C.Structure):
    _fields_ = [("n", C.c_int64),
                ("tid", P), ("pos", P), ("mtid", P), ("mpos", P), ("tlen", P),
                ("flag", P), ("mapq", P),
                ("cigar_id", P), ("qlen", P), ("lseq", P), ("bc_id", P), ("rg_id", P),
                ("rflags", P),
                ("qn_off", P), ("qn_len", P), ("qn_blob", P), ("qn_blob_bytes", C.c_uint64),
                ("pay_off", P), ("payload", P), ("payload_bytes", C.c_uint64), ("rdig", P)]


class cc_out_spec(C.Structure):
    _fields_ = [("kind", C.c_int32), ("src_file", C.c_int32), ("src_rec", C.c_int64), ("name_id", C.c_int64),
                ("flag", C.c_int32), ("mapq", C.c_int32), ("tlen", C.c_int32), ("rg_id", C.c_int32),
                ("cons_off", C.c_int64), ("cons_len", C.c_int32), ("pad", C.c_int32)]


OUT_SPEC_DTYPE = np.dtype([("kind", "<i4"), ("src_file", "<i4"), ("src_rec", "<i8"), ("name_id", "<i8"),
                           ("flag", "<i4"), ("mapq", "<i4"), ("tlen", "<i4"), ("rg_id", "<i4"),
                           ("cons_off", "<i8"), ("cons_len", "<i4"), ("pad", "<i4")], align=True)
assert OUT_SPEC_DTYPE.itemsize == C.sizeof(cc_out_spec)


class cc_read_bam_params(C.Structure):
    _fields_ = [("delim_filter", C.c_int32), ("badread_file", C.c_int32), ("scope_by_run", C.c_int32),
                ("coord_sorted", C.c_int32), ("seed", C.c_uint64)]


_io = None
_amd = None

IO_SIGS = {
    "ccio_last_error": (C.c_char_p, []),
    "ccio_flush": (C.c_int, []),
    "ccio_value_census": (C.c_int, [P, C.c_int64, C.c_int32, P, P]),
    "ccio_interner_new": (P, []),
    "ccio_interner_free": (None, [P]),
    "ccio_interner_size": (C.c_int64, [P, C.c_int]),
    "ccio_interner_get": (C.c_int, [P, C.c_int, C.c_int64, C.c_char_p, C.c_int]),
    "ccio_interner_intern": (C.c_int32, [P, C.c_int, C.c_char_p]),
    "ccio_interner_swap_table": (C.c_int64, [P, P, C.c_int64]),
    "ccio_bam_open": (P, [C.c_char_p, C.c_int]),
    "ccio_bam_close": (None, [P]),
    "ccio_bam_nrec": (C.c_int64, [P]),
    "ccio_bam_nref": (C.c_int32, [P]),
    "ccio_bam_ref": (C.c_int, [P, C.c_int32, C.c_char_p, C.c_int, i32p]),
    "ccio_bam_qname": (C.c_int, [P, C.c_int64, C.c_char_p, C.c_int]),
    "ccio_bam_layout": (C.c_int, [P, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), i32p, C.c_int]),
    "ccio_bam_decode": (C.c_int, [P, P, C.c_int, C.c_char_p, C.POINTER(cc_records), C.c_int]),
    "ccio_format_csn_names": (C.c_int64, [P, C.c_int64, P, P, P, C.c_int64, P]),
    "ccio_dcs_name": (C.c_int, [C.c_char_p, C.c_char_p, C.c_char_p, C.c_int]),
    "ccio_duplex_tag": (C.c_int, [C.c_char_p, C.c_char_p, C.c_int]),
    "ccio_format_dcs_names": (C.c_int64, [P, C.c_int64, P, P, P, C.c_int64, P]),
    "ccio_write_bam": (C.c_int, [C.c_char_p, P, P, C.c_int64, P, P, C.c_int, P, P, P, P, C.c_int, C.c_int]),
    "ccio_sort_bam": (C.c_int, [C.c_char_p, C.c_char_p, C.c_int, C.c_int]),
    "ccio_merge_bams": (C.c_int, [C.c_char_p, P, C.c_int, C.c_int, C.c_int]),
    "ccio_write_bam_ex": (C.c_int, [C.c_char_p, P, P, C.c_int64, P, P, C.c_int, P, P, P, P, C.c_int, C.c_int, C.c_int,
                                    C.POINTER(P)]),
    "ccio_sort_bam_ex": (C.c_int, [C.c_char_p, C.c_char_p, C.c_int, C.c_int, C.c_int]),
    "ccio_merge_handles": (C.c_int, [C.c_char_p, P, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(P)]),
    "ccio_concat_bams": (C.c_int, [C.c_char_p, P, C.c_int, C.c_int, C.c_int]),
    "ccio_index_bam": (C.c_int, [C.c_char_p]),
    "ccio_extract_barcodes": (C.c_int, [C.c_char_p, C.c_char_p, C.c_char_p, C.c_char_p, P, C.c_int32, C.c_int, P, P,
                                        P, P]),
    "ccio_fq_open": (P, [C.c_char_p, C.c_char_p, C.c_int32, C.c_int]),
    "ccio_fq_close": (None, [P]),
    "ccio_fq_info": (C.c_int, [P, i64p, i32p]),
    "ccio_fq_heads": (C.c_int, [P, C.c_int32, P, P, P, P]),
    "ccio_fq_write": (C.c_int, [P, C.c_char_p, C.c_int, P, P, C.c_int32, P, P, P, P, P, C.c_int32, C.c_int]),
    "ccio_bam_open_regions": (P, [C.c_char_p, C.c_int32, P, P, P, C.c_int]),
    "ccio_bam_cores": (C.c_int, [P, P, P, P, P, P]),
    "ccio_bam_pack": (C.c_int64, [P, C.c_int64, P, P, C.c_int64]),
    "ccio_bam_combine": (P, [P, P, C.c_int32, P, P, C.c_int32, C.c_int, C.c_int]),
    "ccio_bam_origin": (C.c_int, [P, P]),
    "ccio_bam_write_all": (C.c_int, [C.c_char_p, P, C.c_int, C.c_int]),
    "ccio_bai_mapped": (C.c_int64, [C.c_char_p]),
    "ccio_bai_region_bytes": (C.c_int, [C.c_char_p, C.c_int32, P, P, P, P]),
    "ccio_write_columns": (C.c_int, [C.c_char_p, C.c_char_p, C.c_int32, P, P, C.c_int64, P, P, P, P, P, P, P, P,
                                     P, P, P, P, C.c_int32, P, P, P, P, C.c_int, C.c_int]),
}

AMD_SIGS = {
    "cc_create": (C.c_int, [C.c_int, C.POINTER(P)]),
    "cc_destroy": (C.c_int, [P]),
    "cc_last_error": (C.c_char_p, [P]),
    "cc_host_alloc": (P, [P, C.c_uint64]),
    "cc_host_free": (None, [P, P]),
    "cc_set_profiling": (C.c_int, [P, C.c_int]),
    "cc_profile_only": (C.c_int, [P, C.c_char_p]),
    "cc_kernel_times": (C.c_int, [P, C.c_char_p, C.c_int, P, P, C.c_int]),
    "cc_synchronize": (C.c_int, [P]),
    "cc_defer": (C.c_int, [P, C.c_int]),
    "cc_commit": (C.c_int, [P]),
    "cc_debug_skew_plan": (C.c_int, [P, C.c_int32, C.c_char_p, C.c_int64]),
    "cc_debug_build": (C.c_int, []),
    "cc_launch_count": (C.c_int64, []),
    "cc_table_upload": (C.c_int, [P, C.POINTER(cc_records), C.c_int32, i32p]),
    "cc_table_free": (C.c_int, [P, C.c_int32]),
    "cc_read_bam": (C.c_int, [P, C.c_int32, C.c_int64, P, P, C.c_int32, P, C.POINTER(cc_read_bam_params), i32p]),
    "cc_read_bam_rerun": (C.c_int, [P, C.c_int32, C.c_uint64]),
    "cc_group_counters": (C.c_int, [P, C.c_int32, P]),
    "cc_group_free": (C.c_int, [P, C.c_int32]),
    "cc_consensus_maker": (C.c_int, [P, C.c_int32, C.c_double, i64p]),
    "cc_duplex_consensus": (C.c_int, [P, C.c_int32, P, C.c_int32, i64p]),
    "cc_singleton_correction": (C.c_int, [P, C.c_int32, C.c_int32, P, C.c_int32, i64p]),
    "cc_fetch": (C.c_int64, [P, C.c_int32, C.c_char_p, P, C.c_int64]),
    "cc_sscs_vote": (C.c_int, [P, C.c_int32, P, P, C.c_int64, C.c_double, P, P, P, C.c_int32]),
    "cc_pair_vote": (C.c_int, [P, C.c_int32, C.c_int32, C.c_int32, P, P, C.c_int64, P, P, P, C.c_int32]),
    "cc_group": (C.c_int, [P, C.c_int64, P, C.c_int32, P, P, i64p]),
    "cc_duplex_join": (C.c_int, [P, C.c_int32, C.c_int64, P, P, C.c_int64, P, C.c_int32, P, P, C.c_int32, P,
                                 C.c_int32, P, P, P, P, C.c_int32]),
    "cc_extract_barcodes": (C.c_int, [P, C.c_int64, P, P, P, P, C.c_char_p, P, C.c_int32, P, P, P, P, P, P, P, P, P]),
    "cc_comm_unique_id": (C.c_int, [C.c_char_p, C.c_int32]),
    "cc_comm_init": (C.c_int, [P, C.c_int32, C.c_int32, C.c_char_p, C.POINTER(P)]),
    "cc_comm_destroy": (C.c_int, [P]),
    "cc_reduce_stats": (C.c_int, [P, P, P, C.c_int32, P, P, C.c_int32]),
    "cc_allreduce_max": (C.c_int, [P, P, P, C.c_int32]),
}


def _bind(lib, sigs):
    for name, (res, args) in sigs.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


def io():
    global _io
    if _io is None:
        path = os.path.join(LIBDIR, "libccio.so")
        if not os.path.exists(path):
            raise ImportError("libccio.so not built; run __graft_entry__.build()")
        _io = _bind(C.CDLL(path), IO_SIGS)
    return _io


def amd():
    """The HIP engine.  Raises if the extension is missing: no CPU fallback."""
    global _amd
    if _amd is None:
        # CCAMD_LIB: an alternative in-tree build of the same engine (tuning variants)
        path = os.environ.get("CCAMD_LIB") or os.path.join(LIBDIR, "libccamd.so")
        if not os.path.exists(path):
            raise ImportError("libccamd.so (HIP engine) not built; run __graft_entry__.build()")
        _amd = _bind(C.CDLL(path), AMD_SIGS)
    return _amd


def ptr(a):
    return None if a is None else a.ctypes.data_as(P)


def io_error():
    return io().ccio_last_error().decode(errors="replace")
