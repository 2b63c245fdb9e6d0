"""ctypes front of the C++ oracle (oracle/cc_oracle.cpp, built as oracle/lib/libccoracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the cpu_baseline leg of
bench.py, never by the product.  The stages and the orchestration mirror oracle/cc_oracle.py (the
pinned Python restatement) and ConsensusCruncher.py:127-346; tests/test_oracle_native.py pins this
one to the same reference fixtures.  Each stage reports its consensus-only time (records decoded
in memory -> output records in memory, BAM I/O excluded) for the CPU baseline.
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib", "libccoracle.so")
_lib = None


class OracleError(Exception):
    """Raised where the reference raises (IndexError / ValueError / KeyError ...)."""


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise OSError("%s missing: run `make -C oracle` (or __graft_entry__.build())" % LIB_PATH)
        L = C.CDLL(LIB_PATH)
        L.ccor_last_error.restype = C.c_char_p
        L.ccor_sscs.argtypes = [C.c_char_p, C.c_char_p, C.c_double, C.c_char_p, C.c_char_p, C.POINTER(C.c_double)]
        L.ccor_dcs.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p, C.POINTER(C.c_double)]
        L.ccor_sc.argtypes = [C.c_char_p, C.c_char_p, C.POINTER(C.c_double)]
        L.ccor_sort.argtypes = [C.c_char_p, C.c_char_p]
        L.ccor_merge.argtypes = [C.c_char_p, C.POINTER(C.c_char_p), C.c_int]
        L.ccor_digests.argtypes = [C.c_char_p, C.c_void_p, C.c_int64]
        L.ccor_digests.restype = C.c_int64
        L.ccor_py_float.argtypes = [C.c_double, C.c_char_p, C.c_int]
        _lib = L
    return _lib


def _b(s):
    return None if s is None else s.encode()


def _check(rc):
    if rc != 0:
        raise OracleError(lib().ccor_last_error().decode(errors="replace"))


def sscs_stage(infile, outfile, cutoff, bedfile=None, bdelim="|"):
    t = C.c_double(0)
    _check(lib().ccor_sscs(_b(infile), _b(outfile), float(cutoff), _b(bedfile), _b(bdelim), C.byref(t)))
    return t.value


def dcs_stage(infile, outfile, bedfile=None):
    t = C.c_double(0)
    _check(lib().ccor_dcs(_b(infile), _b(outfile), _b(bedfile), C.byref(t)))
    return t.value


def sc_stage(singleton, bedfile=None):
    t = C.c_double(0)
    _check(lib().ccor_sc(_b(singleton), _b(bedfile), C.byref(t)))
    return t.value


def sort_index(bam):
    out = bam.split(".bam", 1)[0] + ".sorted.bam"
    _check(lib().ccor_sort(_b(bam), _b(out)))
    return out


def merge(out, *inputs):
    arr = (C.c_char_p * len(inputs))(*[p.encode() for p in inputs])
    _check(lib().ccor_merge(_b(out), arr, len(inputs)))
    return out


def digests(path):
    """Per-record canonical digests of a BAM file in file order (uint64)."""
    n = lib().ccor_digests(_b(path), None, 0)
    if n < 0:
        raise OracleError(lib().ccor_last_error().decode())
    out = np.zeros(max(n, 1), np.uint64)
    lib().ccor_digests(_b(path), out.ctypes.data, n)
    return out[:n]


def py_float(x):
    buf = C.create_string_buffer(64)
    lib().ccor_py_float(float(x), buf, 64)
    return buf.value.decode()


def consensus_pipeline(bam, c_output, bedfile="False", cutoff=0.7, bdelim="|", scorrect="True", times=None):
    """ConsensusCruncher.py:127-346 with the C++ oracle stages and the samtools stand-in
    (the same orchestration as oracle/cc_oracle.consensus_pipeline).  times (dict, optional)
    receives each stage's consensus-only seconds."""
    ident = os.path.basename(bam).split(".bam", 1)[0]
    sd = os.path.join(c_output, ident)
    bed = None if bedfile == "False" else bedfile
    times = {} if times is None else times
    for sub in ("sscs", "dcs", "sscs_sc", "dcs_sc"):
        os.makedirs(os.path.join(sd, sub), exist_ok=True)
    p = lambda sub, name: os.path.join(sd, sub, "%s.%s" % (ident, name))  # noqa: E731
    times["sscs"] = sscs_stage(bam, p("sscs", "sscs.bam"), cutoff, bed, bdelim)
    out = dict(badreads=p("sscs", "badReads.bam"), read_families=p("sscs", "read_families.txt"))
    out["sscs"] = sort_index(p("sscs", "sscs.bam"))
    out["singleton"] = sort_index(p("sscs", "singleton.bam"))
    os.rename(p("sscs", "stats.txt"), p("dcs", "stats.txt"))
    times["dcs"] = dcs_stage(out["sscs"], p("dcs", "dcs.bam"), bed)
    out["dcs"] = sort_index(p("dcs", "dcs.bam"))
    out["sscs_singleton"] = sort_index(p("dcs", "sscs.singleton.bam"))
    stats = p("dcs", "stats.txt")
    if scorrect != "False":
        os.rename(stats, p("sscs", "stats.txt"))
        times["sc"] = sc_stage(out["singleton"], bed)
        for name in ("sscs.correction", "singleton.correction", "uncorrected"):
            os.rename(p("sscs", name + ".bam"), p("sscs_sc", name + ".bam"))
            out[name.replace(".", "_")] = sort_index(p("sscs_sc", name + ".bam"))
        merge(p("sscs_sc", "sscs.sc.bam"), out["sscs"], out["sscs_correction"], out["singleton_correction"])
        out["sscs_sc"] = sort_index(p("sscs_sc", "sscs.sc.bam"))
        os.rename(p("sscs", "stats.txt"), p("dcs_sc", "stats.txt"))
        times["dcs_sc"] = dcs_stage(out["sscs_sc"], p("dcs_sc", "dcs.sc.bam"), bed)
        out["dcs_sc"] = sort_index(p("dcs_sc", "dcs.sc.bam"))
        out["sscs_sc_singleton"] = sort_index(p("dcs_sc", "sscs.sc.singleton.bam"))
        merge(p("dcs_sc", "all.unique.dcs.bam"), out["dcs_sc"], out["sscs_sc_singleton"], out["uncorrected"])
        out["all_unique"] = sort_index(p("dcs_sc", "all.unique.dcs.bam"))
        stats = p("dcs_sc", "stats.txt")
    out["stats"] = stats
    return out
