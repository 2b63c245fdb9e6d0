"""Host orchestration around the C ABI: BAM decode -> SoA -> HBM -> GPU stages -> BAM.

Result arrays fetched from a read_bam group (cc_fetch names):
  read_bam            fam_sizes_by_creation[F] (after cc_consensus_maker), bad_rec[NB]
  cc_consensus_maker  emit_fam/emit_n/emit_rec/emit_vslot[NE], emit_ckey[9*NE/2] (per entry),
                      vote_meta[5*NV] (L, mapq, tlen, flag, rg), cons_seq, cons_qual
  cc_duplex_consensus dec/t_rec/p_rec/vslot[Q], vote_meta, cons_seq, cons_qual
  cc_singleton_corr.  dec/t_rec/p_rec/vslot[Q], q_ckey[9*Q], vote_meta, cons_seq, cons_qual
dec codes: DCS 0 = duplex made, 1 = SSCS singleton, 2 = partner already used, 3 = empty slot;
           SC  0 = corrected by SSCS, 1 = by singleton, 2 = uncorrected, 3 = empty slot.
"""
import ctypes as C
import os

import numpy as np

from . import native as N
from .consensus_helper import region_list, region_runs

MODE_SSCS, MODE_DUPLEX = 0, 1


class Interner(object):
    def __init__(self):
        self.h = N.io().ccio_interner_new()

    def __del__(self):
        try:
            if self.h:
                N.io().ccio_interner_free(self.h)
        except Exception:
            pass

    def size(self, kind):
        return int(N.io().ccio_interner_size(self.h, kind))

    def get(self, kind, i):
        buf = C.create_string_buffer(4096)
        n = N.io().ccio_interner_get(self.h, kind, int(i), buf, 4096)
        if n < 0:
            raise KeyError(i)
        return buf.value.decode()

    def intern(self, kind, s):
        return int(N.io().ccio_interner_intern(self.h, kind, s.encode()))

    def swap_table(self):
        n = int(N.io().ccio_interner_swap_table(self.h, None, 0))
        out = np.zeros(max(n, 1), np.int32)
        N.io().ccio_interner_swap_table(self.h, N.ptr(out), n)
        return out[:n]


class Records(object):
    """cc_records SoA as numpy arrays (owned here, pointed to by .struct)."""

    FIELDS = [("tid", np.int32), ("pos", np.int32), ("mtid", np.int32), ("mpos", np.int32), ("tlen", np.int32),
              ("flag", np.uint16), ("mapq", np.uint8), ("cigar_id", np.int32), ("qlen", np.int32),
              ("lseq", np.int32), ("bc_id", np.int32), ("rg_id", np.int32), ("rflags", np.uint8),
              ("qn_off", np.uint64), ("qn_len", np.uint16), ("pay_off", np.uint64), ("rdig", np.uint64)]

    def __init__(self, n, qn_bytes, pay_bytes, max_len):
        self.n = int(n)
        self.max_len = int(max_len)
        for name, dt in self.FIELDS:
            setattr(self, name, np.zeros(max(self.n, 1), dt))
        self.qn_blob = np.zeros(int(qn_bytes) + 16, np.uint8)
        self.payload = np.zeros(int(pay_bytes) + 64, np.uint8)
        s = N.cc_records()
        s.n = self.n
        for name, _ in self.FIELDS:
            setattr(s, name, getattr(self, name).ctypes.data)
        s.qn_blob = self.qn_blob.ctypes.data
        s.qn_blob_bytes = int(qn_bytes)
        s.payload = self.payload.ctypes.data
        s.payload_bytes = int(pay_bytes)
        s.rdig = self.rdig.ctypes.data
        self.struct = s


class Bam(object):
    """A BAM file decoded into memory by libccio (pysam.AlignmentFile stand-in)."""

    def __init__(self, path, nthreads=0):
        self.path = path
        self._attach(N.io().ccio_bam_open(path.encode(), nthreads))

    def _attach(self, h):
        if not h:
            raise IOError(N.io_error())
        self.h = h
        self.n = int(N.io().ccio_bam_nrec(self.h))
        self.refs = []
        buf = C.create_string_buffer(4096)
        ln = C.c_int32()
        for i in range(int(N.io().ccio_bam_nref(self.h))):
            N.io().ccio_bam_ref(self.h, i, buf, 4096, C.byref(ln))
            self.refs.append((buf.value.decode(), ln.value))

    @classmethod
    def _handle(cls, h, path=None):
        b = cls.__new__(cls)
        b.path = path
        b.h = None
        b._attach(h)
        return b

    # ---- rank-local record sets (the multi-GPU driver, sharded.py)
    @classmethod
    def open_regions(cls, path, tids, begs, ends, nthreads=0):
        """The records with beg <= pos < end on tid of one of the regions, in file order, read through
        path's BAI (only the regions' BGZF blocks are read)."""
        t = np.ascontiguousarray(tids, np.int32)
        b = np.ascontiguousarray(begs, np.int64)
        e = np.ascontiguousarray(ends, np.int64)
        return cls._handle(N.io().ccio_bam_open_regions(path.encode(), len(t), N.ptr(t), N.ptr(b), N.ptr(e),
                                                        nthreads), path)

    @classmethod
    def combine(cls, parts, blobs=(), key=1, tmpl=None):
        """parts' records then the raw record blobs', in that order, stably sorted by key (0: tid, pos;
        1: the samtools-sort stand-in key tid, pos, is_reverse; 2: unsorted)."""
        hs = (N.P * max(len(parts), 1))(*[p.h for p in parts])
        blobs = [np.ascontiguousarray(x, np.uint8) for x in blobs]
        bp = (N.P * max(len(blobs), 1))(*[x.ctypes.data for x in blobs])
        bn = np.array([len(x) for x in blobs] or [0], np.int64)
        h = N.io().ccio_bam_combine(tmpl.h if tmpl is not None else None, hs, len(parts), bp, N.ptr(bn), len(blobs),
                                    int(key), 0)
        return cls._handle(h)

    def origin(self):
        out = np.zeros(max(self.n, 1), np.int64)
        if N.io().ccio_bam_origin(self.h, N.ptr(out)) != 0:
            raise IOError(N.io_error())
        return out[:self.n]

    def cores(self):
        """(tid, pos, mtid, mpos, flag) of every record."""
        n = max(self.n, 1)
        t, p, mt, mp = (np.zeros(n, np.int32) for _ in range(4))
        f = np.zeros(n, np.uint16)
        N.io().ccio_bam_cores(self.h, N.ptr(t), N.ptr(p), N.ptr(mt), N.ptr(mp), N.ptr(f))
        return t[:self.n], p[:self.n], mt[:self.n], mp[:self.n], f[:self.n]

    def pack(self, idx):
        """The raw records idx (block_size first), concatenated."""
        i = np.ascontiguousarray(idx, np.int64)
        need = N.io().ccio_bam_pack(self.h, len(i), N.ptr(i), None, 0)
        if need < 0:
            raise IOError(N.io_error())
        out = np.zeros(max(int(need), 1), np.uint8)
        N.io().ccio_bam_pack(self.h, len(i), N.ptr(i), N.ptr(out), int(need))
        return out[:int(need)]

    def write_all(self, path, level=6, nthreads=0):
        if N.io().ccio_bam_write_all(path.encode(), self.h, level, nthreads) != 0:
            raise IOError(N.io_error())

    def close(self):
        if self.h:
            N.io().ccio_bam_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def qname(self, i):
        buf = C.create_string_buffer(1024)
        N.io().ccio_bam_qname(self.h, int(i), buf, 1024)
        return buf.value.decode()

    def decode(self, interner, mode, delim="|", nthreads=0):
        qn = C.c_uint64()
        pay = C.c_uint64()
        ml = C.c_int32()
        N.io().ccio_bam_layout(self.h, C.byref(qn), C.byref(pay), C.byref(ml), nthreads)
        rec = Records(self.n, qn.value, pay.value, ml.value)
        rc = N.io().ccio_bam_decode(self.h, interner.h, mode, (delim or "|").encode(), C.byref(rec.struct), nthreads)
        if rc != 0:
            raise IOError(N.io_error())
        return rec


class Stream(object):
    """The order in which read_bam sees records: whole file (until_eof) or the bed
    regions in file order, each region = records with start <= pos < end on its
    contig (pysam overlap fetch + the pos filter of consensus_helper.py:391-396)."""

    def __init__(self, rec_idx, region, region_run, region_keys):
        self.rec = np.ascontiguousarray(rec_idx, np.int32)
        self.region = np.ascontiguousarray(region, np.int32)
        self.region_run = np.ascontiguousarray(region_run, np.int32)
        self.region_keys = region_keys

    @property
    def n(self):
        return len(self.rec)


def whole_file_stream(records):
    n = records.n
    return Stream(np.arange(n, dtype=np.int32), np.zeros(n, np.int32), np.zeros(1, np.int32), None)


def bed_stream(records, refs, bedfile):
    regions = region_list(bedfile)
    names = {name: i for i, (name, _) in enumerate(refs)}
    n = records.n
    tid = records.tid[:n].astype(np.int64)
    pos = records.pos[:n].astype(np.int64)
    key = np.where(tid < 0, np.int64(1) << 62, (tid << 32) + pos)
    if n > 1 and np.any(np.diff(key) < 0):
        raise ValueError("--bedfile needs a coordinate-sorted BAM (indexed fetch)")
    pieces, regs = [], []
    for r, (k, chrom, start, end) in enumerate(regions):
        if chrom not in names:
            raise ValueError("invalid contig `%s`" % chrom)   # pysam fetch on an unknown contig
        t = names[chrom]
        lo = np.searchsorted(key, (t << 32) + max(start, 0), "left")
        hi = np.searchsorted(key, (t << 32) + max(end, 0), "left")
        if hi > lo:
            pieces.append(np.arange(lo, hi, dtype=np.int32))
            regs.append(np.full(hi - lo, r, np.int32))
    rec = np.concatenate(pieces) if pieces else np.zeros(0, np.int32)
    reg = np.concatenate(regs) if regs else np.zeros(0, np.int32)
    return Stream(rec, reg, np.array(region_runs(regions), np.int32), [x[0] for x in regions])


def coord_sorted(records):
    """True when records are in (tid, pos) order with unmapped (tid -1) last: position groups are
    then contiguous and the engine groups tags per position group instead of a global sort."""
    if not hasattr(records, "_coord_sorted"):
        n = records.n
        tid = records.tid[:n].astype(np.int64)
        key = np.where(tid < 0, np.int64(1) << 62, (tid << 32) + records.pos[:n].astype(np.int64))
        records._coord_sorted = bool(n < 2 or np.all(key[1:] >= key[:-1]))
    return records._coord_sorted


class Engine(object):
    """One HIP context on one GPU (cc_ctx)."""

    def __init__(self, device=0):
        self.lib = N.amd()
        h = N.P()
        rc = self.lib.cc_create(int(device), C.byref(h))
        if rc != 0:
            raise N.CCError(rc, "cc_create failed (no usable GPU?)")
        self.h = h
        self.tables = {}

    def close(self):
        if self.h:
            self.lib.cc_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc != 0:
            raise N.CCError(rc, self.lib.cc_last_error(self.h).decode(errors="replace"))

    def upload(self, records):
        tid = C.c_int32()
        self._check(self.lib.cc_table_upload(self.h, C.byref(records.struct), records.max_len, C.byref(tid)))
        self.tables[tid.value] = records
        return tid.value

    def free_table(self, t):
        self.lib.cc_table_free(self.h, t)
        self.tables.pop(t, None)

    def read_bam(self, table, stream, delim_filter, badread_file, scope_by_run, seed=0x5eed):
        sorted_ok = coord_sorted(self.tables[table])
        for attempt in range(6):
            prm = N.cc_read_bam_params(int(delim_filter), int(badread_file), int(scope_by_run), int(sorted_ok),
                                       (seed + 0x9E3779B97F4A7C15 * attempt) & 0xFFFFFFFFFFFFFFFF)
            gid = C.c_int32(0)
            rc = self.lib.cc_read_bam(self.h, table, stream.n, N.ptr(stream.rec), N.ptr(stream.region),
                                      len(stream.region_run), N.ptr(stream.region_run), C.byref(prm), C.byref(gid))
            if rc == N.CC_E_COLLISION:
                self.lib.cc_group_free(self.h, gid.value)
                continue
            if rc != 0:
                msg = self.lib.cc_last_error(self.h).decode(errors="replace")
                self.lib.cc_group_free(self.h, gid.value)
                raise N.CCError(rc, msg)
            return gid.value
        raise N.CCError(N.CC_E_COLLISION, "repeated hash collisions")

    def rerun(self, group, seed):
        self._check(self.lib.cc_read_bam_rerun(self.h, group, seed))

    def counters(self, group):
        a = np.zeros(N.NUM_COUNTERS, np.int64)
        self._check(self.lib.cc_group_counters(self.h, group, N.ptr(a)))
        return {k: int(a[v]) for k, v in N.CNT.items()}

    def fetch(self, group, name, dtype):
        nb = self.lib.cc_fetch(self.h, group, name.encode(), None, 0)
        if nb < 0:
            raise N.CCError(int(nb), self.lib.cc_last_error(self.h).decode())
        out = np.zeros(nb // np.dtype(dtype).itemsize, dtype)
        if nb:
            self.lib.cc_fetch(self.h, group, name.encode(), N.ptr(out), nb)
        return out

    def free_group(self, g):
        self.lib.cc_group_free(self.h, g)

    def consensus_maker(self, group, cutoff):
        n = C.c_int64()
        self._check(self.lib.cc_consensus_maker(self.h, group, float(cutoff), C.byref(n)))
        return n.value

    def duplex_consensus(self, group, swap):
        n = C.c_int64()
        self._check(self.lib.cc_duplex_consensus(self.h, group, N.ptr(swap), len(swap), C.byref(n)))
        return n.value

    def singleton_correction(self, sgroup, ssgroup, swap):
        n = C.c_int64()
        self._check(self.lib.cc_singleton_correction(self.h, sgroup, ssgroup, N.ptr(swap), len(swap), C.byref(n)))
        return n.value

    # ---- function-level boundary
    def sscs_vote(self, table, member_index, fam_offsets, cutoff, stride=None):
        """consensus_maker(readList, cutoff) (SSCS_maker.py:81-168) over caller-given families of a
        table's records: family k = records member_index[fam_offsets[k]:fam_offsets[k+1]], its first
        member the template.  Returns (seq codes (nfam, stride) as BAM nibble codes one per base,
        quals (nfam, stride), meta (nfam, 5) = L, mapq, tlen, flag, rg id)."""
        rec = self.tables[table]
        stride = stride or ((rec.max_len + 15) & ~15)
        mi = np.ascontiguousarray(member_index, np.int32)
        fo = np.ascontiguousarray(fam_offsets, np.int64)
        nf = len(fo) - 1
        seq = np.zeros((max(nf, 1), stride // 2), np.uint8)
        qual = np.zeros((max(nf, 1), stride), np.uint8)
        meta = np.zeros((max(nf, 1), 5), np.int32)
        self._check(self.lib.cc_sscs_vote(self.h, table, N.ptr(mi), N.ptr(fo), nf, float(cutoff), N.ptr(seq),
                                          N.ptr(qual), N.ptr(meta), stride))
        return unpack_nibbles(seq[:nf], stride), qual[:nf], meta[:nf]

    def pair_vote(self, mode, table_a, table_b, rec_a, rec_b, stride=None):
        """duplex_consensus(read1, read2) over caller-given pairs: mode 0 DCS (DCS_maker.py:99-123),
        mode 1 singleton correction's Q>29 variant (singleton_correction.py:61-86)."""
        ml = max(self.tables[table_a].max_len, self.tables[table_b].max_len)
        stride = stride or ((ml + 15) & ~15)
        a = np.ascontiguousarray(rec_a, np.int32)
        b = np.ascontiguousarray(rec_b, np.int32)
        n = len(a)
        seq = np.zeros((max(n, 1), stride // 2), np.uint8)
        qual = np.zeros((max(n, 1), stride), np.uint8)
        meta = np.zeros((max(n, 1), 5), np.int32)
        self._check(self.lib.cc_pair_vote(self.h, int(mode), table_a, table_b, N.ptr(a), N.ptr(b), n, N.ptr(seq),
                                          N.ptr(qual), N.ptr(meta), stride))
        return unpack_nibbles(seq[:n], stride), qual[:n], meta[:n]

    def group(self, keys):
        """cc_group: read_dict's grouping of caller-given keys ((n, key_bytes) uint8, key_bytes a
        multiple of 4): (perm int32, fam_offsets int64), families in first-seen order."""
        k = np.ascontiguousarray(keys, np.uint8)
        n = k.shape[0]
        perm = np.zeros(max(n, 1), np.int32)
        off = np.zeros(n + 1, np.int64)
        nf = C.c_int64()
        self._check(self.lib.cc_group(self.h, n, N.ptr(k), k.shape[1], N.ptr(perm), N.ptr(off), C.byref(nf)))
        return perm[:n], off[:nf.value + 1]

    def duplex_join(self, mode, keys, partner_keys, x_keys=None, vote=None):
        """cc_duplex_join: (decision int32, partner int64) per entry; vote = (table_a, rec_a, table_x,
        rec_x) also returns (seq codes, quals, meta) rows per entry."""
        k = np.ascontiguousarray(keys, np.uint8)
        p = np.ascontiguousarray(partner_keys, np.uint8)
        x = np.ascontiguousarray(x_keys if x_keys is not None else np.zeros((0, k.shape[1]), np.uint8), np.uint8)
        n, m = k.shape[0], x.shape[0]
        dec = np.zeros(max(n, 1), np.int32)
        part = np.zeros(max(n, 1), np.int64)
        seq = qual = meta = None
        ta, ra, tx, rx, stride = -1, None, -1, None, 0
        if vote is not None:
            ta, ra, tx, rx = vote
            ra = np.ascontiguousarray(ra, np.int32)
            rx = np.ascontiguousarray(rx if rx is not None else np.zeros(0, np.int32), np.int32)
            ml = max(self.tables[ta].max_len, self.tables[tx].max_len if tx >= 0 else 0)
            stride = (ml + 15) & ~15
            seq = np.zeros((max(n, 1), stride // 2), np.uint8)
            qual = np.zeros((max(n, 1), stride), np.uint8)
            meta = np.zeros((max(n, 1), 5), np.int32)
        self._check(self.lib.cc_duplex_join(self.h, int(mode), n, N.ptr(k), N.ptr(p), m, N.ptr(x), k.shape[1],
                                            N.ptr(dec), N.ptr(part), ta, N.ptr(ra), tx, N.ptr(rx), N.ptr(seq),
                                            N.ptr(qual), N.ptr(meta), stride))
        if vote is None:
            return dec[:n], part[:n]
        return dec[:n], part[:n], (unpack_nibbles(seq[:n], stride), qual[:n], meta[:n])

    def comm_init(self, world, rank, uid):
        c = N.P()
        self._check(self.lib.cc_comm_init(self.h, int(world), int(rank), uid, C.byref(c)))
        return c

    def reduce_stats(self, comm, counters, fam_count=None, fam_first=None):
        """The sharded pipeline's one collective (RCCL): counters and fam_count summed, fam_first
        min-reduced over the ranks, in place (int64 arrays)."""
        fl = 0 if fam_count is None else len(fam_count)
        self._check(self.lib.cc_reduce_stats(self.h, comm, N.ptr(counters), len(counters),
                                             N.ptr(fam_count) if fl else None, N.ptr(fam_first) if fl else None, fl))

    def allreduce_max(self, comm, v):
        self._check(self.lib.cc_allreduce_max(self.h, comm, N.ptr(v), len(v)))

    def set_profiling(self, on):
        self._check(self.lib.cc_set_profiling(self.h, int(on)))

    def profile_only(self, names=()):
        """Time only these kernel scopes (all when empty)."""
        self._check(self.lib.cc_profile_only(self.h, "\n".join(names).encode()))

    def launch_count(self):
        """Device operations enqueued so far by this process (cc_launch_count)."""
        return int(self.lib.cc_launch_count())

    def kernel_times(self):
        names = C.create_string_buffer(1 << 16)
        ms = np.zeros(256, np.float64)
        cnt = np.zeros(256, np.int64)
        k = self.lib.cc_kernel_times(self.h, names, 1 << 16, N.ptr(ms), N.ptr(cnt), 256)
        nm = names.value.decode().split("\n")[:k]
        return {nm[i]: (float(ms[i]), int(cnt[i])) for i in range(k)}

    def synchronize(self):
        self._check(self.lib.cc_synchronize(self.h))

    def deferred(self, calls):
        """Runs calls() (stage calls on resident groups, e.g. one bench step) with the planned passes'
        end-of-pass checks deferred to one wait at the end (cc_defer / cc_commit).  When a deferred
        pass did not hold its plan, calls() runs again with deferral off: every pass then checks
        itself and re-runs exactly where needed, as without deferral."""
        self._check(self.lib.cc_defer(self.h, 1))
        try:
            calls()
        finally:
            self.lib.cc_defer(self.h, 0)
            rc = self.lib.cc_commit(self.h)
        if rc == N.CC_E_REPLAY:
            calls()
        else:
            self._check(rc)


def comm_unique_id():
    """A fresh RCCL unique id (128 bytes) for cc_comm_init; rank 0 makes it, the others receive it."""
    buf = C.create_string_buffer(128)
    rc = N.amd().cc_comm_unique_id(buf, 128)
    if rc != 0:
        raise N.CCError(rc, "RCCL unique id")
    return buf.raw


def duplex_tag(tag):
    """duplex_tag(tag) (consensus_helper.py:639-683) through libccio (ccio_duplex_tag); IndexError for
    fewer than nine '_' fields, as the reference."""
    t = tag.encode()
    buf = C.create_string_buffer(2 * len(t) + 16)
    k = N.io().ccio_duplex_tag(t, buf, len(buf))
    if k < 0:
        raise IndexError(N.io_error())
    return buf.value.decode()


def pack_keys(tags, width=None):
    """Tag strings as fixed-width byte keys (zero padded to a multiple of 4) for cc_group /
    cc_duplex_join: (n, width) uint8."""
    raw = [t.encode() for t in tags]
    w = width or max([len(r) for r in raw] + [1])
    w = (w + 3) & ~3
    out = np.zeros((len(raw), w), np.uint8)
    for i, r in enumerate(raw):
        if len(r) > w:
            raise ValueError("tag longer than the key width")
        out[i, :len(r)] = np.frombuffer(r, np.uint8)
    return out


def unpack_nibbles(packed, stride):
    """(n, stride/2) BAM nibble bytes -> (n, stride) base codes (first base in the high nibble)."""
    out = np.zeros((packed.shape[0], stride), np.uint8)
    out[:, 0::2] = packed >> 4
    out[:, 1::2] = packed & 15
    return out


# ---------------------------------------------------------------- output helpers
def csn_names(interner, ckey9, suffix):
    n = len(suffix)
    off = np.zeros(n + 1, np.int64)
    ck = np.ascontiguousarray(ckey9, np.int32)
    sf = np.ascontiguousarray(suffix, np.int64)
    need = N.io().ccio_format_csn_names(interner.h, n, N.ptr(ck), N.ptr(sf), None, 0, N.ptr(off))
    if need < 0:
        raise RuntimeError(N.io_error())
    blob = np.zeros(max(int(need), 1), np.uint8)
    N.io().ccio_format_csn_names(interner.h, n, N.ptr(ck), N.ptr(sf), N.ptr(blob), int(need), N.ptr(off))
    return blob, off


def dcs_names(bam, rec_tag, rec_ds):
    n = len(rec_tag)
    off = np.zeros(n + 1, np.int64)
    a = np.ascontiguousarray(rec_tag, np.int64)
    b = np.ascontiguousarray(rec_ds, np.int64)
    need = N.io().ccio_format_dcs_names(bam.h, n, N.ptr(a), N.ptr(b), None, 0, N.ptr(off))
    if need < 0:
        raise RuntimeError(N.io_error())
    blob = np.zeros(max(int(need), 1), np.uint8)
    N.io().ccio_format_dcs_names(bam.h, n, N.ptr(a), N.ptr(b), N.ptr(blob), int(need), N.ptr(off))
    return blob, off


def write_bam(path, template, interner, specs, srcs, names=None, name_off=None, cons_seq=None, cons_qual=None,
              level=6, nthreads=0, sink=None):
    """Assembles and writes one output BAM (ccio_write_bam).  sink (the orchestrator's fused
    sort_index, Sink) may redirect it: written sorted and indexed under its sorted name, and kept in
    memory for the next stage.  Returns the path written."""
    specs = np.ascontiguousarray(specs, N.OUT_SPEC_DTYPE)
    arr = (N.P * len(srcs))(*[s.h for s in srcs])
    dummy = np.zeros(1, np.uint8)
    dummy_off = np.zeros(2, np.int64)
    out, flags, keep = path, 0, None
    if sink is not None:
        out, flags, k = sink.route(path)
        keep = N.P() if k else None
    rc = N.io().ccio_write_bam_ex(out.encode(), template.h, interner.h, len(specs), N.ptr(specs), arr, len(srcs),
                                  N.ptr(names if names is not None else dummy),
                                  N.ptr(name_off if name_off is not None else dummy_off),
                                  N.ptr(cons_seq if cons_seq is not None and len(cons_seq) else dummy),
                                  N.ptr(cons_qual if cons_qual is not None and len(cons_qual) else dummy),
                                  level, nthreads, flags, C.byref(keep) if keep is not None else None)
    if rc != 0:
        raise IOError(N.io_error())
    if keep is not None:
        sink.kept[out] = Bam._handle(keep.value, out)
    return out


class Sink(object):
    """The orchestrator's fused sort_index (ConsensusCruncher.py:10-34): a stage output X.bam that the
    pipeline would write, then sort to X.sorted.bam (removing X.bam) and index, is written sorted and
    indexed under X.sorted.bam at once; the records of the outputs named in `keep` stay in memory
    (kept) for the stage that reads that file next.  Outputs not named in `fused` are written as the
    stage names them."""

    def __init__(self, fused=(), keep=(), async_writes=False):
        self.fused = set(os.path.abspath(p) for p in fused)
        self.keep = set(os.path.abspath(p) for p in keep)
        self.kept = {}
        # fused outputs compressed and written in the background (CCIO_W_ASYNC): the caller runs
        # flush_writes() before it moves or hands over those files
        self.async_flag = N.W_ASYNC if async_writes else 0

    def route(self, path):
        """(path to write, writer flags, keep the records)"""
        ap = os.path.abspath(path)
        if ap in self.fused:
            return ('{}.sorted.bam'.format(path.split('.bam', 1)[0]), N.W_SORT | N.W_INDEX | self.async_flag,
                    ap in self.keep)
        return path, 0, False

    def take(self, path):
        """The kept records of a written file (Bam, by the path it was written to), or None."""
        return self.kept.pop(path, None)


def flush_writes():
    """Waits for every background (CCIO_W_ASYNC) write; raises the first failure."""
    if N.io().ccio_flush() != 0:
        raise IOError(N.io_error())


def merge_kept(out, bams, level=6, nthreads=0, index=True, keep=True, async_writes=False):
    """samtools merge of sorted record sets in memory (ties keep input order) written to out (+ .bai);
    returns the merged records (Bam) when keep.  async_writes: compressed and written in the
    background (flush_writes)."""
    arr = (N.P * len(bams))(*[b.h for b in bams])
    k = N.P() if keep else None
    fl = (N.W_INDEX if index else 0) | (N.W_ASYNC if async_writes else 0)
    rc = N.io().ccio_merge_handles(out.encode(), C.cast(arr, N.P), len(bams), level, nthreads, fl,
                                   C.byref(k) if keep else None)
    if rc != 0:
        raise IOError(N.io_error())
    return Bam._handle(k.value, out) if keep else None


def make_specs(n):
    s = np.zeros(n, N.OUT_SPEC_DTYPE)
    s["name_id"] = -1
    s["rg_id"] = -1
    return s


def sort_bam(inp, out, level=6, nthreads=0):
    if N.io().ccio_sort_bam(inp.encode(), out.encode(), level, nthreads) != 0:
        raise IOError(N.io_error())


def merge_bams(out, inputs, level=6, nthreads=0):
    arr = (C.c_char_p * len(inputs))(*[p.encode() for p in inputs])
    if N.io().ccio_merge_bams(out.encode(), C.cast(arr, N.P), len(inputs), level, nthreads) != 0:
        raise IOError(N.io_error())


def concat_bams(out, inputs, level=6, nthreads=0):
    arr = (C.c_char_p * len(inputs))(*[p.encode() for p in inputs])
    if N.io().ccio_concat_bams(out.encode(), C.cast(arr, N.P), len(inputs), level, nthreads) != 0:
        raise IOError(N.io_error())


def index_bam(path):
    """samtools index: writes path + '.bai'."""
    if N.io().ccio_index_bam(path.encode()) != 0:
        raise IOError(N.io_error())


class BarcodeAssertion(AssertionError):
    """extract_barcodes.py:291 `assert r1.id == r2.id`."""


EB_WIDTH, EB_BC = 32, 72   # cc_extract_barcodes: bases per read it reads, barcode bytes per pair


def extract_barcodes_gpu(engine, read1, read2, out_prefix, pattern=None, blist=None, nthreads=0):
    """The UMI extraction with the per-pair decision on the GPU (cc_extract_barcodes): libccio reads the
    FASTQs (ccio_fq_open / ccio_fq_heads) and writes the outputs from the decisions (ccio_fq_write).
    Same results as extract_barcodes; None when the barcodes exceed the kernel's sizes (32 bases,
    1024 listed barcodes, 31 lengths)."""
    io = N.io()
    if pattern is not None:
        if len(pattern) > EB_WIDTH:
            return None
        min_len, lens = len(pattern), None
    else:
        lens = sorted({len(b) for b in blist}, reverse=True)
        if len(blist) > 1024 or max(lens) > EB_WIDTH or len(lens) > 31:
            return None
        min_len = 0
    f = io.ccio_fq_open(read1.encode(), read2.encode(), min_len, nthreads)
    if not f:
        raise IOError(N.io_error())
    try:
        n = C.c_int64()
        stop = C.c_int32()
        io.ccio_fq_info(f, C.byref(n), C.byref(stop))
        stop_msg = N.io_error() if stop.value else None
        n = n.value
        h1 = np.zeros((max(n, 1), EB_WIDTH), np.uint8)
        h2 = np.zeros((max(n, 1), EB_WIDTH), np.uint8)
        l1 = np.zeros(max(n, 1), np.int32)
        l2 = np.zeros(max(n, 1), np.int32)
        if io.ccio_fq_heads(f, EB_WIDTH, N.ptr(h1), N.ptr(h2), N.ptr(l1), N.ptr(l2)) != 0:
            raise IOError(N.io_error())
        nh = 5 * len(pattern) if pattern is not None else len(blist)
        st = np.zeros(max(n, 1), np.uint8)
        bc = np.zeros((max(n, 1), EB_BC), np.uint8)
        c1 = np.zeros(max(n, 1), np.int32)
        c2 = np.zeros(max(n, 1), np.int32)
        b1 = np.zeros(max(n, 1), np.uint32)
        b2 = np.zeros(max(n, 1), np.uint32)
        cnt = np.zeros(3, np.int64)
        r1 = np.zeros(max(nh, 1), np.int64)
        r2 = np.zeros(max(nh, 1), np.int64)
        arr = (C.c_char_p * len(blist))(*[b.encode() for b in blist]) if pattern is None else None
        engine._check(engine.lib.cc_extract_barcodes(
            engine.h, n, N.ptr(h1), N.ptr(h2), N.ptr(l1), N.ptr(l2),
            pattern.encode() if pattern is not None else None, C.cast(arr, N.P) if arr is not None else None,
            len(blist) if pattern is None else 0, N.ptr(st), N.ptr(bc), N.ptr(c1), N.ptr(c2), N.ptr(b1), N.ptr(b2),
            N.ptr(cnt), N.ptr(r1), N.ptr(r2)))
        la = np.array(lens if lens else [0], np.int32)
        if io.ccio_fq_write(f, out_prefix.encode(), 0 if pattern is not None else 1, N.ptr(st), N.ptr(bc), EB_BC,
                            N.ptr(c1), N.ptr(c2), N.ptr(b1), N.ptr(b2), N.ptr(la), len(lens) if lens else 0,
                            nthreads) != 0:
            raise IOError(N.io_error())
    finally:
        io.ccio_fq_close(f)
    counts = dict(pairs=n + (1 if stop.value else 0), bad_spacer=int(cnt[0]), bad_barcode=int(cnt[1]),
                  good=int(cnt[2]), written=n)
    if stop.value == -2:
        raise BarcodeAssertion(stop_msg)
    if stop.value:
        raise IOError(stop_msg)
    if pattern is not None:
        return counts, r1[:nh].reshape(len(pattern), 5), r2[:nh].reshape(len(pattern), 5)
    return counts, r1[:nh], r2[:nh]


def extract_barcodes(read1, read2, out_prefix, pattern=None, blist=None, nthreads=0, engine=None):
    """libccio's UMI extraction (extract_barcodes.py:287-405).  Returns (counts dict, r1_hist, r2_hist):
    pattern mode histograms are (len(pattern), 5) over A,C,G,T,N; list mode one count per entry of
    `blist` (distinct barcodes).  Raises BarcodeAssertion where the reference's id assertion fails
    (the pairs before it written).  With an engine the per-pair decisions run on the GPU
    (extract_barcodes_gpu), barcodes beyond its sizes on the host."""
    if pattern is None and not blist:
        raise ValueError("No barcode specifications inputted. Please specify barcode list or pattern.")
    if engine is not None:
        got = extract_barcodes_gpu(engine, read1, read2, out_prefix, pattern, blist, nthreads)
        if got is not None:
            return got
    nh = 5 * len(pattern) if pattern is not None else len(blist)
    h1 = np.zeros(max(nh, 1), np.int64)
    h2 = np.zeros(max(nh, 1), np.int64)
    cnt = np.zeros(4, np.int64)
    nw = np.zeros(1, np.int64)
    arr = None
    if pattern is None:
        arr = (C.c_char_p * len(blist))(*[b.encode() for b in blist])
    rc = N.io().ccio_extract_barcodes(read1.encode(), read2.encode(), out_prefix.encode(),
                                      pattern.encode() if pattern is not None else None,
                                      C.cast(arr, N.P) if arr is not None else None,
                                      len(blist) if blist else 0, nthreads, N.ptr(cnt), N.ptr(h1), N.ptr(h2),
                                      N.ptr(nw))
    counts = dict(pairs=int(cnt[0]), bad_spacer=int(cnt[1]), bad_barcode=int(cnt[2]), good=int(cnt[3]),
                  written=int(nw[0]))
    if rc == -2:
        raise BarcodeAssertion(N.io_error())
    if rc != 0:
        raise IOError(N.io_error())
    if pattern is not None:
        return counts, h1[:nh].reshape(len(pattern), 5), h2[:nh].reshape(len(pattern), 5)
    return counts, h1[:nh], h2[:nh]
