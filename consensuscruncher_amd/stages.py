"""The three consensus stages (SSCS, DCS, SC) on the GPU engine.

Each function reproduces the file contract of the reference stage script
(SURVEY.md §8b): the same output files, names, headers (template=input) and
stats text, with the per-read work done by libccamd on the GPU and the
BAM I/O by libccio.
"""
import collections
import math
import os
import re
import sys
import time

import numpy as np

from . import native as N
from .engine import (MODE_DUPLEX, MODE_SSCS, Bam, Engine, Interner, bed_stream, csn_names, dcs_names,
                     make_specs, whole_file_stream, write_bam)

__all__ = ["SSCSRun", "DCSRun", "SCRun", "run_sscs", "run_dcs", "run_sc", "get_engine", "sscs_side", "dcs_side",
           "sc_side"]

_ENGINE = None


def get_engine():
    global _ENGINE
    if _ENGINE is None:
        _ENGINE = Engine(int(os.environ.get("CC_DEVICE", "0")))
    return _ENGINE


def _stream(bam, rec, bedfile):
    return whole_file_stream(rec) if bedfile is None else bed_stream(rec, bam.refs, bedfile)


# ---------------------------------------------------------------- SSCS
class SSCSRun(object):
    """Device side of SSCS_maker.main (SSCS_maker.py:183-425): input decoded and
    resident in HBM, read_bam + consensus_maker run on the GPU.  step() re-runs
    the whole GPU chain on the resident input (bench); emit() writes the outputs."""

    def __init__(self, eng, infile, cutoff, bedfile=None, bdelim="|", shard=None, src=None, bam=None):
        """src: (bam, interner, records, stream) already decoded (a rank's records of a multi-GPU
        run, sharded.py); otherwise infile is decoded whole."""
        self.eng, self.cutoff, self.bedfile = eng, float(cutoff), bedfile
        self.times = {}   # host / device pieces of the first pass (bench's end-to-end breakdown)
        t = time.time()
        if src is not None:
            self.bam, self.it, self.rec, self.stream = src
        else:
            self.it = Interner()
            self.bam = bam if bam is not None else Bam(infile)
            self.times["open"] = time.time() - t
            self.rec = self.bam.decode(self.it, MODE_SSCS, bdelim)
            self.stream = _stream(self.bam, self.rec, bedfile) if shard is None else shard(self.bam, self.rec)
        self.times["decode"] = time.time() - t - self.times.get("open", 0.0)
        t = time.time()
        self.table = eng.upload(self.rec)
        self.times["upload"] = time.time() - t
        t = time.time()
        self.g = eng.read_bam(self.table, self.stream, delim_filter=1, badread_file=1, scope_by_run=0)
        eng.consensus_maker(self.g, self.cutoff)
        self.times["gpu_exact"] = time.time() - t

    @property
    def n_input(self):
        return self.stream.n

    def step(self, seed):
        self.eng.rerun(self.g, seed)
        self.eng.consensus_maker(self.g, self.cutoff)

    def close(self):
        if self.g is not None:
            self.eng.free_group(self.g)
            self.eng.free_table(self.table)
            self.g = None

    def emit(self, outfile, level=6, verbose=True, start_time=None, plot=True, side=True, sink=None):
        """Writes the three BAMs; side=False (a shard of a multi-GPU run) leaves stats.txt,
        read_families.txt, the time tracker and the plot to sscs_side over the summed parts."""
        eng, g, it, bam, rec = self.eng, self.g, self.it, self.bam, self.rec
        start_time = start_time or time.time()
        t0 = time.time()
        prefix = outfile.split('.sscs')[0]
        c = eng.counters(g)
        emit_n = eng.fetch(g, "emit_n", np.int32)
        emit_rec = eng.fetch(g, "emit_rec", np.int32)
        emit_vslot = eng.fetch(g, "emit_vslot", np.int32)
        # one sscs_qname per entry, shared by the entry's two emitted records
        emit_ckey = np.repeat(eng.fetch(g, "emit_ckey", np.int32).reshape(-1, 9), 2, axis=0).reshape(-1)
        meta = eng.fetch(g, "vote_meta", np.int32).reshape(-1, 5)
        cons_seq = eng.fetch(g, "cons_seq", np.uint8)
        cons_qual = eng.fetch(g, "cons_qual", np.uint8)
        bad_rec = eng.fetch(g, "bad_rec", np.int32)
        fam_sizes = eng.fetch(g, "fam_sizes_by_creation", np.int32)
        qstride = (rec.max_len + 15) & ~15
        ne = len(emit_n)
        self.times["emit_fetch"] = time.time() - t0
        t0 = time.time()
        names, name_off = csn_names(it, emit_ckey, emit_n)
        self.times["emit_names"] = time.time() - t0
        t0 = time.time()
        voted = emit_vslot >= 0
        # SSCS records (create_aligned_segment) and renamed singletons, in emission order
        sp = _new_specs(voted, emit_rec[voted], np.nonzero(voted)[0], emit_vslot[voted], meta, qstride)
        write_bam(outfile, bam, it, sp, [bam], names, name_off, cons_seq, cons_qual, level, sink=sink)
        ss = make_specs(int((~voted).sum()))
        ss["kind"] = N.OUT_RENAME
        ss["src_rec"] = emit_rec[~voted]
        ss["name_id"] = np.nonzero(~voted)[0]
        write_bam('{}.singleton.bam'.format(prefix), bam, it, ss, [bam], names, name_off, level=level, sink=sink)
        bs = make_specs(len(bad_rec))
        bs["kind"] = N.OUT_RAW
        bs["src_rec"] = bad_rec
        write_bam('{}.badReads.bam'.format(prefix), bam, it, bs, [bam], level=level, sink=sink)
        self.times["emit_write"] = time.time() - t0
        t0 = time.time()
        items = size_census(fam_sizes)
        mapped = int((rec.flag[:rec.n] & 4 == 0).sum())
        # (a whole-file stream holds every record once: its own records are the file's)
        mapped_own = mapped if self.stream.region_keys is None else int(
            (rec.flag[self.stream.rec[self.stream.region >= 0]] & 4 == 0).sum())
        part = dict(counters=c, sscs=int(voted.sum()), singletons=ne - int(voted.sum()), families=items,
                    mapped=mapped, never_emitted=c["FAMILIES"] - ne, mapped_own=mapped_own)
        if side:
            sscs_side(prefix, part, self.stream.region_keys, start_time, verbose, plot)
        self.times["emit_side"] = time.time() - t0
        return part


def sscs_side(prefix, part, region_keys, start_time, verbose=True, plot=True):
    """SSCS_maker.py:341-418: time tracker, stats.txt, QC prints, read_families.txt and the plot,
    from one run's numbers or the sums over the shards of one sample (multi-GPU)."""
    c = part["counters"]
    # time tracker: one line per region (SSCS_maker.py:341-346)
    with open('{}.time_tracker.txt'.format(prefix), 'w') as tt:
        if region_keys is not None:
            el = str((time.time() - start_time) / 60)
            for k in region_keys:
                tt.write(k + ': ')
                tt.write(el + '\n')
    summary = '''# === SSCS ===
Uncollapsed - Total reads: {}
Uncollapsed - Unmapped reads: {}
Uncollapsed - Secondary/Supplementary reads: {}
SSCS reads: {}
Singletons: {}
Bad spacers: {}\n'''.format(c["COUNTER"], c["UNMAPPED_MATE"], c["MULTIPLE_MAPPING"], part["sscs"], part["singletons"],
                            c["BAD_SPACER"])
    with open('{}.stats.txt'.format(prefix), 'w') as st:
        st.write(summary)
    if verbose:
        print(summary)
        print('# QC: Total uncollapsed reads should be equivalent to mapped reads in bam file.')
        print('Total uncollapsed reads: {}'.format(c["COUNTER"]))
        print('Total mapped reads in bam file: {}'.format(part["mapped"]))
        print("QC: check dictionaries to see if there are any remaining reads")
        print('=== pair_dict remaining ===')
        if c["UNPAIRED"]:
            print('%d unpaired reads' % c["UNPAIRED"])
        print('=== read_dict remaining ===')
        if part["never_emitted"]:
            print('%d tags never emitted' % part["never_emitted"])
        print('=== csn_pair_dict remaining ===')
    # read_families.txt: Counter over tag_dict values in insertion order (SSCS_maker.py:401-408)
    items = part["families"]
    with open(prefix + '.read_families.txt', "w") as f:
        f.write('family_size\tfrequency\n')
        f.write('\n'.join('%s\t%s' % x for x in items))
    if plot:
        _family_plot(items, prefix + '_tag_fam_size.png')
    return dict(counters=c, sscs=part["sscs"], singletons=part["singletons"], families=items)


def size_census(fam_sizes):
    """[(family size, families of that size)] in first-seen order (Counter over tag_dict's values,
    SSCS_maker.py:401-408), by one native pass (ccio_value_census)."""
    v = np.ascontiguousarray(fam_sizes, np.int32)
    if len(v) == 0:
        return []
    mx = int(v.max())
    first = np.empty(mx + 1, np.int64)
    count = np.empty(mx + 1, np.int64)
    if N.io().ccio_value_census(N.ptr(v), len(v), mx, N.ptr(first), N.ptr(count)) != 0:
        raise ValueError(N.io_error())
    present = np.flatnonzero(count)
    order = present[np.argsort(first[present], kind="stable")]
    return [(int(k), int(count[k])) for k in order]


def _new_specs(mask_or_n, src_rec, name_ids, vslot, meta, qstride):
    k = int(np.sum(mask_or_n)) if not np.isscalar(mask_or_n) else int(mask_or_n)
    sp = make_specs(k)
    sp["kind"] = N.OUT_NEW
    sp["src_rec"] = src_rec
    sp["name_id"] = name_ids
    sp["cons_len"] = meta[vslot, 0]
    sp["mapq"] = meta[vslot, 1]
    sp["tlen"] = meta[vslot, 2]
    sp["flag"] = meta[vslot, 3]
    sp["rg_id"] = meta[vslot, 4]
    sp["cons_off"] = vslot.astype(np.int64) * qstride
    return sp


def run_sscs(infile, outfile, cutoff, bedfile=None, bdelim="|", engine=None, level=6, verbose=True, sink=None,
             bam=None):
    """SSCS_maker.main (SSCS_maker.py:183-425).  sink / bam: the orchestrator's fused sort_index
    (engine.Sink) and an input already in memory (pipeline.consensus_pipeline)."""
    start_time = time.time()
    run = SSCSRun(engine or get_engine(), infile, cutoff, bedfile, bdelim, bam=bam)
    try:
        return run.emit(outfile, level, verbose, start_time, sink=sink)
    finally:
        run.close()


def _family_plot(items, path):
    """SSCS_maker.py:410-418.  Raises IndexError on an empty family table, as the reference does."""
    total_reads = sum(i * j for i, j in items)
    read_fraction = [(i * j) / total_reads for i, j in items]
    xmax = math.ceil(items[-1][0] / 10) * 10   # IndexError when there is no family (reference crash)
    try:
        import matplotlib
        matplotlib.use('Agg')
        import matplotlib.pyplot as plt
    except Exception:   # plotting is a side output; missing matplotlib is not fatal
        return
    plt.figure()
    plt.bar([i for i, _ in items], read_fraction)
    plt.xlim([0, xmax])
    plt.savefig(path)
    plt.close('all')


# ---------------------------------------------------------------- DCS
class DCSRun(object):
    """Device side of DCS_maker.main (DCS_maker.py:130-317)."""

    def __init__(self, eng, infile, bedfile=None, shard=None, src=None, bam=None):
        self.eng = eng
        self.times = {}   # host / device pieces of the first pass (bench's end-to-end breakdown)
        t = time.time()
        if src is not None:
            self.bam, self.it, self.rec, self.stream = src
        else:
            self.it = Interner()
            self.bam = bam if bam is not None else Bam(infile)
            self.rec = self.bam.decode(self.it, MODE_DUPLEX)
            self.stream = _stream(self.bam, self.rec, bedfile) if shard is None else shard(self.bam, self.rec)
        self.swap = self.it.swap_table()
        self.times["decode"] = time.time() - t
        t = time.time()
        self.table = eng.upload(self.rec)
        self.times["upload"] = time.time() - t
        t = time.time()
        self.g = eng.read_bam(self.table, self.stream, delim_filter=0, badread_file=0, scope_by_run=0)
        eng.duplex_consensus(self.g, self.swap)
        self.times["gpu_exact"] = time.time() - t

    @property
    def n_input(self):
        return self.stream.n

    def step(self, seed):
        self.eng.rerun(self.g, seed)
        self.eng.duplex_consensus(self.g, self.swap)

    def close(self):
        if self.g is not None:
            self.eng.free_group(self.g)
            self.eng.free_table(self.table)
            self.g = None

    def emit(self, outfile, level=6, verbose=True, start_time=None, side=True, sink=None):
        eng, g, it, bam, rec = self.eng, self.g, self.it, self.bam, self.rec
        start_time = start_time or time.time()
        if re.search(r'dcs\.sc', outfile) is not None:
            singleton_path = '{}.sscs.sc.singleton.bam'.format(outfile.split('.dcs.sc')[0])
        else:
            singleton_path = '{}.sscs.singleton.bam'.format(outfile.split('.dcs')[0])
        t0 = time.time()
        c = eng.counters(g)
        dec = eng.fetch(g, "dec", np.int32)
        t_rec = eng.fetch(g, "t_rec", np.int32)
        p_rec = eng.fetch(g, "p_rec", np.int32)
        vslot = eng.fetch(g, "vslot", np.int32)
        meta = eng.fetch(g, "vote_meta", np.int32).reshape(-1, 5)
        cons_seq = eng.fetch(g, "cons_seq", np.uint8)
        cons_qual = eng.fetch(g, "cons_qual", np.uint8)
        qstride = (rec.max_len + 15) & ~15
        made = dec == 0
        nm = int(made.sum())
        self.times["emit_fetch"] = time.time() - t0
        t0 = time.time()
        names, name_off = dcs_names(bam, t_rec[made], p_rec[made])
        self.times["emit_names"] = time.time() - t0
        t0 = time.time()
        sp = _new_specs(nm, t_rec[made], np.arange(nm), vslot[made], meta, qstride)
        write_bam(outfile, bam, it, sp, [bam], names, name_off, cons_seq, cons_qual, level, sink=sink)
        single = dec == 1
        ss = make_specs(int(single.sum()))
        ss["kind"] = N.OUT_RAW
        ss["src_rec"] = t_rec[single]
        write_bam(singleton_path, bam, it, ss, [bam], level=level, sink=sink)
        self.times["emit_write"] = time.time() - t0
        t0 = time.time()
        part = dict(counters=c, dcs=nm, sscs_singletons=int(single.sum()))
        if side:
            dcs_side(outfile, part, start_time, verbose)
        self.times["emit_side"] = time.time() - t0
        return part


def dcs_side(outfile, part, start_time, verbose=True):
    """DCS_maker.py:286-309: the stats.txt block and the time tracker line (one run or summed shards)."""
    c = part["counters"]
    if re.search(r'dcs\.sc', outfile) is not None:
        dcs_header, sc_header = "DCS - Singleton Correction", " SC"
    else:
        dcs_header, sc_header = "DCS", ""
    prefix = outfile.split('.dcs')[0]
    summary = '''# === {} ===
SSCS{} - Total reads: {}
SSCS{} - Unmapped reads: {}
SSCS{} - Secondary/Supplementary reads: {}
DCS{} reads: {}
SSCS{} singletons: {} \n'''.format(dcs_header, sc_header, c["COUNTER"], sc_header, c["UNMAPPED_MATE"],
                                       sc_header, 0, sc_header, part["dcs"], sc_header, part["sscs_singletons"])
    with open('{}.stats.txt'.format(prefix), 'a') as st:
        st.write(summary)
    if verbose:
        print(summary)
    with open('{}.time_tracker.txt'.format(prefix), 'a') as tt:
        tt.write('DCS: ')
        tt.write(str((time.time() - start_time) / 60) + '\n')
    return dict(counters=c, dcs=part["dcs"], sscs_singletons=part["sscs_singletons"])


def run_dcs(infile, outfile, bedfile=None, engine=None, level=6, verbose=True, sink=None, bam=None):
    """DCS_maker.main (DCS_maker.py:130-317)."""
    start_time = time.time()
    run = DCSRun(engine or get_engine(), infile, bedfile, bam=bam)
    try:
        return run.emit(outfile, level, verbose, start_time, sink=sink)
    finally:
        run.close()


# ---------------------------------------------------------------- SC
class SCRun(object):
    """Device side of singleton_correction.main (singleton_correction.py:118-345)."""

    def __init__(self, eng, singleton, bedfile=None, shard=None, src=None, sscs_run=None, bam=None, xbam=None):
        """src: (interner, (singleton bam, records, stream), (sscs bam, records, stream)) already decoded
        (sharded.py); singleton then only names the outputs.  sscs_run: the DCSRun resident on this
        sample's sorted SSCS file (the file SC reads as its SSCS side) without a bed file: its grouping
        is SC's SSCS-side grouping (one chromosome scope, so scope_by_run changes nothing), and SC
        joins against it instead of grouping the file again."""
        self.eng = eng
        self.base = singleton.split('.singleton')[0]
        rest = singleton.split('.singleton')[1]
        self.x_shared = sscs_run is not None
        if sscs_run is not None:
            if bedfile is not None or shard is not None or len(set(sscs_run.stream.region_run.tolist())) > 1:
                raise ValueError("an SSCS grouping is shared only for one chromosome scope (no bed file)")
            self.it = sscs_run.it
            self.sbam = bam if bam is not None else Bam(singleton)
            self.srec = self.sbam.decode(self.it, MODE_DUPLEX)
            self.sstream = _stream(self.sbam, self.srec, None)
            self.xbam, self.xrec, self.xstream = sscs_run.bam, sscs_run.rec, sscs_run.stream
            self.swap = self.it.swap_table()
            self.ts = eng.upload(self.srec)
            self.tx, self.gx = sscs_run.table, sscs_run.g
            self.gs = eng.read_bam(self.ts, self.sstream, delim_filter=0, badread_file=0, scope_by_run=0)
            eng.singleton_correction(self.gs, self.gx, self.swap)
            return
        if src is not None:
            self.it, (self.sbam, self.srec, self.sstream), (self.xbam, self.xrec, self.xstream) = src
        else:
            self.it = Interner()
            self.sbam = bam if bam is not None else Bam(singleton)
            self.xbam = xbam if xbam is not None else Bam('{}.sscs{}'.format(self.base, rest))
            self.srec = self.sbam.decode(self.it, MODE_DUPLEX)
            self.xrec = self.xbam.decode(self.it, MODE_DUPLEX)
            if shard is None:
                self.sstream = _stream(self.sbam, self.srec, bedfile)
                self.xstream = _stream(self.xbam, self.xrec, bedfile)
            else:
                self.sstream = shard(self.sbam, self.srec)
                self.xstream = shard(self.xbam, self.xrec)
        self.swap = self.it.swap_table()
        self.ts = eng.upload(self.srec)
        self.tx = eng.upload(self.xrec)
        self.gs = eng.read_bam(self.ts, self.sstream, delim_filter=0, badread_file=0, scope_by_run=0)
        self.gx = eng.read_bam(self.tx, self.xstream, delim_filter=0, badread_file=0, scope_by_run=1)
        eng.singleton_correction(self.gs, self.gx, self.swap)

    @property
    def n_input(self):
        return self.sstream.n + self.xstream.n

    def step(self, seed):
        self.eng.rerun(self.gs, seed)
        if not self.x_shared:   # a shared SSCS grouping is re-run by its DCS stage
            self.eng.rerun(self.gx, seed)
        self.eng.singleton_correction(self.gs, self.gx, self.swap)

    def close(self):
        if self.gs is not None:
            self.eng.free_group(self.gs)
            self.eng.free_table(self.ts)
            if not self.x_shared:
                self.eng.free_group(self.gx)
                self.eng.free_table(self.tx)
            self.gs = None

    def emit(self, level=6, verbose=True, side=True, sink=None):
        eng, gs, it, sbam, base = self.eng, self.gs, self.it, self.sbam, self.base
        c = eng.counters(gs)
        dec = eng.fetch(gs, "dec", np.int32)
        t_rec = eng.fetch(gs, "t_rec", np.int32)
        vslot = eng.fetch(gs, "vslot", np.int32)
        q_ckey = eng.fetch(gs, "q_ckey", np.int32).reshape(-1, 9)
        meta = eng.fetch(gs, "vote_meta", np.int32).reshape(-1, 5)
        cons_seq = eng.fetch(gs, "cons_seq", np.uint8)
        cons_qual = eng.fetch(gs, "cons_qual", np.uint8)
        qstride = (max(self.srec.max_len, self.xrec.max_len) + 15) & ~15
        outs = {}
        for code, name in ((0, "sscs.correction"), (1, "singleton.correction")):
            m = dec == code
            k = int(m.sum())
            names, name_off = csn_names(it, q_ckey[m], np.ones(k, np.int64))
            sp = _new_specs(k, t_rec[m], np.arange(k), vslot[m], meta, qstride)
            write_bam('{}.{}.bam'.format(base, name), sbam, it, sp, [sbam], names, name_off, cons_seq, cons_qual,
                      level, sink=sink)
            outs[name] = k
        m = dec == 2
        us = make_specs(int(m.sum()))
        us["kind"] = N.OUT_RAW
        us["src_rec"] = t_rec[m]
        write_bam('{}.uncorrected.bam'.format(base), sbam, it, us, [sbam], level=level, sink=sink)
        part = dict(counters=c, processed=int((dec < 3).sum()), sscs_correction=outs["sscs.correction"],
                    singleton_correction=outs["singleton.correction"], uncorrected=int(m.sum()))
        if side:
            sc_side(base, part, verbose)
        return part


def sc_side(base, part, verbose=True):
    """singleton_correction.py:321-345: the stats.txt block (one run or summed shards).  Raises
    ZeroDivisionError on an empty singleton file, as the reference does."""
    singleton_counter = part["counters"]["COUNTER"]
    sscs_dup, sing_dup = part["sscs_correction"], part["singleton_correction"]
    sscs_frac = (sscs_dup / singleton_counter) * 100          # ZeroDivisionError as in the reference
    sing_frac = (sing_dup / singleton_counter) * 100
    summary = '''# === Singleton Correction ===
Total singletons: {}
Singleton Correction by SSCS: {}
% Singleton Correction by SSCS: {}
Singleton Correction by Singletons: {}
% Singleton Correction by Singletons : {}
Uncorrected Singletons: {} \n'''.format(part["processed"], sscs_dup, sscs_frac, sing_dup, sing_frac,
                                            part["uncorrected"])
    with open('{}.stats.txt'.format(base), 'a') as st:
        st.write(summary)
    if verbose:
        print(summary)
    return dict(counters=part["counters"], sscs_correction=sscs_dup, singleton_correction=sing_dup,
                uncorrected=part["uncorrected"])


def run_sc(singleton, bedfile=None, engine=None, level=6, verbose=True, sscs_run=None, sink=None, bam=None,
           xbam=None):
    """singleton_correction.main (singleton_correction.py:118-345)."""
    run = SCRun(engine or get_engine(), singleton, bedfile, sscs_run=sscs_run, bam=bam, xbam=xbam)
    try:
        return run.emit(level, verbose, sink=sink)
    finally:
        run.close()
