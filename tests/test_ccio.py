"""Host BAM I/O (libccio) against the independent pysam shim."""
import os

import numpy as np
import pytest

import pysam
import synthbam
from consensuscruncher_amd import native as N
from consensuscruncher_amd import synth
from consensuscruncher_amd.engine import (MODE_DUPLEX, MODE_SSCS, Bam, Interner, bed_stream, make_specs,
                                          merge_bams, sort_bam, write_bam)
from samtools_shim import samtools_merge, samtools_sort_index


@pytest.fixture(scope="module")
def small_bam(tmp_path_factory):
    d = tmp_path_factory.mktemp("ccio")
    b = synth.generate(600, seed=7, contigs=(("chr1", 100_000), ("chr2", 80_000)), transloc_frac=0.05)
    path = str(d / "in.bam")
    synthbam.write_batch(b, path)
    return path


def _seq_of(rec, i):
    L = int(rec.lseq[i])
    o = int(rec.pay_off[i])
    nib = rec.payload[o + ((L + 15) & ~15):]
    return "".join("=ACMGRSVTWYHKDBN"[(int(nib[k >> 1]) >> (4 * (1 - (k & 1)))) & 15] for k in range(L))


@pytest.mark.parametrize("mode", [MODE_SSCS, MODE_DUPLEX])
def test_decode_matches_shim(small_bam, mode):
    it = Interner()
    bam = Bam(small_bam)
    rec = bam.decode(it, mode, "|")
    recs = list(pysam.AlignmentFile(small_bam).fetch(until_eof=True))
    assert bam.n == len(recs)
    for i, x in enumerate(recs):
        assert (rec.tid[i], rec.pos[i], rec.flag[i], rec.mtid[i], rec.mpos[i], rec.tlen[i], rec.mapq[i]) == (
            x.reference_id, x.reference_start, x.flag, x.next_reference_id, x.next_reference_start,
            x.template_length, x.mapping_quality)
        assert it.get(1, rec.cigar_id[i]) == str(x.cigarstring)
        assert bytes(rec.qn_blob[rec.qn_off[i]:rec.qn_off[i] + rec.qn_len[i]]).decode() == x.query_name
        o = int(rec.pay_off[i])
        assert bytes(rec.payload[o:o + rec.lseq[i]]) == bytes(x.query_qualities)
        assert _seq_of(rec, i) == x.query_sequence
        assert rec.qlen[i] == (x.infer_query_length() if x.cigartuples else -1)
        if mode == MODE_SSCS:
            if "|" in x.query_name:
                assert it.get(0, rec.bc_id[i]) == x.query_name.split("|")[1]
            else:
                assert rec.rflags[i] & N.RF_BAD_SPACER
        else:
            assert it.get(0, rec.bc_id[i]) == x.query_name.split("_")[0]
        assert it.get(2, rec.rg_id[i]) == x.get_tag("RG")


def test_swap_table_is_duplex_tag_barcode_rule():
    from consensuscruncher_amd.consensus_helper import swap_barcode
    it = Interner()
    for s in ("AC.GT", "ACG.T", "TTTG", "ACGTA", "A.B.C"):
        it.intern(0, s)
    sw = it.swap_table()
    for i in range(it.size(0)):
        assert it.get(0, sw[i]) == swap_barcode(it.get(0, i))


def test_write_raw_rename_new_roundtrip(small_bam, tmp_path):
    it = Interner()
    bam = Bam(small_bam)
    bam.decode(it, MODE_SSCS, "|")
    recs = list(pysam.AlignmentFile(small_bam).fetch(until_eof=True))
    sp = make_specs(3)
    sp["kind"] = [N.OUT_RAW, N.OUT_RENAME, N.OUT_NEW]
    sp["src_rec"] = [0, 1, 2]
    sp["name_id"] = [-1, 0, 1]
    names = np.frombuffer(b"renamed:1NEW:7", np.uint8).copy()
    off = np.array([0, 9, 14], np.int64)
    L = recs[2].query_length
    cq = np.full(16 * ((L + 15) // 16), 33, np.uint8)
    cs = np.zeros(len(cq) // 2, np.uint8)
    cs[:] = 0x12   # A C A C ...
    sp["cons_len"][2] = L
    sp["flag"][2] = 99
    sp["mapq"][2] = 42
    sp["tlen"][2] = -5
    sp["rg_id"][2] = 0
    out = str(tmp_path / "o.bam")
    write_bam(out, bam, it, sp, [bam], names, off, cs, cq)
    got = list(pysam.AlignmentFile(out).fetch(until_eof=True))
    assert pysam.canonical_sam_line(got[0]) == pysam.canonical_sam_line(recs[0])
    r1 = recs[1]
    r1.query_name = "renamed:1"
    assert pysam.canonical_sam_line(got[1]) == pysam.canonical_sam_line(r1)
    g = got[2]
    assert (g.query_name, g.flag, g.mapping_quality, g.template_length) == ("NEW:7", 99, 42, -5)
    assert g.reference_id == recs[2].reference_id and g.cigarstring == recs[2].cigarstring
    assert g.query_sequence == ("AC" * L)[:L] and list(g.query_qualities) == [33] * L
    assert g.get_tag("RG") == it.get(2, 0) and len(g.get_tags()) == 1


def test_sort_and_merge_match_samtools_standin(small_bam, tmp_path):
    import shutil
    a = str(tmp_path / "a.bam")
    shutil.copy(small_bam, a)
    # shuffle records to make the sort do work
    h, raws = pysam.read_bam_file(a)
    rng = np.random.default_rng(3)
    raws = [raws[i] for i in rng.permutation(len(raws))]
    pysam.write_bam_file(a, h, raws)
    b = str(tmp_path / "b.bam")
    shutil.copy(a, b)
    sort_bam(a, str(tmp_path / "a.sorted.bam"))
    ref = samtools_sort_index(b)
    assert pysam.sam_lines(str(tmp_path / "a.sorted.bam")) == pysam.sam_lines(ref)
    m1 = str(tmp_path / "m1.bam")
    m2 = str(tmp_path / "m2.bam")
    merge_bams(m1, [ref, ref])
    samtools_merge(m2, ref, ref)
    assert pysam.sam_lines(m1) == pysam.sam_lines(m2)


def test_bed_stream_is_fetch_semantics(small_bam, tmp_path):
    bed = str(tmp_path / "r.bed")
    with open(bed, "w") as f:
        f.write("chr2\t0\t40000\tp1\tx\nchr1\t0\t50000\tp1\tx\nchr1\t50000\t100000\tq1\tx\nchr2\t40000\t80000\tq1\tx\n")
    it = Interner()
    bam = Bam(small_bam)
    rec = bam.decode(it, MODE_SSCS, "|")
    st = bed_stream(rec, bam.refs, bed)
    shim = pysam.AlignmentFile(small_bam)
    raws = shim._raw
    want = []
    import cc_oracle
    for k, chrom, s, e in cc_oracle.regions_of(bed):
        for r in shim.fetch(chrom, s, e):
            if s <= r.reference_start <= e:
                want.append(r.query_name + str(r.flag) + str(r.reference_start))
    got = []
    for i in st.rec:
        got.append(bam.qname(i) + str(rec.flag[i]) + str(rec.pos[i]))
    assert got == want
    assert list(st.region_run) == [1, 2, 2, 3]


def test_csn_names_format(tmp_path):
    """ccio_format_csn_names (parallel) against sscs_qname's text (consensus_helper.py:240-247) +
    ':' + the family size (SSCS_maker.py:327), on random fields incl. negative coordinates."""
    from consensuscruncher_amd.engine import csn_names
    it = Interner()
    bcs = ["AC.GT", "TTAA", "N.N", "GATTACA.CC"]
    cigs = ["150M", "5S145M", "None", "30M2I118M"]
    bid = [it.intern(0, b) for b in bcs]
    cid = [it.intern(1, c) for c in cigs]
    rng = np.random.default_rng(5)
    n = 50_000
    f9 = np.zeros((n, 9), np.int32)
    f9[:, 0] = rng.choice(bid, n)
    f9[:, 1:5] = rng.integers(-3, 2 ** 31 - 1, (n, 4))
    f9[:, 5] = rng.choice(cid, n)
    f9[:, 6] = rng.choice(cid, n)
    f9[:, 7] = rng.integers(0, 3, n)
    f9[:, 8] = rng.integers(0, 2 ** 32 - 1, n, dtype=np.uint32).view(np.int32)
    suf = rng.integers(1, 10 ** 12, n)
    blob, off = csn_names(it, f9, suf)
    for i in list(range(200)) + list(rng.integers(0, n, 500)):
        f = f9[i]
        want = "%s_%d_%d_%d_%d_%s_%s_%s_%d:%d" % (bcs[bid.index(f[0])], f[1], f[2], f[3], f[4], cigs[cid.index(f[5])],
                                                  cigs[cid.index(f[6])], ("pos", "neg", "None")[f[7]],
                                                  int(np.uint32(f[8])), suf[i])
        assert bytes(blob[off[i]:off[i + 1]]).decode() == want


def test_dcs_names_format(tmp_path):
    """ccio_format_dcs_names (parallel) against dcs_consensus_tag (DCS_maker.py:60-96, the oracle's
    restatement) on SSCS-style qnames of both strands."""
    import cc_oracle
    from consensuscruncher_amd.engine import dcs_names
    rng = np.random.default_rng(9)
    b = synth.generate(1500, seed=11, contigs=(("chr1", 1_000_000),))
    header, recs = synthbam.batch_records(b)
    for r in recs:
        bc = "".join(rng.choice(list("ACGT"), 2)) + "." + "".join(rng.choice(list("ACGT"), 2))
        st = rng.choice(["pos", "neg"])
        r.query_name = "%s_0_%d_0_%d_150M_150M_%s_%d:%d" % (bc, rng.integers(0, 10 ** 6), rng.integers(0, 10 ** 6), st,
                                                            rng.integers(100, 900), rng.integers(1, 50))
    path = str(tmp_path / "n.bam")
    pysam.write_bam_file(path, header, recs, 1)
    bam = Bam(path)
    n = bam.n
    qn = [bam.qname(i) for i in range(n)]
    a = rng.integers(0, n, 4000)
    c = rng.integers(0, n, 4000)
    blob, off = dcs_names(bam, a, c)
    for k in range(4000):
        assert bytes(blob[off[k]:off[k + 1]]).decode() == cc_oracle.duplex_name(qn[a[k]], qn[c[k]])


def test_fused_sorted_write_matches_sort_index(small_bam, tmp_path):
    """ccio_write_bam_ex with CCIO_W_SORT | CCIO_W_INDEX (the orchestrator's fused sort_index) writes
    the same records and the same .bai as writing the file, then sort + index (ConsensusCruncher.py:
    10-34); the kept handle holds the written records; merge_kept equals merge_bams of the files."""
    from consensuscruncher_amd.engine import Sink, index_bam, merge_kept
    it = Interner()
    bam = Bam(small_bam)
    bam.decode(it, MODE_SSCS, "|")
    rng = np.random.default_rng(3)
    idx = rng.permutation(bam.n)
    sp = make_specs(len(idx))
    sp["kind"] = N.OUT_RAW
    sp["src_rec"] = idx
    plain = str(tmp_path / "a.bam")
    write_bam(plain, bam, it, sp, [bam], level=1)
    sort_bam(plain, str(tmp_path / "a.sorted.bam"), 1)
    index_bam(str(tmp_path / "a.sorted.bam"))
    fused = str(tmp_path / "f" / "a.bam")
    os.makedirs(os.path.dirname(fused))
    sink = Sink(fused=[fused], keep=[fused])
    out = write_bam(fused, bam, it, sp, [bam], level=1, sink=sink)
    assert out == str(tmp_path / "f" / "a.sorted.bam") and not os.path.exists(fused)
    assert pysam.sam_lines(out) == pysam.sam_lines(str(tmp_path / "a.sorted.bam"))
    # the index of the fused write is computed from its own BGZF members: it must index the same
    # records (block layouts agree, both written at level 1 by the same writer)
    assert open(out + ".bai", "rb").read() == open(str(tmp_path / "a.sorted.bam.bai"), "rb").read()
    kept = sink.take(out)
    assert kept.n == bam.n
    m1 = str(tmp_path / "m1.bam")
    merge_bams(m1, [out, out], 1)
    m2 = str(tmp_path / "m2.sorted.bam")
    merge_kept(m2, [kept, kept], 1, keep=False)
    assert pysam.sam_lines(m1) == pysam.sam_lines(m2)
    assert os.path.exists(m2 + ".bai")


@pytest.mark.parametrize("scan_min", ["1", "4096", "100000"])
def test_parallel_record_scan(small_bam, tmp_path, monkeypatch, scan_min):
    """ccio_bam_open's record-offset walk in pieces (scan_records: pieces started at chained plausible
    records, joined where the chains meet) gives the serial walk's records, whatever the cut points."""
    import ctypes as C
    big = str(tmp_path / "big.bam")
    b = synth.generate(20_000, seed=21, contigs=(("chr1", 500_000),))
    synthbam.write_batch(b, big)
    ref = Bam(big, nthreads=1)
    monkeypatch.setenv("CCIO_SCAN_MIN", scan_min)
    for nt in (2, 3, 8, 13):
        x = Bam(big, nthreads=nt)
        assert x.n == ref.n
        for i in list(range(0, ref.n, 997)) + [ref.n - 1]:
            assert x.qname(i) == ref.qname(i)
        t1, p1, _, _, f1 = x.cores()
        t0, p0, _, _, f0 = ref.cores()
        assert (t1 == t0).all() and (p1 == p0).all() and (f1 == f0).all()


def test_async_writes_equal_synchronous(small_bam, tmp_path):
    """CCIO_W_ASYNC (the pipeline's background compression): the files, indexes and kept records equal
    the synchronous write's; a reader of the path waits for the pending write; ccio_flush reports a
    failed background write."""
    from consensuscruncher_amd.engine import Sink, flush_writes, merge_kept
    it = Interner()
    bam = Bam(small_bam)
    bam.decode(it, MODE_SSCS, "|")
    rng = np.random.default_rng(4)
    sp = make_specs(bam.n)
    sp["kind"] = N.OUT_RAW
    sp["src_rec"] = rng.permutation(bam.n)
    outs = {}
    for mode in (False, True):
        d = tmp_path / ("async" if mode else "sync")
        os.makedirs(str(d))
        path = str(d / "a.bam")
        sink = Sink(fused=[path], keep=[path], async_writes=mode)
        out = write_bam(path, bam, it, sp, [bam], level=1, sink=sink)
        kept = sink.take(out)
        # read back at once: ccio_bam_open waits for the background write of this path
        again = Bam(out)
        m = str(d / "m.sorted.bam")
        merge_kept(m, [kept, again], 1, keep=False, async_writes=mode)
        flush_writes()
        outs[mode] = [open(p, "rb").read() for p in (out, out + ".bai", m, m + ".bai")]
        assert kept.n == again.n == bam.n
    assert outs[False] == outs[True]
    # a background write that fails surfaces at the flush
    sink = Sink(fused=[str(tmp_path / "nodir" / "x.bam")], async_writes=True)
    write_bam(str(tmp_path / "nodir" / "x.bam"), bam, it, sp, [bam], level=1, sink=sink)
    with pytest.raises(IOError):
        flush_writes()
    flush_writes()   # nothing pending any more
