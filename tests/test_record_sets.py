"""Rank-local record sets of the multi-GPU driver (libccio, CPU): reading a block of bed regions
through the BAI must give exactly the records the whole-file region stream holds (pysam fetch +
consensus_helper.py:391-396), in file order; packing and combining records must keep their bytes
and the stable sort orders of the samtools stand-in."""
import os

import numpy as np
import pytest

import pysam
from parity import GOLDEN

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DATA = os.path.join(ROOT, "consensuscruncher_amd", "data")


def _sample(tmp_path, n_pairs=30_000, seed=31):
    from consensuscruncher_amd import synth
    from consensuscruncher_amd.engine import index_bam
    contigs = synth.band_contigs("hg38_cytoBand.txt")
    batch = synth.generate(n_pairs, seed=synth.SEED_BASE + seed, contigs=contigs, transloc_frac=0.02)
    bam = str(tmp_path / "s.bam")
    synth.write_bam_native(batch, bam)
    index_bam(bam)
    return bam, os.path.join(DATA, "hg38_cytoBand.txt")


def _regions(bam, bedfile):
    from consensuscruncher_amd.consensus_helper import region_list
    from consensuscruncher_amd.engine import Bam
    names = {n: i for i, (n, _) in enumerate(Bam(bam).refs)}
    return [(names[c], s, e) for _, c, s, e in region_list(bedfile)]


@pytest.mark.parametrize("world", [1, 3, 8])
def test_open_regions_equals_whole_file_stream(tmp_path, world):
    from consensuscruncher_amd.engine import Bam, Interner, bed_stream
    from consensuscruncher_amd.shard import plan_blocks
    bam, bed = _sample(tmp_path)
    whole = Bam(bam)
    rec = whole.decode(Interner(), 0, "|")
    st = bed_stream(rec, whole.refs, bed)
    regs = _regions(bam, bed)
    blocks = plan_blocks(np.bincount(st.region, minlength=len(regs)), world)
    lines = pysam.sam_lines(bam)
    got_all = []
    for lo, hi in blocks:
        t, b, e = zip(*regs[lo:hi]) if hi > lo else ((), (), ())
        sub = Bam.open_regions(bam, t, b, e)
        want = np.sort(st.rec[(st.region >= lo) & (st.region < hi)])
        part = str(tmp_path / ("part%d.bam" % lo))
        sub.write_all(part, 1)
        assert pysam.sam_lines(part) == [lines[i] for i in want]   # same records, file order
        got_all.extend(want.tolist())
    assert sorted(got_all) == sorted(st.rec.tolist())


def test_pack_and_combine(tmp_path):
    from consensuscruncher_amd.engine import Bam, sort_bam
    src = os.path.join(GOLDEN, "basic", "expected", "sscs.bam")
    b = Bam(src)
    lines = pysam.sam_lines(src)
    rng = np.random.default_rng(5)
    idx = rng.permutation(b.n)
    a, c = idx[: b.n // 3], idx[b.n // 3:]
    blob_a, blob_c = b.pack(a), b.pack(c)
    # unsorted: blob order kept, origin = concatenation index
    u = Bam.combine([], [blob_a, blob_c], key=2, tmpl=b)
    u.write_all(str(tmp_path / "u.bam"), 1)
    assert pysam.sam_lines(str(tmp_path / "u.bam")) == [lines[i] for i in np.concatenate([a, c])]
    assert u.origin().tolist() == list(range(b.n))
    # key 1: the samtools stand-in's stable sort of the concatenation (ccio_sort_bam)
    s = Bam.combine([u], [], key=1)
    s.write_all(str(tmp_path / "s.bam"), 1)
    sort_bam(str(tmp_path / "u.bam"), str(tmp_path / "ref.bam"), 1)
    assert pysam.sam_lines(str(tmp_path / "s.bam")) == pysam.sam_lines(str(tmp_path / "ref.bam"))
    perm = s.origin()
    assert sorted(perm.tolist()) == list(range(b.n))
    t, p, mt, mp, f = s.cores()
    key = (t.astype(np.int64) << 32) + p
    assert np.all(np.diff(key) >= 0)
