"""GPU parity at sizes and shapes the golden fixtures cannot reach, against the C++ oracle
(oracle/cc_oracle.cpp, pinned to the reference by tests/test_oracle_native.py) on the same seeded
synthetic BAM.  Every output BAM must hold the oracle's records IN FILE ORDER; stats.txt and
read_families.txt byte for byte.

  c2_600k      the C2 model (NNT barcodes, mean family 4, 2x150) at ~600 k reads, contig scaled to
               keep C2's read density: many scan tiles, vote waves, planned re-runs
  c4_families  C4 shape: Zipf families up to 5000 members on a few loci (the exact per-family vote,
               position groups deeper than 64 through the tag sort, large-family modes)
  hg38_bands   hg38 contigs at real lengths, the bundled hg38_cytoBand.txt as the bed (chrM after
               chr9 at line 812, chrM's empty arm), translocations across chromosomes
  hg38_noalt   the bundled hg38_noAlt_cytoBand.txt: chrUn_* / *_random contigs split by rsplit('_')
  c4_fieldnoise  C4 families with a third of the reads carrying a random mapq (0..254) and tlen:
               the large-family modes through the LDS hash (k_big_final), past its 256 slots
               (the wave_mode fallback), Counter ties broken first-seen
  long_reads   2x1100 reads: more than 64 SWAR chunks, so every family takes the split vote
  ident_transloc  three contigs without a bed (the identity stream's tiled mate search), 3%
               translocated mates and pair quirks: mates far outside the staged window take the
               global bucket walk, long pairs the exact long-pair table
  ident_dense  150 loci with Zipf families up to 60 members, no bed: ~1700 position groups of 41-64
               records and ~800 deeper ones, straddling the mate search's 1024-entry tiles and
               their 512-entry halo and the ranking's 256-record tiles
  deep_bad     2 loci, families up to 6000 members, 20% bad reads: position groups of thousands of
               records searched and ranked per group (k_deep_qsort / k_deep_rank), some holding more
               records than read ends
"""
import numpy as np
import os

import pytest

from parity import assert_same_in_order

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DATA = os.path.join(ROOT, "consensuscruncher_amd", "data")
OUTS = ("sscs", "singleton", "badreads", "dcs", "sscs_singleton", "sscs_correction", "singleton_correction",
        "uncorrected", "sscs_sc", "dcs_sc", "sscs_sc_singleton", "all_unique")


def band_contigs(name):
    ends = {}
    for line in open(os.path.join(DATA, name)):
        c = line.split("\t")
        ends[c[0]] = max(ends.get(c[0], 0), int(c[2]))
    return tuple(ends.items())


CASES = {
    "c2_600k": dict(n_pairs=300_000, seed=601, contigs=(("chr1", 3_000_000),)),
    "c4_families": dict(n_pairs=60_000, seed=602, contigs=(("chr1", 2_000_000),), loci=5, zipf_s=1.9,
                        max_fam=5000),
    "hg38_bands": dict(n_pairs=40_000, seed=603, contigs="hg38_cytoBand.txt", transloc_frac=0.01, bed=True),
    "c4_fieldnoise": dict(n_pairs=30_000, seed=605, contigs=(("chr1", 2_000_000),), loci=3, zipf_s=1.9,
                          max_fam=3000, noise=True),
    "long_reads": dict(n_pairs=4_000, seed=606, read_len=1100, contigs=(("chr1", 1_000_000),)),
    "ident_transloc": dict(n_pairs=60_000, seed=607, contigs=(("chr1", 600_000), ("chr2", 400_000), ("chr3", 300_000)),
                           transloc_frac=0.03, quirk_frac=0.01),
    "ident_dense": dict(n_pairs=100_000, seed=608, contigs=(("chr1", 400_000),), loci=150, zipf_s=1.3, max_fam=60),
    # two loci, Zipf families up to 6000 and a fifth of the reads bad: position groups of thousands of
    # records (the deep paths: k_deep_qsort / k_deep_rank), some with more records than read ends
    "deep_bad": dict(n_pairs=60_000, seed=609, contigs=(("chr1", 300_000),), loci=2, zipf_s=1.4, max_fam=6000,
                     bad_frac=0.2),
    "hg38_noalt": dict(n_pairs=30_000, seed=604, contigs="hg38_noAlt_cytoBand.txt", transloc_frac=0.01, bed=True),
}


@pytest.fixture(scope="module")
def engine():
    from consensuscruncher_amd.engine import Engine
    e = Engine(0)
    yield e
    e.close()


@pytest.mark.parametrize("name", sorted(CASES))
def test_large_matches_native_oracle(name, engine, tmp_path):
    import cc_oracle_native as O
    from consensuscruncher_amd import synth
    from consensuscruncher_amd.pipeline import consensus_pipeline
    kw = dict(CASES[name])
    n = kw.pop("n_pairs")
    seed = synth.SEED_BASE + kw.pop("seed")
    bedfile = "False"
    if kw.pop("bed", False):
        bedfile = os.path.join(DATA, kw["contigs"])
        kw["contigs"] = band_contigs(kw["contigs"])
    noise = kw.pop("noise", False)
    batch = synth.generate(n, seed=seed, **kw)
    if noise:
        rng = np.random.default_rng(seed)
        pick = rng.random(len(batch.mapq)) < 0.33
        batch.mapq[pick] = rng.integers(0, 255, int(pick.sum()), dtype=np.uint8)
        batch.tlen[pick] = rng.integers(-5000, 5000, int(pick.sum()), dtype=np.int32)
    bam = str(tmp_path / "sample.bam")
    synth.write_bam_native(batch, bam)
    ours = consensus_pipeline(bam, str(tmp_path / "gpu"), engine=engine, bedfile=bedfile, level=1)
    ref = O.consensus_pipeline(bam, str(tmp_path / "oracle"), bedfile=bedfile)
    errs = []
    for k in OUTS:
        try:
            assert_same_in_order(ours[k], ref[k], "%s/%s" % (name, k))
        except AssertionError as e:
            errs.append(str(e))
    assert not errs, "\n".join(errs)
    for k in ("stats", "read_families"):
        assert open(ours[k]).read() == open(ref[k]).read(), k
    if name == "c4_families":
        sizes = [int(x.split("\t")[0]) for x in open(ref["read_families"]).read().split("\n")[1:]]
        assert max(sizes) >= 1000, "the case must hold families of 1000+ members"
