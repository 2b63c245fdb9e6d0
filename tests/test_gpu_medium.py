"""GPU parity at sizes past the small-input code paths (many scan tiles, many vote
workgroups, families above the 64-member batched-vote limit, several contigs and
translocated pairs): the whole consensus pipeline against the oracle
(oracle/cc_oracle.py, itself pinned to the reference by tests/golden) on the same
seeded synthetic BAM.  Outputs must match record for record; stats and family
tables byte for byte."""
import os

import pytest

from parity import assert_same_records

pytestmark = pytest.mark.gpu

OUTS = ("sscs", "singleton", "badreads", "dcs", "sscs_singleton", "sscs_correction", "singleton_correction",
        "uncorrected", "sscs_sc", "dcs_sc", "sscs_sc_singleton", "all_unique")

MEDIUM = {
    # ~60k reads over three contigs with translocations and reference quirks
    "multi_contig": dict(n_pairs=30_000, seed=501, contigs=(("chr1", 6_000_000), ("chr2", 4_000_000), ("chr3", 500_000)),
                         transloc_frac=0.01, quirk_frac=0.002),
    # deep targeted-panel shape: Zipf families, many above 64 members
    "deep_loci": dict(n_pairs=1_500, seed=502, contigs=(("chr1", 2_000_000),), loci=6, zipf_s=1.3, max_fam=300),
}


@pytest.fixture(scope="module")
def engine():
    from consensuscruncher_amd.engine import Engine
    e = Engine(0)
    yield e
    e.close()


@pytest.mark.parametrize("name", sorted(MEDIUM))
def test_medium_matches_oracle(name, engine, tmp_path):
    import cc_oracle
    from consensuscruncher_amd import synth
    from consensuscruncher_amd.pipeline import consensus_pipeline
    kw = dict(MEDIUM[name])
    n = kw.pop("n_pairs")
    seed = synth.SEED_BASE + kw.pop("seed")
    batch = synth.generate(n, seed=seed, **kw)
    bam = str(tmp_path / "sample.bam")
    synth.write_bam_native(batch, bam)
    ours = consensus_pipeline(bam, str(tmp_path / "gpu"), engine=engine)
    ref = cc_oracle.consensus_pipeline(bam, str(tmp_path / "oracle"))
    errs = []
    for k in OUTS:
        if k not in ref:
            continue
        try:
            assert_same_records(ours[k], ref[k], "%s/%s" % (name, k))
        except AssertionError as e:
            errs.append(str(e))
    assert not errs, "\n".join(errs)
    for k in ("stats", "read_families"):
        if k in ref:
            assert open(ours[k]).read() == open(ref[k]).read(), k
