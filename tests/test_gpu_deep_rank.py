"""Deep position groups (more than 64 records at one position: config C4's shape) ranked in place
(k_deep_fam, k_deep_emit, k_deep_sortfam), no global sort: the whole pipeline against the oracle
(oracle/cc_oracle.py), record for record, with the kernel scopes showing which path ran, and the
sorted fallback (CC_DEEP_SORT=1) the same.  Cases: Zipf families up to 300 members over a few loci,
the same records with each position's ties shuffled (families out of end order: k_deep_sortfam),
and one position holding more than k_deep_fam's 512 families (that pass takes the sorted path)."""
import os

import pytest

from parity import assert_same_records

pytestmark = pytest.mark.gpu

OUTS = ("sscs", "singleton", "badreads", "dcs", "sscs_singleton", "sscs_correction", "singleton_correction",
        "uncorrected", "sscs_sc", "dcs_sc", "sscs_sc_singleton", "all_unique")

CASES = {
    # Zipf families up to 300 members at 4 loci, records at one position in random order: families
    # out of end order (k_deep_sortfam)
    "zipf_loci": dict(n_pairs=4_000, seed=611, contigs=(("chr1", 1_000_000),), loci=4, zipf_s=1.2, max_fam=300),
    # the same shape with ties in generation order (samtools' stable sort of name-grouped input):
    # record order is end order (k_deep_emit alone)
    "zipf_loci_input_ties": dict(n_pairs=4_000, seed=613, contigs=(("chr1", 1_000_000),), loci=4, zipf_s=1.2,
                                 max_fam=300, ties="input"),
    # every molecule's left read at one position: ~2,600 families there (over the 512 limit)
    "one_position": dict(n_pairs=10_000, seed=612, contigs=(("chr1", 200_000),), windows=[(0, 50_000, 50_200)]),
}


@pytest.fixture(scope="module")
def engine():
    from consensuscruncher_amd.engine import Engine
    e = Engine(0)
    yield e
    e.close()


def _run(engine, bam, out, deep_fam):
    """deep_fam False: CC_DEEP_SORT=1, the sorted deep-group path (the fallback)."""
    from consensuscruncher_amd.pipeline import consensus_pipeline
    old = os.environ.get("CC_DEEP_SORT")
    if deep_fam:
        os.environ.pop("CC_DEEP_SORT", None)
    else:
        os.environ["CC_DEEP_SORT"] = "1"
    try:
        engine.set_profiling(True)
        engine.profile_only(())
        res = consensus_pipeline(bam, out, engine=engine)
        kt = engine.kernel_times()
        engine.set_profiling(False)
    finally:
        if old is None:
            os.environ.pop("CC_DEEP_SORT", None)
        else:
            os.environ["CC_DEEP_SORT"] = old
    return res, kt


@pytest.mark.parametrize("name", sorted(CASES))
def test_deep_rank_matches_oracle(name, engine, tmp_path):
    import cc_oracle
    from consensuscruncher_amd import synth
    kw = dict(CASES[name])
    n = kw.pop("n_pairs")
    seed = synth.SEED_BASE + kw.pop("seed")
    batch = synth.generate(n, seed=seed, **kw)
    bam = str(tmp_path / "sample.bam")
    synth.write_bam_native(batch, bam)
    ref = cc_oracle.consensus_pipeline(bam, str(tmp_path / "oracle"))
    for deep_fam in (True, False):
        ours, kt = _run(engine, bam, str(tmp_path / ("fam" if deep_fam else "sort")), deep_fam)
        errs = []
        for k in OUTS:
            if k not in ref:
                continue
            try:
                assert_same_records(ours[k], ref[k], "%s/%s/%s" % (name, deep_fam, k))
            except AssertionError as e:
                errs.append(str(e))
        assert not errs, "\n".join(errs)
        for k in ("stats", "read_families"):
            if k in ref:
                assert open(ours[k]).read() == open(ref[k]).read(), k
        assert "k_group" in kt, sorted(kt)
        if deep_fam:
            assert "k_deep_fam" in kt, sorted(kt)
            if name == "one_position":
                assert "sort_tags_big" in kt, sorted(kt)   # the over-limit pass took the sorted path
            else:
                assert "sort_tags_big" not in kt, sorted(kt)
                assert "k_deep_emit" in kt, sorted(kt)
                if name == "zipf_loci":   # random ties: families out of end order are sorted
                    assert "k_deep_sortfam" in kt, sorted(kt)
        else:
            assert "k_deep_fam" not in kt and "sort_tags_big" in kt, sorted(kt)
