"""GPU SSCS vote (k_sscs_vote_swar and its hand-over to the exact k_sscs_vote) against the
oracle on adversarial families: a 25% substitution rate (many split positions, including
count[best] == 1 < pass), qualities drawn from the edges of every byte test the SWAR form makes
(29/30, 60/61, 127/128, 157/158, 254), consensus lengths shorter than the longest read and not
a multiple of 16, cutoffs 0.5 / 0.7 / 1.0 / 1.01, and a base outside ACGTN in a voted family.

The oracle (oracle/cc_oracle.py) is pinned to the reference by tests/golden; here it is the
checker on inputs the golden cases do not reach.  Parity: every output BAM record for record."""
import numpy as np
import pytest

from parity import assert_same_records

pytestmark = pytest.mark.gpu

QSET = np.array([0, 2, 10, 29, 30, 31, 45, 59, 60, 61, 62, 93, 126, 127, 128, 157, 158, 200, 254], np.uint8)
OUTS = ("sscs", "singleton", "dcs", "sscs_singleton", "sscs_correction", "singleton_correction", "uncorrected",
        "dcs_sc", "all_unique")


@pytest.fixture(scope="module")
def engine():
    from consensuscruncher_amd.engine import Engine
    e = Engine(0)
    yield e
    e.close()


def _adversarial_bam(path, seed, read_len=137, err=0.25, n_pairs=3000, bad_base=False):
    import pysam
    import synthbam
    from consensuscruncher_amd import synth
    batch = synth.generate(n_pairs, seed=seed, read_len=read_len, contigs=(("chr1", 400_000),), err_rate=err,
                           fam_mean=3.0, bad_frac=0.0, spacer_bad_frac=0.0)
    rng = np.random.default_rng(seed)
    q = batch.qual
    m = rng.random(q.shape) < 0.35
    q[m] = rng.choice(QSET, int(m.sum()))
    q[batch.seq == ord("N")] = 2          # an N at Q >= 30 is the reference's IndexError (golden case)
    header, recs = synthbam.batch_records(batch)
    # read ends starting in these windows are truncated: consensus length below the table's longest
    # read, and not a multiple of the 16-position lane chunk
    windows = ((100_000, 160_000, 100), (200_000, 230_000, 33), (260_000, 280_000, 17))
    for r in recs:
        for lo, hi, k in windows:
            if lo <= r.reference_start < hi and r.cigartuples:
                s, qq = r.query_sequence, list(r.query_qualities)
                r.query_sequence = s[:k]
                r.query_qualities = qq[:k]
                r.cigartuples = [(0, k)]
    if bad_base:
        # an IUPAC code in a member of a family of size >= 2 (SSCS_maker.py:122 ValueError)
        by_pos = {}
        for i, r in enumerate(recs):
            by_pos.setdefault((r.reference_id, r.reference_start, r.flag, r.query_name.split("|")[-1]), []).append(i)
        i = next(v[0] for v in by_pos.values() if len(v) >= 3)
        s, qq = recs[i].query_sequence, list(recs[i].query_qualities)
        recs[i].query_sequence = s[:5] + "R" + s[6:]
        recs[i].query_qualities = qq
    pysam.write_bam_file(path, header, recs, 1)
    return path


@pytest.mark.parametrize("cutoff", [0.7, 0.5, 1.0, 1.01])
def test_adversarial_votes_match_oracle(cutoff, engine, tmp_path):
    import cc_oracle
    from consensuscruncher_amd.pipeline import consensus_pipeline
    bam = _adversarial_bam(str(tmp_path / "adv.bam"), seed=20261015 + 700)
    ours = consensus_pipeline(bam, str(tmp_path / "gpu"), cutoff=cutoff, engine=engine)
    ref = cc_oracle.consensus_pipeline(bam, str(tmp_path / "oracle"), cutoff=cutoff)
    errs = []
    for k in OUTS:
        try:
            assert_same_records(ours[k], ref[k], "cutoff %s/%s" % (cutoff, k))
        except AssertionError as e:
            errs.append(str(e))
    assert not errs, "\n".join(errs)
    assert open(ours["stats"]).read() == open(ref["stats"]).read()


def test_base_outside_acgtn_raises_like_reference(engine, tmp_path):
    import cc_oracle
    from consensuscruncher_amd import native as N
    from consensuscruncher_amd.pipeline import consensus_pipeline
    bam = _adversarial_bam(str(tmp_path / "bad.bam"), seed=20261015 + 701, err=0.005, bad_base=True)
    with pytest.raises(cc_oracle.OracleError) as eo:
        cc_oracle.consensus_pipeline(bam, str(tmp_path / "oracle"))
    assert str(eo.value).startswith("ValueError")
    with pytest.raises(N.CCError) as ei:
        consensus_pipeline(bam, str(tmp_path / "gpu"), engine=engine)
    assert ei.value.code == -4          # CC_E_BAD_BASE


def test_vote_after_pass_without_member_records(engine, tmp_path):
    """A read_bam pass that does not list bad reads (badread_file=0) leaves the votes' member records
    unwritten (only the SSCS stage's pass writes them as it ranks); consensus_maker then builds them
    itself (k_mem_meta).  On an input with nothing filtered the two passes group alike, so the votes
    must agree byte for byte."""
    from consensuscruncher_amd import synth
    from consensuscruncher_amd.engine import MODE_SSCS, Bam, Interner, whole_file_stream
    batch = synth.generate(4000, seed=synth.SEED_BASE + 731, contigs=(("chr1", 300_000),), bad_frac=0.0,
                           spacer_bad_frac=0.0, err_rate=0.05)
    bam = str(tmp_path / "in.bam")
    synth.write_bam_native(batch, bam)
    it = Interner()
    b = Bam(bam)
    rec = b.decode(it, MODE_SSCS, "|")
    table = engine.upload(rec)
    stream = whole_file_stream(rec)
    out = {}
    for bad in (1, 0):
        g = engine.read_bam(table, stream, delim_filter=1, badread_file=bad, scope_by_run=0)
        engine.consensus_maker(g, 0.7)
        engine.rerun(g, 0x1234)               # planned re-run: the on-demand build runs again
        engine.consensus_maker(g, 0.7)
        out[bad] = {k: engine.fetch(g, k, dt) for k, dt in (("cons_seq", np.uint8), ("cons_qual", np.uint8),
                                                               ("vote_meta", np.int32), ("emit_n", np.int32))}
        engine.free_group(g)
    engine.free_table(table)
    assert len(out[1]["emit_n"]) > 1000
    for k in out[1]:
        assert np.array_equal(out[0][k], out[1][k]), k
