"""The function-level C ABI (include/consensuscruncher_amd.h: cc_sscs_vote, cc_pair_vote), called
through ctypes on caller-given families and pairs of an uploaded table, against the reference's
worked example (SSCS_maker.py:27-35) and the pinned Python oracle's restatements of
consensus_maker (oracle/cc_oracle.py single_strand_vote, SSCS_maker.py:81-168) and of the two
duplex_consensus variants (pair_vote, DCS_maker.py:99-123 / singleton_correction.py:61-86).

The families are random partitions of random reads: sizes 1..80 (across the SWAR vote's 63-member
limit), one family of 300 (the split vote), mixed mapq / tlen / flags (the create_aligned_segment
modes with first-seen ties, consensus_flag's 99 > 83 > 147 > 163 priority)."""
import numpy as np
import pytest

import cc_oracle
import pysam
from consensuscruncher_amd import native as N

pytestmark = pytest.mark.gpu

BASES = "ACGTN"
NT16 = "=ACMGRSVTWYHKDBN"


def random_bam(path, n, L, seed, n_frac=0.01):
    rng = np.random.default_rng(seed)
    hdr = pysam.AlignmentHeader("@HD\tVN:1.6\tSO:unsorted\n@SQ\tSN:chr1\tLN:1000000\n@RG\tID:1\n",
                                [("chr1", 1000000)])
    recs = []
    consensus = rng.integers(0, 4, L)
    for i in range(n):
        r = pysam.AlignedSegment(hdr)
        r.query_name = "r%d|AC.GT" % i
        r.flag = int(rng.choice([99, 83, 147, 163, 99, 99, 97, 145]))
        r.reference_id = 0
        r.reference_start = 1000
        r.mapping_quality = int(rng.choice([60, 60, 60, 40, 17]))
        r.cigartuples = [(0, L)]
        r.next_reference_id = 0
        r.next_reference_start = 1200
        r.template_length = int(rng.choice([350, 350, -350, 351]))
        b = consensus.copy()
        flip = rng.random(L) < 0.2
        b[flip] = rng.integers(0, 4, int(flip.sum()))
        q = rng.choice([2, 20, 29, 30, 35, 37, 40, 41], L)
        isn = rng.random(L) < n_frac
        b[isn] = 4
        q[isn] = np.minimum(q[isn], 25)   # N at Q >= 30 is the reference's IndexError (tested apart)
        r.query_sequence = "".join(BASES[x] for x in b)
        r.query_qualities = [int(x) for x in q]
        r.set_tag("RG", "1")
        recs.append(r)
    pysam.write_bam_file(path, hdr, recs)
    return recs


def upload(eng, path):
    from consensuscruncher_amd.engine import MODE_SSCS, Bam, Interner
    it = Interner()
    bam = Bam(path)
    rec = bam.decode(it, MODE_SSCS, "|")
    return eng.upload(rec), it


def families(n, seed, big=300):
    rng = np.random.default_rng(seed)
    perm = rng.permutation(n)
    sizes, tot = [big], big
    while tot < n:
        s = int(min(rng.integers(1, 81), n - tot))
        sizes.append(s)
        tot += s
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    return perm.astype(np.int32), off


def seq_str(codes, L):
    return "".join(NT16[c] for c in codes[:L])


@pytest.fixture(scope="module")
def engine():
    from consensuscruncher_amd.engine import Engine
    e = Engine(0)
    yield e
    e.close()


@pytest.mark.parametrize("cutoff", [0.7, 0.5, 1.0])
def test_sscs_vote_matches_oracle(engine, tmp_path, cutoff):
    L = 150
    recs = random_bam(str(tmp_path / "r.bam"), 4000, L, seed=11)
    table, it = upload(engine, str(tmp_path / "r.bam"))
    mi, off = families(len(recs), seed=12)
    seq, qual, meta = engine.sscs_vote(table, mi, off, cutoff)
    for k in range(len(off) - 1):
        fam = [recs[j] for j in mi[off[k]:off[k + 1]]]
        s, q = cc_oracle.single_strand_vote(fam, cutoff)
        assert seq_str(seq[k], L) == s, k
        assert list(qual[k][:L]) == list(q), k
        assert meta[k][0] == L
        assert meta[k][1] == cc_oracle.most_common_first([m.mapping_quality for m in fam]), k
        assert meta[k][2] == cc_oracle.most_common_first([m.template_length for m in fam]), k
        assert meta[k][3] == cc_oracle.pick_flag(fam), k
        assert it.get(2, meta[k][4]) == "1"
    engine.free_table(table)


def test_sscs_vote_worked_example(engine, tmp_path):
    """SSCS_maker.py:27-35: cutoff 0.7 over the four reads gives ACTGATACNT."""
    hdr = pysam.AlignmentHeader("@HD\tVN:1.6\n@SQ\tSN:chr1\tLN:1000\n", [("chr1", 1000)])
    recs = []
    for i, s in enumerate(["ACTGATACTT", "ACTGAAACCT", "ACTGATACCT", "ACTGATACTT"]):
        r = pysam.AlignedSegment(hdr)
        r.query_name = "w%d|AC.GT" % i
        r.flag = 99
        r.reference_id = 0
        r.reference_start = 100
        r.mapping_quality = 60
        r.cigartuples = [(0, 10)]
        r.next_reference_id = 0
        r.next_reference_start = 300
        r.template_length = 210
        r.query_sequence = s
        r.query_qualities = [40] * 10
        recs.append(r)
    pysam.write_bam_file(str(tmp_path / "w.bam"), hdr, recs)
    table, _ = upload(engine, str(tmp_path / "w.bam"))
    seq, qual, meta = engine.sscs_vote(table, [0, 1, 2, 3], [0, 4], 0.7)
    assert seq_str(seq[0], 10) == "ACTGATACNT"
    assert list(qual[0][:10]) == [60] * 10
    assert list(meta[0]) == [10, 60, 210, 99, -1]
    engine.free_table(table)


def test_sscs_vote_raises_like_the_reference(engine, tmp_path):
    """An N with Q >= 30 in a family (SSCS_maker.py:129 IndexError) -> CC_E_N_HIGHQ; an empty family
    (readList[0]) -> CC_E_INVALID."""
    recs = random_bam(str(tmp_path / "r.bam"), 8, 20, seed=13, n_frac=0.0)
    q = list(recs[3].query_qualities)
    recs[3].query_sequence = "N" + recs[3].query_sequence[1:]   # (pysam resets the qualities here)
    q[0] = 37
    recs[3].query_qualities = q
    hdr = pysam.AlignmentFile(str(tmp_path / "r.bam")).header
    pysam.write_bam_file(str(tmp_path / "n.bam"), hdr, recs)
    table, _ = upload(engine, str(tmp_path / "n.bam"))
    with pytest.raises(N.CCError) as e:
        engine.sscs_vote(table, [0, 1, 2, 3], [0, 2, 4], 0.7)
    assert e.value.code == N.CC_E_N_HIGHQ
    with pytest.raises(cc_oracle.OracleError):
        cc_oracle.single_strand_vote(recs[2:4], 0.7)
    with pytest.raises(N.CCError):
        engine.sscs_vote(table, [0, 1], [0, 2, 2], 0.7)
    engine.free_table(table)


@pytest.mark.parametrize("mode", [0, 1])
def test_pair_vote_matches_oracle(engine, tmp_path, mode):
    L = 150
    ra = random_bam(str(tmp_path / "a.bam"), 600, L, seed=21, n_frac=0.05)
    rb = random_bam(str(tmp_path / "b.bam"), 600, L, seed=22, n_frac=0.05)
    ta, ita = upload(engine, str(tmp_path / "a.bam"))
    tb, itb = upload(engine, str(tmp_path / "b.bam"))
    rng = np.random.default_rng(23)
    a = rng.integers(0, len(ra), 900).astype(np.int32)
    b = rng.integers(0, len(rb), 900).astype(np.int32)
    seq, qual, meta = engine.pair_vote(mode, ta, tb, a, b)
    for i in range(len(a)):
        s, q = cc_oracle.pair_vote(ra[a[i]], rb[b[i]], gate=bool(mode))
        assert seq_str(seq[i], L) == s, i
        assert list(qual[i][:L]) == list(q), i
        assert meta[i][0] == L
        if mode == 0:   # create_aligned_segment over [read1, read2]: modes of the two
            pair = [ra[a[i]], rb[b[i]]]
            assert meta[i][1] == cc_oracle.most_common_first([m.mapping_quality for m in pair])
            assert meta[i][2] == cc_oracle.most_common_first([m.template_length for m in pair])
            assert meta[i][3] == cc_oracle.pick_flag(pair)
        else:           # strand_correction: the singleton's own fields
            assert (meta[i][1], meta[i][2], meta[i][3]) == (ra[a[i]].mapping_quality, ra[a[i]].template_length,
                                                            ra[a[i]].flag)
    engine.free_table(ta)
    engine.free_table(tb)


def test_rccl_reduce_stats_single_rank(engine):
    """cc_reduce_stats over an RCCL communicator of one rank (this box has one GPU): in-place identity;
    a NULL communicator is the one-process case.  The multi-rank reduction is the sharded driver's
    (sharded.TorchComm, RCCL on GPUs) and is rehearsed over gloo in tests/test_dist_cpu.py."""
    from consensuscruncher_amd.engine import comm_unique_id
    comm = engine.comm_init(1, 0, comm_unique_id())
    c = np.arange(16, dtype=np.int64)
    cnt = np.array([0, 5, 7], np.int64)
    first = np.array([1 << 62, 3, 1], np.int64)
    engine.reduce_stats(comm, c, cnt, first)
    assert c.tolist() == list(range(16)) and cnt.tolist() == [0, 5, 7] and first.tolist() == [1 << 62, 3, 1]
    v = np.array([4, 9], np.int64)
    engine.allreduce_max(comm, v)
    assert v.tolist() == [4, 9]
    engine.reduce_stats(None, c, cnt, first)
    N.amd().cc_comm_destroy(comm)
