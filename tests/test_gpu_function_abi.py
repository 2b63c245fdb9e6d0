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


# ---- cc_group / cc_duplex_join on caller-given keys ----------------
def random_tags(rng, n, odd_frac=0.2):
    """Tags in unique_tag's grammar (consensus_helper.py:295-304); some barcodes odd-length without a
    '.', whose duplex_tag is a rotation (non-mutual chains)."""
    out = set()
    while len(out) < n:
        if rng.random() < odd_frac:
            bc = "".join(rng.choice(list("ACGT"), 3))
        elif rng.random() < 0.5:
            bc = "".join(rng.choice(list("ACGT"), 2)) + "." + "".join(rng.choice(list("ACGT"), int(rng.integers(1, 4))))
        else:
            bc = "".join(rng.choice(list("ACGT"), 4))
        t = "%s_%d_%d_%d_%d_%dM_%dM_%s_%s" % (bc, rng.integers(0, 2), rng.integers(0, 40), rng.integers(0, 2),
                                             rng.integers(0, 40), 150, 150, rng.choice(["fwd", "rev"]),
                                             rng.choice(["R1", "R2"]))
        out.add(t)
    return sorted(out)


def test_group_matches_read_dict(engine):
    from consensuscruncher_amd.engine import pack_keys
    rng = np.random.default_rng(41)
    for distinct, n in ((5, 1000), (3000, 60000), (60000, 60000)):
        pool = random_tags(rng, distinct, odd_frac=0.0)
        tags = [pool[int(i)] for i in rng.integers(0, len(pool), n)]
        perm, off = engine.group(pack_keys(tags, 48))
        want = cc_oracle.group_keys(tags)
        got = [perm[off[k]:off[k + 1]].tolist() for k in range(len(off) - 1)]
        assert got == want
    perm, off = engine.group(np.zeros((0, 8), np.uint8))
    assert len(perm) == 0 and off.tolist() == [0]


@pytest.mark.parametrize("seed", [51, 52, 53, 54])
def test_duplex_join_dcs_matches_reference_loop(engine, seed):
    from consensuscruncher_amd.engine import duplex_tag, pack_keys
    rng = np.random.default_rng(seed)
    base = random_tags(rng, 3000, odd_frac=0.15 if seed != 54 else 0.0)
    # entries: the base tags, most of their duplex partners, shuffled (csn processing order)
    tags = set(base)
    for t in base:
        if rng.random() < 0.7:
            tags.add(duplex_tag(t))
    tags = list(tags)
    rng.shuffle(tags)
    parts = [duplex_tag(t) for t in tags]
    try:
        want = cc_oracle.dcs_join(tags, parts)
    except cc_oracle.OracleError:
        want = None
    if want is None:
        with pytest.raises(N.CCError) as e:
            engine.duplex_join(0, pack_keys(tags, 48), pack_keys(parts, 48))
        assert e.value.code == N.CC_E_KEYERROR
        # without the chains the reference raises on, the rest pairs
        keep = [i for i, t in enumerate(tags) if "." in t.split("_")[0] or len(t.split("_")[0]) % 2 == 0]
        tags = [tags[i] for i in keep]
        parts = [parts[i] for i in keep]
        want = cc_oracle.dcs_join(tags, parts)
    dec, part = engine.duplex_join(0, pack_keys(tags, 48), pack_keys(parts, 48))
    assert list(zip(dec.tolist(), part.tolist())) == want
    assert (dec == 0).sum() > 100 and (dec == 1).sum() > 10 and (dec == 2).sum() > 100


@pytest.mark.parametrize("seed", [61, 62, 63])
def test_duplex_join_sc_matches_reference_loop(engine, seed):
    from consensuscruncher_amd.engine import duplex_tag, pack_keys
    rng = np.random.default_rng(seed)
    pool = random_tags(rng, 6000, odd_frac=0.15)
    rng.shuffle(pool)
    singles = set(pool[:3000])
    sscs = [t for t in pool[3000:]]
    for t in pool[:3000]:   # complements among the singletons and among the SSCS
        r = rng.random()
        if r < 0.3:
            singles.add(duplex_tag(t))
        elif r < 0.5:
            sscs.append(duplex_tag(t))
    sscs = sorted(set(sscs) - singles)
    singles = list(singles)
    rng.shuffle(singles)
    parts = [duplex_tag(t) for t in singles]
    try:
        want = cc_oracle.sc_join(singles, parts, sscs)
    except cc_oracle.OracleError:
        pytest.skip("this draw raises in the reference")
    dec, part = engine.duplex_join(1, pack_keys(singles, 48), pack_keys(parts, 48), pack_keys(sscs, 48))
    assert list(zip(dec.tolist(), part.tolist())) == want
    assert (dec == 0).sum() > 100 and (dec == 1).sum() > 100 and (dec == 2).sum() > 100


def test_duplex_join_votes_like_pair_vote(engine, tmp_path):
    """The joined pairs' consensus rows equal duplex_consensus of the two reads (entry i's read is
    record i of table A, SSCS entry k's record k of table X)."""
    from consensuscruncher_amd.engine import duplex_tag, pack_keys
    L = 150
    rng = np.random.default_rng(71)
    base = random_tags(rng, 300, odd_frac=0.0)
    singles = list(base[:200]) + [duplex_tag(t) for t in base[:60]]
    sscs = [duplex_tag(t) for t in base[100:160]]
    rng.shuffle(singles)
    ra = random_bam(str(tmp_path / "a.bam"), len(singles), L, seed=72, n_frac=0.05)
    rx = random_bam(str(tmp_path / "x.bam"), len(sscs), L, seed=73, n_frac=0.05)
    ta, _ = upload(engine, str(tmp_path / "a.bam"))
    tx, _ = upload(engine, str(tmp_path / "x.bam"))
    parts = [duplex_tag(t) for t in singles]
    for mode in (0, 1):
        x = sscs if mode == 1 else None
        dec, part, (seq, qual, meta) = engine.duplex_join(
            mode, pack_keys(singles, 48), pack_keys(parts, 48), pack_keys(x, 48) if x else None,
            vote=(ta, np.arange(len(singles)), tx if mode == 1 else -1, np.arange(len(sscs)) if mode == 1 else None))
        want = cc_oracle.dcs_join(singles, parts) if mode == 0 else cc_oracle.sc_join(singles, parts, sscs)
        assert list(zip(dec.tolist(), part.tolist())) == want
        nv = 0
        for i, (d, j) in enumerate(want):
            if (mode == 0 and d != 0) or (mode == 1 and d == 2):
                continue
            other = rx[j] if (mode == 1 and d == 0) else ra[j]
            s, q = cc_oracle.pair_vote(ra[i], other, gate=bool(mode))
            assert seq_str(seq[i], L) == s and list(qual[i][:L]) == list(q), (mode, i)
            nv += 1
        assert nv > 20
    engine.free_table(ta)
    engine.free_table(tx)
