"""Exactness of the multi-GPU region sharding (consensuscruncher_amd/shard.py),
run as sequential shards on one GPU: the union of per-shard outputs must equal
the single-pass outputs record for record, and the per-shard counters must sum
to the single-pass counters."""
import os

import pytest

import pysam
from parity import GOLDEN

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def _shard_fn(bedfile, world, k, blocks=None):
    from consensuscruncher_amd.consensus_helper import region_list
    from consensuscruncher_amd.engine import bed_stream
    from consensuscruncher_amd.shard import shard_streams

    def fn(bam, rec):
        st = bed_stream(rec, bam.refs, bedfile)
        streams, _ = shard_streams(rec, bam.refs, region_list(bedfile), st, world, blocks)
        return streams[k]
    return fn


def _plan(inp, bedfile, world):
    """The sample's region plan, from its input BAM (shared by every stage)."""
    import numpy as np
    from consensuscruncher_amd.consensus_helper import region_list
    from consensuscruncher_amd.engine import Bam, Interner, bed_stream
    from consensuscruncher_amd.shard import plan_blocks
    b = Bam(inp)
    st = bed_stream(b.decode(Interner(), 0), b.refs, bedfile)
    return plan_blocks(np.bincount(st.region, minlength=len(region_list(bedfile))), world)


@pytest.mark.parametrize("case,world", [("bed_multi", 2), ("bed_multi", 3), ("hg19_bed", 4)])
def test_sharded_sscs_dcs_equal_single_pass(case, world, tmp_path):
    from consensuscruncher_amd.engine import sort_bam
    from consensuscruncher_amd.stages import DCSRun, SSCSRun, get_engine
    import json
    d = os.path.join(GOLDEN, case)
    bed = os.path.join(d, json.load(open(os.path.join(d, "params.json")))["run"]["bedfile"])
    inp = os.path.join(d, "input.bam")
    eng = get_engine()
    blocks = _plan(inp, bed, world)
    whole = SSCSRun(eng, inp, 0.7, bedfile=bed)
    cw = whole.emit(str(tmp_path / "w.sscs.bam"), verbose=False)["counters"]
    whole.close()
    lines = {"sscs": [], "singleton": [], "badReads": []}
    tot = {}
    for k in range(world):
        r = SSCSRun(eng, inp, 0.7, bedfile=bed, shard=_shard_fn(bed, world, k, blocks))
        c = r.emit(str(tmp_path / ("s%d.sscs.bam" % k)), verbose=False, side=False)["counters"]
        r.close()
        for kk in ("COUNTER", "UNMAPPED_MATE", "MULTIPLE_MAPPING", "BAD_SPACER", "FAMILIES"):
            tot[kk] = tot.get(kk, 0) + c[kk]
        lines["sscs"] += pysam.sam_lines(str(tmp_path / ("s%d.sscs.bam" % k)))
        lines["singleton"] += pysam.sam_lines(str(tmp_path / ("s%d.singleton.bam" % k)))
        lines["badReads"] += pysam.sam_lines(str(tmp_path / ("s%d.badReads.bam" % k)))
    assert lines["sscs"] == pysam.sam_lines(str(tmp_path / "w.sscs.bam"))        # same records, same order
    assert lines["singleton"] == pysam.sam_lines(str(tmp_path / "w.singleton.bam"))
    assert sorted(lines["badReads"]) == sorted(pysam.sam_lines(str(tmp_path / "w.badReads.bam")))
    for kk, v in tot.items():
        assert v == cw[kk], kk
    # DCS on the sorted SSCS, sharded the same way
    sort_bam(str(tmp_path / "w.sscs.bam"), str(tmp_path / "w.sscs.sorted.bam"))
    dw = DCSRun(eng, str(tmp_path / "w.sscs.sorted.bam"), bedfile=bed)
    dw.emit(str(tmp_path / "w.dcs.bam"), verbose=False)
    dw.close()
    got = []
    for k in range(world):
        r = DCSRun(eng, str(tmp_path / "w.sscs.sorted.bam"), bedfile=bed, shard=_shard_fn(bed, world, k, blocks))
        r.emit(str(tmp_path / ("s%d.dcs.bam" % k)), verbose=False, side=False)
        r.close()
        got += pysam.sam_lines(str(tmp_path / ("s%d.dcs.bam" % k)))
    assert got == pysam.sam_lines(str(tmp_path / "w.dcs.bam"))


@pytest.mark.parametrize("case,world", [("bed_multi", 2), ("bed_multi", 3), ("hg19_bed", 4)])
def test_sharded_sc_equals_single_pass(case, world, tmp_path):
    """Singleton correction over region shards (singleton_correction.py:203-319: per-region loop, SSCS
    dictionaries reset per chromosome): the per-shard corrections concatenated in rank order equal the
    single pass's, record for record and in order."""
    import json
    import shutil
    from consensuscruncher_amd.engine import sort_bam
    from consensuscruncher_amd.stages import SCRun, SSCSRun, get_engine
    d = os.path.join(GOLDEN, case)
    bed = os.path.join(d, json.load(open(os.path.join(d, "params.json")))["run"]["bedfile"])
    eng = get_engine()
    blocks = _plan(os.path.join(d, "input.bam"), bed, world)
    whole = SSCSRun(eng, os.path.join(d, "input.bam"), 0.7, bedfile=bed)
    whole.emit(str(tmp_path / "w.sscs.bam"), verbose=False, plot=False)
    whole.close()
    sort_bam(str(tmp_path / "w.sscs.bam"), str(tmp_path / "w.sscs.sorted.bam"))
    sort_bam(str(tmp_path / "w.singleton.bam"), str(tmp_path / "w.singleton.sorted.bam"))
    r = SCRun(eng, str(tmp_path / "w.singleton.sorted.bam"), bedfile=bed)
    cw = r.emit(verbose=False)
    r.close()
    names = ("sscs.correction", "singleton.correction", "uncorrected")
    got = {n: [] for n in names}
    tot = {"sscs_correction": 0, "singleton_correction": 0, "uncorrected": 0}
    for k in range(world):
        for f in ("singleton", "sscs"):
            shutil.copy(str(tmp_path / ("w.%s.sorted.bam" % f)), str(tmp_path / ("s%d.%s.sorted.bam" % (k, f))))
        r = SCRun(eng, str(tmp_path / ("s%d.singleton.sorted.bam" % k)), bedfile=bed,
                  shard=_shard_fn(bed, world, k, blocks))
        c = r.emit(verbose=False, side=False)
        r.close()
        for kk in tot:
            tot[kk] += c[kk]
        for n in names:
            got[n] += pysam.sam_lines(str(tmp_path / ("s%d.%s.bam" % (k, n))))
    for n in names:
        assert got[n] == pysam.sam_lines(str(tmp_path / ("w.%s.bam" % n))), n
    for kk, v in tot.items():
        assert v == cw[kk], kk


def _hg38_sample(tmp_path):
    from consensuscruncher_amd import synth
    data = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "consensuscruncher_amd", "data")
    bed = os.path.join(data, "hg38_cytoBand.txt")
    ends = {}
    for line in open(bed):
        c = line.split("\t")
        ends[c[0]] = max(ends.get(c[0], 0), int(c[2]))
    batch = synth.generate(20_000, seed=synth.SEED_BASE + 701, contigs=tuple(ends.items()), transloc_frac=0.02)
    bam = str(tmp_path / "hg38.bam")
    synth.write_bam_native(batch, bam)
    return bam, bed


@pytest.mark.parametrize("case,world", [("bed_multi", 3), ("hg19_bed", 4), ("hg38", 4), ("hg38", 8)])
def test_sharded_pipeline_equals_single_pass(case, world, tmp_path):
    """The multi-GPU product path (consensuscruncher_amd/sharded.py) with its ranks run one after
    another on this GPU: every output of the consensus pipeline, stats.txt and read_families.txt
    equal the single-pass pipeline's byte for byte (records in file order)."""
    import json
    import shutil
    from parity import assert_same_in_order
    from consensuscruncher_amd.pipeline import consensus_pipeline
    from consensuscruncher_amd.sharded import LocalComm, sharded_pipeline
    from consensuscruncher_amd.stages import get_engine
    if case == "hg38":
        bam, bed = _hg38_sample(tmp_path)
    else:
        d = os.path.join(GOLDEN, case)
        bed = os.path.join(d, json.load(open(os.path.join(d, "params.json")))["run"]["bedfile"])
        bam = str(tmp_path / "sample.bam")
        shutil.copy(os.path.join(d, "input.bam"), bam)
    import cc_oracle_native as O
    eng = get_engine()
    one = consensus_pipeline(bam, str(tmp_path / "one"), bedfile=bed, engine=eng, level=1)
    many = sharded_pipeline(bam, str(tmp_path / "many"), bed, LocalComm(world), eng, level=1)
    ref = O.consensus_pipeline(bam, str(tmp_path / "oracle"), bedfile=bed)
    errs = []
    for k in sorted(one):
        for other, label in ((one, "single-pass"), (ref, "oracle")):
            if k not in other:
                continue
            if k in ("stats", "read_families"):
                if open(other[k]).read() != open(many[k]).read():
                    errs.append("%s vs %s" % (k, label))
                continue
            try:
                assert_same_in_order(many[k], other[k], "%s/%s x%d vs %s" % (case, k, world, label))
            except AssertionError as e:
                errs.append(str(e))
    assert not errs, "\n".join(errs)


def test_sharded_cli_two_processes(tmp_path):
    """The multi-GPU command line (python -m torch.distributed.run ... -m consensuscruncher_amd.sharded,
    the consensus argv of ConsensusCruncher.py:461-518) as two processes: gloo for the reduction and
    both ranks on this GPU (the box has one).  Outputs equal the single-pass pipeline's."""
    import socket
    import subprocess
    import sys
    from parity import assert_same_in_order
    from consensuscruncher_amd.pipeline import consensus_pipeline
    from consensuscruncher_amd.stages import get_engine
    bam, bed = _hg38_sample(tmp_path)
    one = consensus_pipeline(bam, str(tmp_path / "one"), genome="hg38", engine=get_engine(), level=1)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, CC_DIST_BACKEND="gloo", CC_DEVICE="0", OMP_NUM_THREADS="2")
    os.makedirs(str(tmp_path / "many"))
    subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                    "--master-addr", "127.0.0.1", "--master-port", str(port), "-m", "consensuscruncher_amd.sharded",
                    "-i", bam, "-o", str(tmp_path / "many"), "-g", "hg38"], check=True, env=env, timeout=240,
                   cwd=ROOT)
    many = {k: os.path.join(str(tmp_path / "many"), os.path.relpath(v, str(tmp_path / "one"))) for k, v in one.items()}
    import cc_oracle_native as O
    ref = O.consensus_pipeline(bam, str(tmp_path / "oracle"), bedfile=bed)
    errs = []
    for k in sorted(one):
        for other, label in ((one, "single-pass"), (ref, "oracle")):
            if k not in other:
                continue
            if k in ("stats", "read_families"):
                if open(other[k]).read() != open(many[k]).read():
                    errs.append("%s vs %s" % (k, label))
                continue
            try:
                assert_same_in_order(many[k], other[k], "cli/%s vs %s" % (k, label))
            except AssertionError as e:
                errs.append(str(e))
    assert not errs, "\n".join(errs)


@pytest.mark.parametrize("world", [4, 8])
def test_sharded_tables_are_rank_local(world, tmp_path):
    """Each rank's device tables hold about 1/N of the sample (its block's records plus the routed
    foreign first mates), not the whole file; outputs still equal the single pass."""
    from parity import assert_same_in_order
    from consensuscruncher_amd.pipeline import consensus_pipeline
    from consensuscruncher_amd.sharded import LocalComm, sharded_pipeline
    from consensuscruncher_amd.stages import get_engine
    bam, bed = _hg38_sample(tmp_path)
    eng = get_engine()
    keep = {}
    many = sharded_pipeline(bam, str(tmp_path / "many"), bed, LocalComm(world), eng, level=1, keep=keep)
    try:
        from consensuscruncher_amd.engine import Bam
        n_total = Bam(bam).n
        sizes = [keep["sscs"][r].rec.n for r in range(world)]
        foreign = [int((keep["sscs"][r].stream.region < 0).sum()) for r in range(world)]
        assert sum(sizes) - sum(foreign) <= n_total
        assert max(sizes) < 2.0 * n_total / world, sizes        # a block's share, not the whole sample
        assert sum(foreign) > 0, "no cross-block pair: the routing is untested"
        for st in ("dcs", "sc", "dcs_sc"):
            assert all(keep[st][r].n_input < n_total for r in range(world))
    finally:
        for st in keep.values():
            for run in st.values():
                run.close()
    one = consensus_pipeline(bam, str(tmp_path / "one"), bedfile=bed, engine=eng, level=1)
    for k in sorted(one):
        if k in ("stats", "read_families"):
            assert open(one[k]).read() == open(many[k]).read(), k
        else:
            assert_same_in_order(many[k], one[k], "%s x%d" % (k, world))


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_overlapping_regions_raise_like_single_pass(world, tmp_path):
    """Overlapping bed regions (golden bed_overlap, from the unmodified reference: its SSCS stage raises
    KeyError at consensus_helper.py:490) stay in one rank's block (shard.overlap_safe_blocks), so the
    sharded driver raises the same error instead of emitting the shared families on two ranks."""
    import json
    import shutil
    from consensuscruncher_amd import native as N
    from consensuscruncher_amd.pipeline import consensus_pipeline
    from consensuscruncher_amd.sharded import Geometry, LocalComm, sharded_pipeline
    from consensuscruncher_amd.engine import Bam
    from consensuscruncher_amd.stages import get_engine
    d = os.path.join(GOLDEN, "bed_overlap")
    bed = os.path.join(d, json.load(open(os.path.join(d, "params.json")))["run"]["bedfile"])
    bam = str(tmp_path / "sample.bam")
    shutil.copy(os.path.join(d, "input.bam"), bam)
    eng = get_engine()
    with pytest.raises(N.CCError) as one:
        consensus_pipeline(bam, str(tmp_path / "one"), bedfile=bed, engine=eng, level=1)
    assert one.value.code == N.CC_E_KEYERROR
    geo = Geometry(Bam(bam).refs, bed, [(0, 1), (1, 2)] + [(2, 2)] * (world - 2))
    assert geo.blocks[0] == (0, 2)
    with pytest.raises(N.CCError) as many:
        sharded_pipeline(bam, str(tmp_path / "many"), bed, LocalComm(world), eng, level=1)
    assert many.value.code == N.CC_E_KEYERROR
