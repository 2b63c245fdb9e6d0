"""GPU parity at the BASELINE configs' own sizes, against the C++ oracle (oracle/cc_oracle.cpp,
pinned to the reference by tests/test_oracle_native.py), through the product's whole pipeline
(pipeline.consensus_pipeline / sharded.sharded_pipeline) on the same seeded synthetic BAM.  Every
output BAM must hold the oracle's records IN FILE ORDER (per-record canonical digests); stats.txt
and read_families.txt byte for byte.

  c2_full       BASELINE configs[1]: 10 M pairs 2x150, NNT UMIs, mean family 4, one 100 Mbp contig,
                -b False -- the bench's headline workload, checked whole
  c5_full       configs[4]: 1 M pairs, 70% singletons, variable-length barcode list
  c4_10m        configs[3]'s model at 10 M reads (5 M pairs) on 100 loci, Zipf(1.2) families
                truncated at 5000 (deep position groups, split votes, large-family modes)
  c3_sharded8   configs[2]'s model at 2 M pairs over hg38 (hg38_cytoBand.txt, 0.1% translocations),
                run through sharded_pipeline over 8 region shards (LocalComm: the 8 ranks in turn on
                this GPU) and compared with the single-process oracle

The oracle runs on host threads (its ctypes calls release the GIL) while the GPU side runs, so the
suite's wall time is about the longest oracle run.  CC_FULLSIZE_SCALE (default 1) scales every
case's pair count, for rehearsals only.
"""
import concurrent.futures as cf
import os
import shutil
import tempfile
import time

import pytest

from parity import assert_same_in_order

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DATA = os.path.join(ROOT, "consensuscruncher_amd", "data")
OUTS = ("sscs", "singleton", "badreads", "dcs", "sscs_singleton", "sscs_correction", "singleton_correction",
        "uncorrected", "sscs_sc", "dcs_sc", "sscs_sc_singleton", "all_unique")
SCALE = float(os.environ.get("CC_FULLSIZE_SCALE", "1"))

# name: (synth config, pair count override or None, shard world or None); oracle-heavy cases first
CASES = [("c2_full", "c2", None, None), ("c4_10m", "c4", 5_000_000, None),
         ("c3_sharded8", "c3", 2_000_000, 8), ("c5_full", "c5", None, None)]


def _say(request, msg):
    """A progress line on the real terminal (long waits must not look like a hang)."""
    capman = request.config.pluginmanager.getplugin("capturemanager")
    line = "[fullsize %s] %s" % (time.strftime("%H:%M:%S"), msg)
    if capman is not None:
        with capman.global_and_fixture_disabled():
            print(line, flush=True)
    else:
        print(line, flush=True)


def _wait(request, fut, what):
    while True:
        try:
            return fut.result(timeout=30)
        except cf.TimeoutError:
            _say(request, "waiting for %s" % what)


@pytest.fixture(scope="module")
def prepared(request):
    """Writes every case's input BAM and starts its oracle pipeline on a host thread."""
    from consensuscruncher_amd import synth
    import cc_oracle_native as O
    root = tempfile.mkdtemp(prefix="ccfull_")
    pool = cf.ThreadPoolExecutor(max_workers=len(CASES))
    jobs = {}
    wanted = {it.callspec.params.get("name") for it in request.session.items
              if getattr(it, "originalname", "") == "test_fullsize_matches_oracle" and hasattr(it, "callspec")}
    for name, cfg_name, pairs, world in CASES:
        if name not in wanted:   # only the selected cases
            continue
        cfg, bed = synth.config(cfg_name)
        if pairs is not None:
            cfg["n_pairs"] = pairs
        cfg["n_pairs"] = max(1000, int(cfg["n_pairs"] * SCALE))
        t = time.time()
        batch = synth.generate(seed=synth.SEED_BASE + int(cfg_name[1:]) + 3000, **cfg)
        d = os.path.join(root, name)
        os.makedirs(d)
        bam = os.path.join(d, "sample.bam")
        synth.write_bam_native(batch, bam, level=1)
        n = batch.n
        del batch
        bedfile = bed or "False"
        fut = pool.submit(O.consensus_pipeline, bam, os.path.join(d, "oracle"), bedfile)
        jobs[name] = dict(bam=bam, bedfile=bedfile, world=world, oracle=fut, dir=d, reads=n)
        _say(request, "%s: %d reads written in %.1fs, oracle started" % (name, n, time.time() - t))
    yield jobs
    pool.shutdown(wait=True)
    shutil.rmtree(root, ignore_errors=True)


def _compare(request, name, ours, ref):
    errs = []
    for k in OUTS:
        try:
            assert_same_in_order(ours[k], ref[k], "%s/%s" % (name, k))
        except AssertionError as e:
            errs.append(str(e))
    assert not errs, "\n".join(errs)
    for k in ("stats", "read_families"):
        assert open(ours[k]).read() == open(ref[k]).read(), "%s/%s" % (name, k)
    _say(request, "%s: 12 BAMs in file order, stats.txt and read_families.txt identical" % name)


# the lighter cases first: their GPU runs overlap the longer oracle runs
@pytest.mark.timeout(1500)
@pytest.mark.parametrize("name", ["c5_full", "c3_sharded8", "c4_10m", "c2_full"])
def test_fullsize_matches_oracle(name, prepared, request):
    from consensuscruncher_amd.pipeline import consensus_pipeline
    from consensuscruncher_amd.sharded import LocalComm, sharded_pipeline
    from consensuscruncher_amd.stages import get_engine
    job = prepared[name]
    eng = get_engine()
    t = time.time()
    out_dir = os.path.join(job["dir"], "gpu")
    if job["world"]:
        ours = sharded_pipeline(job["bam"], out_dir, job["bedfile"], LocalComm(job["world"]), eng, level=1)
    else:
        ours = consensus_pipeline(job["bam"], out_dir, engine=eng, bedfile=job["bedfile"], level=1)
    _say(request, "%s: GPU pipeline (%d reads%s) in %.1fs" % (
        name, job["reads"], ", %d shards" % job["world"] if job["world"] else "", time.time() - t))
    ref = _wait(request, job["oracle"], "%s oracle" % name)
    _compare(request, name, ours, ref)
    if name == "c4_10m":
        sizes = [int(x.split("\t")[0]) for x in open(ref["read_families"]).read().split("\n")[1:]]
        assert max(sizes) >= 4000, "C4 must reach families of several thousand members"
    shutil.rmtree(out_dir, ignore_errors=True)
