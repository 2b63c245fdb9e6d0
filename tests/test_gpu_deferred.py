"""Deferred end-of-pass checks (cc_defer / cc_commit, Engine.deferred): the stage calls of one
bench step on resident groups with their planned passes' checks deferred to one wait must leave
every result array and counter exactly as the exact (first) run left them; a planned total that
does not hold (cc_debug_skew_plan) must make cc_commit ask for a replay, and the replay (deferral
off) must re-run the pass exactly and restore the same results.

The first run of each stage is exact (it reads every device total back as it goes); the golden
and oracle suites pin that run to the reference.  Here the checker is that exact run itself."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ARRAYS = {
    "sscs": ("emit_n", "emit_rec", "emit_vslot", "vote_meta", "cons_seq", "cons_qual", "bad_rec",
             "fam_sizes_by_creation"),
    "dcs": ("dec", "t_rec", "p_rec", "vslot", "vote_meta", "cons_seq", "cons_qual"),
    "sc": ("dec", "t_rec", "p_rec", "vslot", "vote_meta", "cons_seq", "cons_qual", "q_ckey"),
    "dcs_sc": ("dec", "t_rec", "p_rec", "vslot", "vote_meta", "cons_seq", "cons_qual"),
}


def _snapshot(eng, runs):
    out = {}
    for tag, r in runs:
        g = r.gs if tag == "sc" else r.g
        for a in ARRAYS[tag]:
            out[(tag, a)] = eng.fetch(g, a, np.uint8).tobytes()
        out[(tag, "counters")] = eng.counters(g)
        if tag == "sc":
            out[(tag, "counters_x")] = eng.counters(r.gx)
    return out


def _diff(a, b):
    return [k for k in a if a[k] != b[k]]


@pytest.fixture(scope="module")
def stages(tmp_path_factory):
    import bench
    from consensuscruncher_amd import synth
    from consensuscruncher_amd.engine import Engine
    d = str(tmp_path_factory.mktemp("deferred"))
    batch = synth.generate(60_000, seed=synth.SEED_BASE + 711, contigs=(("chr1", 600_000),))
    inp = os.path.join(d, "sample.bam")
    synth.write_bam_native(batch, inp, level=1)
    eng = Engine(0)
    runs, _ = bench.build_stages(eng, d, inp, 0.7)
    yield eng, runs
    for _, r in runs:
        r.close()
    eng.close()


def _step(eng, runs, seed):
    def calls():
        for _, r in runs:
            r.step(seed)
    eng.deferred(calls)


def test_deferred_steps_keep_results(stages):
    eng, runs = stages
    ref = _snapshot(eng, runs)
    for i in range(3):
        _step(eng, runs, 0x77 + i)
        assert _diff(ref, _snapshot(eng, runs)) == []


# the skewed total is csn_pair_dict's sharing flag: a planned 1 sends the pass down the exact csn
# path (a valid computation, same results), so the failed check is reached without any kernel
# running on sizes that do not hold
@pytest.mark.parametrize("tag,total", [("sscs", "csn_shared"), ("dcs", "csn_shared"), ("sc", "csn_shared")])
def test_deferred_replay_on_failed_plan(stages, tag, total):
    eng, runs = stages
    ref = _snapshot(eng, runs)
    r = dict(runs)[tag]
    g = r.gs if tag == "sc" else r.g
    assert eng.lib.cc_debug_skew_plan(eng.h, g, total.encode(), 1) == 0
    # the commit sees the failed plan and the step replays with deferral off (exact re-run)
    n = []

    def skewed():
        n.append(1)
        for _, rr in runs:
            rr.step(0x99)
    eng.deferred(skewed)
    assert len(n) == 2
    assert _diff(ref, _snapshot(eng, runs)) == []
    # the exact re-run recorded the true plan again: the next deferred step needs no replay
    calls = []

    def probe():
        calls.append(1)
        for _, rr in runs:
            rr.step(0x9a)
    eng.deferred(probe)
    assert len(calls) == 1
    assert _diff(ref, _snapshot(eng, runs)) == []
