"""The engine's measurement switches (INTEGRATION.md "Engine switches") change no output: the whole
pipeline with each switch set, record for record against the default run on the same input."""
import os

import pytest

pytestmark = pytest.mark.gpu

SWITCHES = [("CC_PC_TILE", "1024"), ("CC_PC_TILE", "512"), ("CC_RESID_SORT", "1"), ("CC_SCAN1", "1"),
            ("CC_SCAN1", "0")]


@pytest.fixture(scope="module")
def case(tmp_path_factory):
    from consensuscruncher_amd import synth
    from consensuscruncher_amd.engine import Engine
    from consensuscruncher_amd.pipeline import consensus_pipeline
    d = tmp_path_factory.mktemp("switches")
    batch = synth.generate(40_000, seed=synth.SEED_BASE + 931)
    bam = str(d / "s.bam")
    synth.write_bam_native(batch, bam)
    e = Engine(0)
    base = consensus_pipeline(bam, str(d / "base"), engine=e)
    yield e, bam, d, base
    e.close()


@pytest.mark.parametrize("name,value", SWITCHES)
def test_switch_changes_no_output(case, name, value):
    from parity import assert_same_records
    from consensuscruncher_amd.pipeline import consensus_pipeline
    e, bam, d, base = case
    os.environ[name] = value
    try:
        got = consensus_pipeline(bam, str(d / ("%s_%s" % (name, value))), engine=e)
    finally:
        os.environ.pop(name, None)
    assert sorted(got) == sorted(base)
    n = 0
    for k in base:
        if not (isinstance(base[k], str) and os.path.isfile(base[k])):
            continue
        if base[k].endswith(".bam"):
            assert_same_records(got[k], base[k], "%s=%s/%s" % (name, value, k))
        else:
            assert open(got[k], "rb").read() == open(base[k], "rb").read(), k
        n += 1
    assert n >= 5
