"""GPU parity against the reference's own outputs (tests/golden, made by
oracle/make_golden.py from the unmodified reference scripts).  Every output BAM
of the consensus pipeline must hold exactly the reference's records in the
reference's file order (emission order, samtools tie order); stats.txt and
read_families.txt must be byte-identical.  Where the reference raises, the
pipeline must raise the matching error after writing the same outputs for the
stages that completed."""
import json
import os
import shutil

import pytest

from parity import GOLDEN, assert_same_in_order, cases, check_partial

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    from consensuscruncher_amd.engine import Engine
    e = Engine(0)
    yield e
    e.close()


@pytest.mark.parametrize("case", cases())
def test_pipeline_matches_reference(case, engine, tmp_path):
    from consensuscruncher_amd import native as N
    from consensuscruncher_amd.pipeline import consensus_pipeline
    d = os.path.join(GOLDEN, case)
    params = json.load(open(os.path.join(d, "params.json")))["run"]
    kw = dict(params)
    if kw.get("bedfile", "False") != "False":
        kw["bedfile"] = os.path.join(d, kw["bedfile"])
    shutil.copy(os.path.join(d, "input.bam"), str(tmp_path / "sample.bam"))
    exp = os.path.join(d, "expected")
    if os.path.exists(os.path.join(exp, "error.txt")):
        err = open(os.path.join(exp, "error.txt")).read().split(":")[0]
        with pytest.raises(N.CCError) as ei:
            consensus_pipeline(str(tmp_path / "sample.bam"), str(tmp_path), engine=engine, **kw)
        assert ei.value.code == {"IndexError": N.CC_E_N_HIGHQ, "KeyError": N.CC_E_KEYERROR}[err], str(ei.value)
        check_partial(str(tmp_path), exp, case)
        return
    out = consensus_pipeline(str(tmp_path / "sample.bam"), str(tmp_path), engine=engine, **kw)
    n, errs = 0, []
    for f in sorted(os.listdir(exp)):
        if f.endswith(".bam"):
            try:
                n += assert_same_in_order(out[f[:-4]], os.path.join(exp, f), "%s/%s" % (case, f))
            except AssertionError as e:
                errs.append(str(e))
    assert not errs, "\n".join(errs)
    assert open(out["stats"]).read() == open(os.path.join(exp, "stats.txt")).read()
    assert open(out["read_families"]).read() == open(os.path.join(exp, "read_families.txt")).read()
    assert n > 0
    if case == "unsorted":
        from consensuscruncher_amd.engine import Bam, Interner, coord_sorted
        b = Bam(str(tmp_path / "sample.bam"))
        assert not coord_sorted(b.decode(Interner(), 0)), "the unsorted case must take the global-sort path"


def test_loaded_engine_build():
    """The library the suite runs on: the debug build when tests/test_gpu_debug_bounds.py runs it."""
    from consensuscruncher_amd import native as N
    assert N.amd().cc_debug_build() == (1 if os.environ.get("CC_EXPECT_DEBUG") else 0)
