"""The single-launch look-back scan (k_scan_one, forced for every scan with CC_SCAN1=1) against the
reduce-then-scan pair (CC_SCAN1=0): the whole pipeline's outputs record for record, on a case with
scans of one tile and of many (the default picks k_scan_one for scans of at most 64 tiles)."""
import os

import pytest

pytestmark = pytest.mark.gpu


def test_scan_one_matches_scan_pair(tmp_path):
    from consensuscruncher_amd import synth
    from consensuscruncher_amd.engine import Engine
    from consensuscruncher_amd.pipeline import consensus_pipeline
    batch = synth.generate(60_000, seed=synth.SEED_BASE + 917)
    bam = str(tmp_path / "s.bam")
    synth.write_bam_native(batch, bam)
    e = Engine(0)
    try:
        outs = {}
        for one in (False, True):
            os.environ["CC_SCAN1"] = "1" if one else "0"
            try:
                outs[one] = consensus_pipeline(bam, str(tmp_path / ("one" if one else "pair")), engine=e)
            finally:
                os.environ.pop("CC_SCAN1", None)
    finally:
        e.close()
    a, b = outs[False], outs[True]
    assert sorted(a) == sorted(b)
    from parity import assert_same_records
    n = 0
    for k in a:
        if not (isinstance(a[k], str) and os.path.isfile(a[k])):
            continue
        if a[k].endswith(".bam"):
            assert_same_records(b[k], a[k], "scan_one/" + k)
        else:
            assert open(a[k], "rb").read() == open(b[k], "rb").read(), k
        n += 1
    assert n >= 5
