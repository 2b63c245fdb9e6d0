"""Pin the CPU oracle (oracle/cc_oracle.py) to the reference's own outputs."""
import json
import os
import shutil

import pytest

import cc_oracle
from parity import GOLDEN, assert_same_records, cases


@pytest.mark.parametrize("case", cases())
def test_oracle_matches_reference(case, tmp_path):
    d = os.path.join(GOLDEN, case)
    params = json.load(open(os.path.join(d, "params.json")))["run"]
    kw = dict(params)
    if kw.get("bedfile", "False") != "False":
        kw["bedfile"] = os.path.join(d, kw["bedfile"])
    shutil.copy(os.path.join(d, "input.bam"), str(tmp_path / "sample.bam"))
    exp = os.path.join(d, "expected")
    if os.path.exists(os.path.join(exp, "error.txt")):
        kind = open(os.path.join(exp, "error.txt")).read().split(":")[0]
        with pytest.raises(cc_oracle.OracleError) as ei:
            cc_oracle.consensus_pipeline(str(tmp_path / "sample.bam"), str(tmp_path), **kw)
        assert str(ei.value).startswith(kind)
        return
    out = cc_oracle.consensus_pipeline(str(tmp_path / "sample.bam"), str(tmp_path), **kw)
    for f in sorted(os.listdir(exp)):
        if f.endswith(".bam"):
            assert_same_records(out[f[:-4]], os.path.join(exp, f), "%s/%s" % (case, f))
    assert open(out["stats"]).read() == open(os.path.join(exp, "stats.txt")).read()
    assert open(out["read_families"]).read() == open(os.path.join(exp, "read_families.txt")).read()
