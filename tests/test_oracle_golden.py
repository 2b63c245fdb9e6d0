"""Pin the CPU oracle (oracle/cc_oracle.py) to the reference's own outputs."""
import json
import os
import shutil

import pytest

import cc_oracle
from parity import GOLDEN, cases, check_partial
import pysam


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
        check_partial(str(tmp_path), exp, case)
        return
    out = cc_oracle.consensus_pipeline(str(tmp_path / "sample.bam"), str(tmp_path), **kw)
    for f in sorted(os.listdir(exp)):
        if f.endswith(".bam"):
            assert pysam.sam_lines(out[f[:-4]]) == pysam.sam_lines(os.path.join(exp, f)), "%s/%s" % (case, f)
    assert open(out["stats"]).read() == open(os.path.join(exp, "stats.txt")).read()
    assert open(out["read_families"]).read() == open(os.path.join(exp, "read_families.txt")).read()
