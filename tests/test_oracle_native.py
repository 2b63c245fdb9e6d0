"""Pin the C++ oracle (oracle/cc_oracle.cpp) to the reference's own outputs and to the Python
oracle: every golden case record for record IN FILE ORDER (the reference's emission order and the
samtools stand-in's tie order), stats.txt and read_families.txt byte for byte; a seeded sample with
several contigs, translocations and a bed file identical to oracle/cc_oracle.py; Python float repr."""
import json
import os
import shutil

import pytest

import cc_oracle
import cc_oracle_native as O
import pysam
from parity import GOLDEN, cases, check_partial

KEYS = ["sscs", "singleton", "badreads", "dcs", "sscs_singleton", "sscs_correction", "singleton_correction",
        "uncorrected", "sscs_sc", "dcs_sc", "sscs_sc_singleton", "all_unique"]


@pytest.mark.parametrize("case", cases())
def test_native_oracle_matches_reference(case, tmp_path):
    d = os.path.join(GOLDEN, case)
    kw = dict(json.load(open(os.path.join(d, "params.json")))["run"])
    if kw.get("bedfile", "False") != "False":
        kw["bedfile"] = os.path.join(d, kw["bedfile"])
    shutil.copy(os.path.join(d, "input.bam"), str(tmp_path / "sample.bam"))
    exp = os.path.join(d, "expected")
    if os.path.exists(os.path.join(exp, "error.txt")):
        kind = open(os.path.join(exp, "error.txt")).read().split(":")[0]
        with pytest.raises(O.OracleError) as ei:
            O.consensus_pipeline(str(tmp_path / "sample.bam"), str(tmp_path), **kw)
        assert str(ei.value).startswith(kind)
        check_partial(str(tmp_path), exp, case)
        return
    out = O.consensus_pipeline(str(tmp_path / "sample.bam"), str(tmp_path), **kw)
    for f in sorted(os.listdir(exp)):
        if f.endswith(".bam"):
            assert pysam.sam_lines(out[f[:-4]]) == pysam.sam_lines(os.path.join(exp, f)), "%s/%s" % (case, f)
    assert open(out["stats"]).read() == open(os.path.join(exp, "stats.txt")).read()
    assert open(out["read_families"]).read() == open(os.path.join(exp, "read_families.txt")).read()


def test_native_oracle_matches_python_oracle(tmp_path):
    import synthbam
    from consensuscruncher_amd import synth
    batch = synth.generate(4000, seed=synth.SEED_BASE + 301, transloc_frac=0.03, quirk_frac=0.02,
                           contigs=(("chr1", 300_000), ("chr2", 200_000)))
    bam = str(tmp_path / "s.bam")
    synthbam.write_batch(batch, bam)
    bed = str(tmp_path / "r.bed")
    with open(bed, "w") as f:
        f.write("chr2\t0\t120000\tp1\tgneg\nchr1\t0\t160000\tp1\tgneg\nchr1\t160000\t300000\tq1\tgneg\n"
                "chr2\t120000\t200000\tq1\tgneg\n")
    for bedfile in ("False", bed):
        a = O.consensus_pipeline(bam, str(tmp_path / ("n" + str(bedfile != "False"))), bedfile=bedfile)
        b = cc_oracle.consensus_pipeline(bam, str(tmp_path / ("p" + str(bedfile != "False"))), bedfile=bedfile)
        for k in KEYS:
            assert pysam.sam_lines(a[k]) == pysam.sam_lines(b[k]), k
        assert open(a["stats"]).read() == open(b["stats"]).read()
        assert open(a["read_families"]).read() == open(b["read_families"]).read()


@pytest.mark.parametrize("x", [0.0, 12.5, 100.0, 33.33333333333333, 2 / 3 * 100, 1e-5, 3.3333333333333335e-05,
                               0.0005, 7 / 11, 1e16, 123456789.125])
def test_python_float_repr(x):
    assert O.py_float(x) == repr(x)
