"""fastq2bam's UMI extraction: the product CLI
(consensuscruncher_amd/extract_barcodes.py over libccio's ccio_extract_barcodes) against fixtures
made by the reference's own extract_barcodes.py (oracle/make_golden_fastq.py) on pairs from the
reference's bundled test FASTQs.  Output FASTQs, bad-barcode lists and the stats text byte for
byte; a raise of the reference is a raise of the same type here, with the same partial outputs.
Host code only (no GPU)."""
import builtins
import gzip
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GF = os.path.join(ROOT, "tests", "golden_fastq")
sys.path.insert(0, os.path.join(ROOT, "oracle"))

# host-only fixtures: not sent to the GPU box (.gpurunignore), where nothing here is collected
CASES = sorted(d for d in os.listdir(GF) if d != "inputs") if os.path.isdir(GF) else []


def _read(path):
    if path.endswith(".gz"):
        return gzip.open(path, "rb").read()
    return open(path, "rb").read()


@pytest.mark.parametrize("case", CASES)
def test_extraction_matches_reference(case, tmp_path):
    from make_golden_fastq import OUTPUTS, argv_for, variant_inputs
    from consensuscruncher_amd import extract_barcodes as X
    p = json.load(open(os.path.join(GF, case, "params.json")))
    r1, r2 = variant_inputs(GF, p, str(tmp_path))
    os.makedirs(str(tmp_path / "fastq_tag"))
    outfile = str(tmp_path / "fastq_tag" / "sample")
    exp = os.path.join(GF, case, "expected")
    err = None
    try:
        X.main(argv_for(p, r1, r2, outfile, os.path.join(GF, "inputs", "blist.txt")))
    except BaseException as e:   # noqa: B902
        err = e
    if os.path.exists(os.path.join(exp, "error.txt")):
        want = open(os.path.join(exp, "error.txt")).read().split(":", 1)[0]
        assert isinstance(err, getattr(builtins, want)), (err, want)
    else:
        assert err is None, err
    for suf in OUTPUTS:
        e = os.path.join(exp, suf[1:] + ".gz")
        assert os.path.exists(outfile + suf) == os.path.exists(e), suf
        if os.path.exists(e):
            assert _read(outfile + suf) == _read(e), suf
    st = str(tmp_path / "fastq_tag_barcode_stats.txt")
    assert open(st).read() == open(os.path.join(exp, "barcode_stats.txt")).read()


@pytest.mark.skipif(not os.path.isdir(GF), reason="host-only fixtures absent")
def test_threads_do_not_change_outputs(tmp_path):
    """Pairs split over 1 or 8 threads: the same bytes in pair order."""
    from consensuscruncher_amd.engine import extract_barcodes
    from make_golden_fastq import variant_inputs
    r1, r2 = variant_inputs(GF, {"argv": []}, str(tmp_path))
    outs = []
    for t in (1, 8):
        pre = str(tmp_path / ("t%d" % t))
        c, h1, h2 = extract_barcodes(r1, r2, pre, pattern="NNT", nthreads=t)
        outs.append((open(pre + "_barcode_R1.fastq", "rb").read(), c, h1.tolist()))
    assert outs[0] == outs[1]
