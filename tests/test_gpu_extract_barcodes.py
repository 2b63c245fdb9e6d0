"""fastq2bam's UMI extraction with the per-pair decisions on the GPU (cc_extract_barcodes, SURVEY.md §8f
row 4): the product CLI with CC_EXTRACT_GPU=1 against the fixtures the reference's own
extract_barcodes.py made (tests/golden_fastq, oracle/make_golden_fastq.py), byte for byte, and the
GPU path against libccio's host path on a larger sample with damaged barcodes (N bases, spacer
errors, short reads) in both modes."""
import builtins
import gzip
import json
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GF = os.path.join(ROOT, "tests", "golden_fastq")
sys.path.insert(0, os.path.join(ROOT, "oracle"))
CASES = sorted(d for d in os.listdir(GF) if d != "inputs") if os.path.isdir(GF) else []


def _read(path):
    if path.endswith(".gz"):
        return gzip.open(path, "rb").read()
    return open(path, "rb").read()


@pytest.mark.parametrize("case", CASES)
def test_gpu_extraction_matches_reference(case, tmp_path, monkeypatch):
    from make_golden_fastq import OUTPUTS, argv_for, variant_inputs
    from consensuscruncher_amd import extract_barcodes as X
    monkeypatch.setenv("CC_EXTRACT_GPU", "1")
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


def _damaged_pairs(path1, path2, n, seed, short=True):
    rng = np.random.default_rng(seed)
    bases = np.array(list("ACGT"))
    with open(path1, "w") as f1, open(path2, "w") as f2:
        for i in range(n):
            for f, mate in ((f1, 1), (f2, 2)):
                L = int(rng.choice([150, 150, 150, 4, 2] if short else [150, 150, 150, 4, 3]))
                s = bases[rng.integers(0, 4, L)]
                if L > 3 and rng.random() < 0.7:
                    s[2] = "T"                                    # the NNT spacer, mostly present
                if rng.random() < 0.05:
                    s[int(rng.integers(0, min(L, 6)))] = "N"
                seq = "".join(s)
                f.write("@r%d x/%d\n%s\n+\n%s\n" % (i, mate, seq, "I" * L))


@pytest.mark.parametrize("mode", ["pattern", "list"])
def test_gpu_path_equals_host_path(mode, tmp_path):
    from consensuscruncher_amd.engine import extract_barcodes
    from consensuscruncher_amd.stages import get_engine
    r1, r2 = str(tmp_path / "a_R1.fastq"), str(tmp_path / "a_R2.fastq")
    _damaged_pairs(r1, r2, 60000, 7, short=mode == "list")   # pattern mode stops at a read shorter than it
    kw = dict(pattern="NNT") if mode == "pattern" else dict(blist=["AAT", "ACT", "CCT", "GT", "TT", "ACGT", "A"])
    outs = []
    for eng in (None, get_engine()):
        pre = str(tmp_path / ("gpu" if eng else "host"))
        try:
            got = extract_barcodes(r1, r2, pre, engine=eng, **kw)
        except IOError as e:   # pattern mode stops at the first read shorter than the pattern
            got = str(e)
        files = [open(pre + s, "rb").read() for s in ("_barcode_R1.fastq", "_barcode_R2.fastq")
                 if os.path.exists(pre + s)]
        if mode == "list":
            files += [open(pre + s, "rb").read() for s in ("_r1_bad_barcodes.txt", "_r2_bad_barcodes.txt")]
        outs.append((got if isinstance(got, str) else (got[0], got[1].tolist(), got[2].tolist()), files))
    assert outs[0] == outs[1]
    assert any(len(f) > 1000 for f in outs[1][1])
