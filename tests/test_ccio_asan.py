"""libccio under AddressSanitizer + UndefinedBehaviorSanitizer: a native driver
(tests/asan/ccio_driver.cpp) built with the sanitizers runs every entry point the stages use on
golden inputs (regular, unsorted, bed, list barcodes, quirks); any report fails the test."""
import os
import subprocess

import pytest

from parity import GOLDEN

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "oracle", "lib", "ccio_asan_driver")


@pytest.fixture(scope="module")
def driver():
    os.makedirs(os.path.dirname(EXE), exist_ok=True)
    src = [os.path.join(ROOT, "consensuscruncher_amd", "csrc", "ccio.cpp"), os.path.join(ROOT, "tests", "asan", "ccio_driver.cpp")]
    if not os.path.exists(EXE) or any(os.path.getmtime(s) > os.path.getmtime(EXE) for s in src):
        subprocess.check_call(["g++", "-O1", "-g", "-std=c++17", "-fsanitize=address,undefined",
                               "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer", "-o", EXE] + src +
                              ["-lz", "-lpthread"])
    return EXE


@pytest.mark.parametrize("case", ["basic", "unsorted", "hg19_bed", "c5_list", "quirks", "dup_qname"])
def test_ccio_clean_under_sanitizers(driver, case, tmp_path):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    p = subprocess.run([driver, os.path.join(GOLDEN, case, "input.bam"), str(tmp_path),
                        os.path.join(GOLDEN, case, "expected", "sscs.bam")], env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0 and "ok" in p.stdout, p.stderr[-3000:]
    assert "runtime error" not in p.stderr and "AddressSanitizer" not in p.stderr, p.stderr[-3000:]


def test_umi_extraction_clean_under_sanitizers(driver, tmp_path):
    """ccio_extract_barcodes on the bundled-FASTQ fixture pairs (gzip input, pattern and list modes)."""
    fq = os.path.join(ROOT, "tests", "golden_fastq", "inputs")
    if not os.path.isdir(fq):
        pytest.skip("host-only fixtures absent")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    p = subprocess.run([driver, os.path.join(GOLDEN, "basic", "input.bam"), str(tmp_path),
                        os.path.join(GOLDEN, "basic", "expected", "sscs.bam"), os.path.join(fq, "R1.fastq.gz"),
                        os.path.join(fq, "R2.fastq.gz")], env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0 and "ok" in p.stdout, p.stderr[-3000:]
    assert "runtime error" not in p.stderr and "AddressSanitizer" not in p.stderr, p.stderr[-3000:]
