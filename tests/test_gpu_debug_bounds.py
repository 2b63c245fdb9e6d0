"""The debug build (consensuscruncher_amd/lib/libccamd_debug.so, -DCC_DEBUG_BOUNDS; SURVEY.md §5 "device
bounds checks in debug builds"): its kernels check record, qname, payload, slot and vote indices and
report the first bad one instead of reading out of bounds.  Run in child processes (CCAMD_LIB picks
the library at first load): the golden parity suite passes unchanged on it, and a table whose payload
offset points past the blob is reported as CC_E_INVALID naming the check."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEBUG_LIB = os.path.join(ROOT, "consensuscruncher_amd", "lib", "libccamd_debug.so")


def _env():
    return dict(os.environ, CCAMD_LIB=DEBUG_LIB, CC_EXPECT_DEBUG="1")


def test_golden_suite_on_the_debug_build():
    assert os.path.exists(DEBUG_LIB), "build() makes the debug library"
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-m", "gpu", "-p", "no:cacheprovider",
                        "tests/test_gpu_golden.py"], cwd=ROOT, env=_env(), capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert " passed" in r.stdout


CORRUPT = r'''
import sys
sys.path[:0] = [sys.argv[1], sys.argv[1] + "/tests", sys.argv[1] + "/oracle", sys.argv[1] + "/oracle/shim"]
import numpy as np
from consensuscruncher_amd import native as N
from consensuscruncher_amd.engine import MODE_SSCS, Bam, Engine, Interner
from test_gpu_function_abi import random_bam
assert N.amd().cc_debug_build() == 1
random_bam(sys.argv[2], 8, 150, seed=3)
rec = Bam(sys.argv[2]).decode(Interner(), MODE_SSCS, "|")
eng = Engine(0)
seq, qual, meta = eng.sscs_vote(eng.upload(rec), [0, 1, 2, 3], [0, 4], 0.7)   # intact table: fine
rec.pay_off[2] = rec.struct.payload_bytes + (1 << 20)                           # past the payload blob
try:
    eng.sscs_vote(eng.upload(rec), [0, 1, 2, 3], [0, 4], 0.7)
except N.CCError as e:
    assert e.code == -1 and "bounds check" in str(e), str(e)
    print("reported:", e)
    sys.exit(0)
sys.exit("the bad payload offset was not reported")
'''


def test_bad_payload_offset_is_reported(tmp_path):
    r = subprocess.run([sys.executable, "-c", CORRUPT, ROOT, str(tmp_path / "r.bam")], cwd=ROOT, env=_env(),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "payload offset" in r.stdout
