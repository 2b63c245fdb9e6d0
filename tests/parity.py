"""Parity helpers: sorted canonical-SAM-line comparison of BAM outputs (the
"sorted record comparison" of BASELINE.json), decoded with the pysam shim so the
product's own reader is not trusted."""
import os

import pysam  # the oracle shim (tests/conftest.py puts oracle/shim on sys.path)

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def sorted_lines(path):
    return sorted(pysam.sam_lines(path))


def assert_same_records(got_path, exp_path, label=""):
    got, exp = sorted_lines(got_path), sorted_lines(exp_path)
    if got == exp:
        return len(got)
    gs, es = set(got), set(exp)
    only_g = [x for x in got if x not in es][:3]
    only_e = [x for x in exp if x not in gs][:3]
    raise AssertionError("%s: %d records vs %d expected\n only ours:\n  %s\n only reference:\n  %s" % (
        label, len(got), len(exp), "\n  ".join(only_g), "\n  ".join(only_e)))


def cases():
    return sorted(d for d in os.listdir(GOLDEN) if os.path.isdir(os.path.join(GOLDEN, d)))
