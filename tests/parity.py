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


def assert_same_in_order(got_path, exp_path, label=""):
    """File-order comparison (emission order, samtools tie order) through the C++ oracle's
    canonical per-record digests; on a mismatch the first differing records are decoded."""
    import numpy as np
    import cc_oracle_native as O
    a, b = O.digests(got_path), O.digests(exp_path)
    if len(a) == len(b) and np.array_equal(a, b):
        return len(a)
    ga, gb = pysam.sam_lines(got_path), pysam.sam_lines(exp_path)
    k = next((i for i in range(min(len(ga), len(gb))) if ga[i] != gb[i]), min(len(ga), len(gb)))
    same_set = sorted(ga) == sorted(gb)
    raise AssertionError("%s: %d records vs %d expected (%s); first difference at record %d:\n ours: %s\n exp:  %s"
                         % (label, len(ga), len(gb), "same records, other order" if same_set else "records differ",
                            k, ga[k] if k < len(ga) else "-", gb[k] if k < len(gb) else "-"))


# outputs of the stages that completed before a raise (oracle/make_golden.py PARTIAL), by key
PARTIAL = {"sscs": "sscs/ID.sscs.sorted.bam", "singleton": "sscs/ID.singleton.sorted.bam",
           "badreads": "sscs/ID.badReads.bam", "dcs": "dcs/ID.dcs.sorted.bam",
           "sscs_singleton": "dcs/ID.sscs.singleton.sorted.bam",
           "sscs_correction": "sscs_sc/ID.sscs.correction.sorted.bam",
           "singleton_correction": "sscs_sc/ID.singleton.correction.sorted.bam",
           "uncorrected": "sscs_sc/ID.uncorrected.sorted.bam", "sscs_sc": "sscs_sc/ID.sscs.sc.sorted.bam"}


def check_partial(out_root, exp_dir, label, ident="sample"):
    """After a raise: every completed-stage output the reference left must match in file order."""
    n = 0
    for f in sorted(os.listdir(exp_dir)):
        if f.endswith(".bam"):
            got = os.path.join(out_root, ident, PARTIAL[f[:-4]].replace("ID", ident))
            assert os.path.exists(got), "%s: %s missing after the raise" % (label, f)
            assert pysam.sam_lines(got) == pysam.sam_lines(os.path.join(exp_dir, f)), "%s/%s" % (label, f)
            n += 1
    return n
