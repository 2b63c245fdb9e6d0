"""Known answers the reference itself states (docstrings, help text), checked
against the oracle, the host helpers, the native name formatter and (gpu) the
HIP engine."""
import os

import pytest

import cc_oracle
import pysam
from consensuscruncher_amd import consensus_helper as H
from consensuscruncher_amd import native as N

# SSCS_maker.py:27-35 / docs/source/sscs.rst: cutoff 0.7 over these four reads -> ACTGATACNT
WORKED = ["ACTGATACTT", "ACTGAAACCT", "ACTGATACCT", "ACTGATACTT"]


def worked_bam(path):
    hdr = pysam.AlignmentHeader("@HD\tVN:1.6\tSO:coordinate\n@SQ\tSN:chr1\tLN:10000\n", [("chr1", 10000)])
    recs = []
    for i, s in enumerate(WORKED):
        for pos, flag, seq in ((100, 99, s), (300, 147, "GGGGGGGGGG")):
            r = pysam.AlignedSegment(hdr)
            r.query_name = "read%d|AC.GT" % i
            r.flag = flag
            r.reference_id = 0
            r.reference_start = pos
            r.mapping_quality = 60
            r.cigartuples = [(0, 10)]
            r.next_reference_id = 0
            r.next_reference_start = 400 - pos
            r.template_length = 210 if flag == 99 else -210
            r.query_sequence = seq
            r.query_qualities = [40] * 10
            recs.append(r)
    recs.sort(key=lambda r: r.reference_start)
    pysam.write_bam_file(path, hdr, recs)
    return path


def test_which_read_doctest():
    # consensus_helper.py:61-67
    assert H.which_read(83) == "R1" and H.which_read(131) == "R2" and H.which_read(177) == "R2"
    assert cc_oracle.read_number(83) == "R1" and cc_oracle.read_number(177) == "R2"


def test_duplex_tag_current_behaviour():
    # consensus_helper.py:654-661 docstring expectations carry stale 'neg_'/'pos_' tokens; the code
    # swaps the barcode halves and R1<->R2 only, which is what the kernels implement.
    assert H.duplex_tag("GTCT_1_1507809_7_55224319_98M_98M_fwd_R1") == "CTGT_1_1507809_7_55224319_98M_98M_fwd_R2"
    assert H.duplex_tag("CTGT_7_55224319_1_1507809_98M_98M_rev_R1") == "GTCT_7_55224319_1_1507809_98M_98M_rev_R2"
    assert H.duplex_tag("AC.GTA_1_2_3_4_5M_5M_fwd_R2") == "GTA.AC_1_2_3_4_5M_5M_fwd_R1"
    for t in ("GTCT_1_1507809_7_55224319_98M_98M_fwd_R1", "AC.GTA_1_2_3_4_5M_5M_rev_R2"):
        assert cc_oracle.complement_key(t) == H.duplex_tag(t)


@pytest.mark.parametrize("tag,ds,want", [
    # DCS_maker.py:67-74 doctests
    ("TTCA_7_55259315_7_55259454_98M_98M_neg:3", "CATT_7_55259315_7_55259454_98M_98M_pos:6",
     "CATT_TTCA_7_55259315_7_55259454_98M_98M:6_3"),
    ("CTTC_23_74804535_23_74804611_98M_98M_pos:2", "TCCT_23_74804535_23_74804611_98M_98M_neg:3",
     "CTTC_TCCT_23_74804535_23_74804611_98M_98M:2_3"),
    ("TTTC_7_140477735_7_140477790_98M_98M_neg:3", "TCTT_7_140477735_7_140477790_98M_98M_pos:2",
     "TCTT_TTTC_7_140477735_7_140477790_98M_98M:2_3"),
])
def test_dcs_consensus_tag_doctests(tag, ds, want):
    import ctypes
    buf = ctypes.create_string_buffer(512)
    n = N.io().ccio_dcs_name(tag.encode(), ds.encode(), buf, 512)
    assert n == len(want) and buf.value.decode() == want
    assert cc_oracle.duplex_name(tag, ds) == want


def test_cutoff_semantics():
    # 10c >= 7p for 0.7 is the Python float rule for small p; the GPU evaluates the same double division
    for p in range(1, 2000):
        for c in (int(0.7 * p) - 1, int(0.7 * p), int(0.7 * p) + 1):
            if 0 <= c <= p:
                assert H.cutoff_pass(c, p, 0.7) == (c / p >= 0.7)


def test_worked_example_oracle(tmp_path):
    bam = worked_bam(str(tmp_path / "w.bam"))
    cc_oracle.sscs_stage(bam, str(tmp_path / "w.sscs.bam"), 0.7)
    got = {r.flag: r for r in pysam.AlignmentFile(str(tmp_path / "w.sscs.bam")).fetch(until_eof=True)}
    assert got[99].query_sequence == "ACTGATACNT"
    assert list(got[99].query_qualities) == [60] * 10


@pytest.mark.gpu
def test_worked_example_gpu(tmp_path):
    from consensuscruncher_amd.stages import run_sscs
    bam = worked_bam(str(tmp_path / "w.bam"))
    run_sscs(bam, str(tmp_path / "w.sscs.bam"), 0.7, verbose=False)
    got = {r.flag: r for r in pysam.AlignmentFile(str(tmp_path / "w.sscs.bam")).fetch(until_eof=True)}
    assert got[99].query_sequence == "ACTGATACNT"
    assert list(got[99].query_qualities) == [60] * 10
    assert got[99].query_name == "AC.GT_0_100_0_300_10M_10M_pos_210:4"


def test_duplex_tag_matches_the_restatement():
    """ccio_duplex_tag (libccio, the function-level duplex_tag) against the oracle's restatement of
    consensus_helper.py:639-683 on tags with '.'-separated, even and odd barcodes, and the
    reference's IndexError for a tag of fewer than nine fields."""
    import numpy as np
    import pytest
    import cc_oracle
    from consensuscruncher_amd.engine import duplex_tag
    rng = np.random.default_rng(5)
    for _ in range(3000):
        k = int(rng.integers(0, 4))
        bc = {0: "".join(rng.choice(list("ACGT"), int(rng.integers(0, 7)))),
              1: "AC.GTT", 2: "..A", 3: "ACGT."}[k]
        fields = [bc] + [str(int(x)) for x in rng.integers(0, 99, 7)] + [str(rng.choice(["R1", "R2", "None", "x"]))]
        fields += [str(int(x)) for x in rng.integers(0, 9, int(rng.integers(0, 3)))]
        t = "_".join(fields)
        assert duplex_tag(t) == cc_oracle.complement_key(t), t
    with pytest.raises(IndexError):
        duplex_tag("AC.GT_1_2_3")
