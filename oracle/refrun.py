"""Run the REFERENCE stage scripts in-process (this container only).

TEST INFRASTRUCTURE — the golden-fixture generator.  Never imported by the
product and never shipped to the GPU box (the reference does not travel).

* injects the pure-Python pysam shim (oracle/shim/pysam) into sys.modules;
* imports /root/reference/ConsensusCruncher/{consensus_helper,SSCS_maker,
  DCS_maker,singleton_correction}.py unmodified;
* patches ``consensus_helper.randint = lambda a, b: a`` so that the mode tie
  breaks in read_mode / consensus_flag (consensus_helper.py:522,561) pick the
  first-seen value;
* provides a samtools stand-in (stable coordinate sort, merge with file-order
  tie break: SURVEY.md Q7) and the consensus() orchestration of
  ConsensusCruncher.py:127-346 without subprocesses.
"""
import contextlib
import io
import os
import struct
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REF_ROOT = "/root/reference"
REF_PKG = os.path.join(REF_ROOT, "ConsensusCruncher")

_mods = None


def load_reference():
    global _mods
    if _mods is not None:
        return _mods
    shim = os.path.join(HERE, "shim")
    if shim not in sys.path:
        sys.path.insert(0, shim)
    if REF_PKG not in sys.path:
        sys.path.insert(0, REF_PKG)
    os.environ.pop("DISPLAY", None)
    import pysam  # noqa: F401  (the shim)
    import consensus_helper
    import SSCS_maker
    import DCS_maker
    import singleton_correction
    consensus_helper.randint = lambda a, b: a
    DCS_maker.time = time          # DCS_maker.main uses the __main__-only `time` import
    _mods = dict(helper=consensus_helper, sscs=SSCS_maker, dcs=DCS_maker, sc=singleton_correction)
    return _mods


def run_main(module, argv):
    """Call module.main() with argv; return captured stdout."""
    old = sys.argv
    sys.argv = [module.__file__] + list(argv)
    buf = io.StringIO()
    try:
        with contextlib.redirect_stdout(buf):
            module.main()
    finally:
        sys.argv = old
        try:
            import matplotlib.pyplot as plt
            plt.close("all")
        except Exception:
            pass
    return buf.getvalue()


from samtools_shim import samtools_merge, samtools_sort_index  # noqa: E402,F401


def load_extract():
    """The reference's extract_barcodes.py, unmodified, on the Biopython stand-in (oracle/shim/Bio)."""
    shim = os.path.join(HERE, "shim")
    if shim not in sys.path:
        sys.path.insert(0, shim)
    if REF_PKG not in sys.path:
        sys.path.insert(0, REF_PKG)
    import warnings
    warnings.filterwarnings("ignore", category=DeprecationWarning)   # open(..., "rU") at :204-205
    import extract_barcodes
    return extract_barcodes


def run_extract(argv):
    """extract_barcodes.main() with argv (its stderr counts are not captured)."""
    return run_main(load_extract(), argv)


def consensus_pipeline(bam, c_output, bedfile="False", cutoff=0.7, bdelim="|", scorrect="True"):
    """ConsensusCruncher.py:127-346 (consensus mode) with in-process stages and the
    samtools stand-in.  Returns dict of output paths and captured stdout."""
    m = load_reference()
    identifier = os.path.basename(bam).split(".bam", 1)[0]
    sd = "%s/%s" % (c_output, identifier)
    os.makedirs(sd + "/sscs", exist_ok=True)
    sscs = "%s/sscs/%s.sscs.bam" % (sd, identifier)
    sing = "%s/sscs/%s.singleton.bam" % (sd, identifier)
    argv = ["--infile", bam, "--outfile", sscs, "--cutoff", str(cutoff)]
    if bedfile != "False":
        argv += ["--bedfile", bedfile]
    if bdelim != "|":
        argv += ["--bdelim", bdelim]
    log = {"sscs": run_main(m["sscs"], argv)}
    sscs = samtools_sort_index(sscs)
    sing = samtools_sort_index(sing)
    os.makedirs(sd + "/dcs", exist_ok=True)
    dcs = "%s/dcs/%s.dcs.bam" % (sd, identifier)
    sscs_sing = "%s/dcs/%s.sscs.singleton.bam" % (sd, identifier)
    os.rename("%s/sscs/%s.stats.txt" % (sd, identifier), "%s/dcs/%s.stats.txt" % (sd, identifier))
    os.rename("%s/sscs/%s.time_tracker.txt" % (sd, identifier), "%s/dcs/%s.time_tracker.txt" % (sd, identifier))
    argv = ["--infile", sscs, "--outfile", dcs] + (["--bedfile", bedfile] if bedfile != "False" else [])
    log["dcs"] = run_main(m["dcs"], argv)
    dcs = samtools_sort_index(dcs)
    sscs_sing = samtools_sort_index(sscs_sing)
    out = dict(sscs=sscs, singleton=sing, dcs=dcs, sscs_singleton=sscs_sing,
               badreads="%s/sscs/%s.badReads.bam" % (sd, identifier))
    if scorrect != "False":
        os.makedirs(sd + "/sscs_sc", exist_ok=True)
        os.rename("%s/dcs/%s.stats.txt" % (sd, identifier), "%s/sscs/%s.stats.txt" % (sd, identifier))
        os.rename("%s/dcs/%s.time_tracker.txt" % (sd, identifier), "%s/sscs/%s.time_tracker.txt" % (sd, identifier))
        argv = ["--singleton", sing] + (["--bedfile", bedfile] if bedfile != "False" else [])
        log["sc"] = run_main(m["sc"], argv)
        moved = {}
        for name in ("sscs.correction", "singleton.correction", "uncorrected"):
            dst = "%s/sscs_sc/%s.%s.bam" % (sd, identifier, name)
            os.rename("%s/sscs/%s.%s.bam" % (sd, identifier, name), dst)
            moved[name] = samtools_sort_index(dst)
        sscs_sc = "%s/sscs_sc/%s.sscs.sc.bam" % (sd, identifier)
        samtools_merge(sscs_sc, sscs, moved["sscs.correction"], moved["singleton.correction"])
        sscs_sc = samtools_sort_index(sscs_sc)
        os.makedirs(sd + "/dcs_sc", exist_ok=True)
        dcs_sc = "%s/dcs_sc/%s.dcs.sc.bam" % (sd, identifier)
        os.rename("%s/sscs/%s.stats.txt" % (sd, identifier), "%s/dcs_sc/%s.stats.txt" % (sd, identifier))
        os.rename("%s/sscs/%s.time_tracker.txt" % (sd, identifier), "%s/dcs_sc/%s.time_tracker.txt" % (sd, identifier))
        argv = ["--infile", sscs_sc, "--outfile", dcs_sc] + (["--bedfile", bedfile] if bedfile != "False" else [])
        log["dcs_sc"] = run_main(m["dcs"], argv)
        dcs_sc = samtools_sort_index(dcs_sc)
        sscs_sc_sing = samtools_sort_index("%s/dcs_sc/%s.sscs.sc.singleton.bam" % (sd, identifier))
        all_unique = "%s/dcs_sc/%s.all.unique.dcs.bam" % (sd, identifier)
        samtools_merge(all_unique, dcs_sc, sscs_sc_sing, moved["uncorrected"])
        all_unique = samtools_sort_index(all_unique)
        os.rename("%s/dcs_sc/%s.stats.txt" % (sd, identifier), "%s/%s.stats.txt" % (sd, identifier))
        out.update(sscs_correction=moved["sscs.correction"], singleton_correction=moved["singleton.correction"],
                   uncorrected=moved["uncorrected"], sscs_sc=sscs_sc, dcs_sc=dcs_sc,
                   sscs_sc_singleton=sscs_sc_sing, all_unique=all_unique)
    else:
        os.rename("%s/dcs/%s.stats.txt" % (sd, identifier), "%s/%s.stats.txt" % (sd, identifier))
    out["stats"] = "%s/%s.stats.txt" % (sd, identifier)
    out["read_families"] = "%s/sscs/%s.read_families.txt" % (sd, identifier)
    out["log"] = log
    return out
