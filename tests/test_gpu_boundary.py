"""The drop-in boundary as the reference's orchestrator drives it: ConsensusCruncher.consensus()
(ConsensusCruncher.py:127-346) launches the three stage scripts as separate processes with the argv
built at :171-185 (SSCS: no bed / --bdelim / --bedfile / both), :206-213 and :280-287 (DCS, DCS+SC)
and :230-237 (singleton correction), with samtools sort/index/merge between them.  Here those exact
command lines run our scripts (consensuscruncher_amd/{SSCS_maker,DCS_maker,singleton_correction}.py)
as subprocesses, with the samtools stand-in between, and every output must equal the in-process
pipeline's (consensuscruncher_amd/pipeline.py) and the reference's fixtures.  Also the orchestrator
rows: the genome=hg38 bed override (:145-153), cleanup (:325-346) and the legacy all.unique.sscs
product (test/bash_scripts/ConsensusCruncher.sh:261-265)."""
import json
import os
import shutil
import subprocess
import sys

import pytest

import pysam
from parity import GOLDEN, assert_same_in_order

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CODE_DIR = os.path.join(ROOT, "consensuscruncher_amd")   # where the orchestrator finds the scripts


def _run(cmd):
    """os.system(cmd) of the orchestrator: the script line, split on spaces as the shell does."""
    parts = cmd.split(" ")
    subprocess.check_call([sys.executable] + parts, cwd=ROOT)


def consensus_by_scripts(bam, c_output, bedfile="False", cutoff=0.7, bdelim="|"):
    """ConsensusCruncher.consensus() with os.system -> our scripts, samtools -> libccio."""
    from consensuscruncher_amd.engine import merge_bams
    from consensuscruncher_amd.pipeline import sort_index
    code_dir = os.path.dirname(CODE_DIR)
    identifier = os.path.basename(bam).split('.bam', 1)[0]
    sample_dir = '{}/{}'.format(c_output, identifier)
    os.makedirs(sample_dir + '/sscs')
    sscs = '{}/sscs/{}.sscs.bam'.format(sample_dir, identifier)
    sing = '{}/sscs/{}.singleton.bam'.format(sample_dir, identifier)
    pkg = "{}/consensuscruncher_amd".format(code_dir)
    if bedfile == 'False' and bdelim == '|':
        sscs_cmd = "{}/SSCS_maker.py --infile {} --outfile {} --cutoff {}".format(pkg, bam, sscs, cutoff)
    elif bedfile == 'False' and bdelim != '|':
        sscs_cmd = "{}/SSCS_maker.py --infile {} --outfile {} --cutoff {} --bdelim {}".format(
            pkg, bam, sscs, cutoff, bdelim)
    elif bedfile != 'False' and bdelim == '|':
        sscs_cmd = "{}/SSCS_maker.py --infile {} --outfile {} --cutoff {} --bedfile {}".format(
            pkg, bam, sscs, cutoff, bedfile)
    else:
        sscs_cmd = "{}/SSCS_maker.py --infile {} --outfile {} --cutoff {} --bedfile {} --bdelim {}".format(
            pkg, bam, sscs, cutoff, bedfile, bdelim)
    _run(sscs_cmd)
    sscs = sort_index(sscs)
    sing = sort_index(sing)
    os.makedirs(sample_dir + '/dcs')
    dcs = '{}/dcs/{}.dcs.bam'.format(sample_dir, identifier)
    sscs_sing = '{}/dcs/{}.sscs.singleton.bam'.format(sample_dir, identifier)
    for f in ("stats.txt", "time_tracker.txt"):
        os.rename('{}/sscs/{}.{}'.format(sample_dir, identifier, f), '{}/dcs/{}.{}'.format(sample_dir, identifier, f))
    bedarg = "" if bedfile == 'False' else " --bedfile {}".format(bedfile)
    _run("{}/DCS_maker.py --infile {} --outfile {}{}".format(pkg, sscs, dcs, bedarg))
    dcs = sort_index(dcs)
    sscs_sing = sort_index(sscs_sing)
    os.makedirs(sample_dir + '/sscs_sc')
    for f in ("stats.txt", "time_tracker.txt"):
        os.rename('{}/dcs/{}.{}'.format(sample_dir, identifier, f), '{}/sscs/{}.{}'.format(sample_dir, identifier, f))
    _run("{}/singleton_correction.py --singleton {}{}".format(pkg, sing, bedarg))
    moved = {}
    for name in ("sscs.correction", "singleton.correction", "uncorrected"):
        dst = '{}/sscs_sc/{}.{}.bam'.format(sample_dir, identifier, name)
        os.rename('{}/sscs/{}.{}.bam'.format(sample_dir, identifier, name), dst)
        moved[name] = sort_index(dst)
    sscs_sc = '{}/sscs_sc/{}.sscs.sc.bam'.format(sample_dir, identifier)
    merge_bams(sscs_sc, [sscs, moved["sscs.correction"], moved["singleton.correction"]])
    sscs_sc = sort_index(sscs_sc)
    os.makedirs(sample_dir + '/dcs_sc')
    dcs_sc = '{}/dcs_sc/{}.dcs.sc.bam'.format(sample_dir, identifier)
    for f in ("stats.txt", "time_tracker.txt"):
        os.rename('{}/sscs/{}.{}'.format(sample_dir, identifier, f), '{}/dcs_sc/{}.{}'.format(sample_dir, identifier, f))
    _run("{}/DCS_maker.py --infile {} --outfile {}{}".format(pkg, sscs_sc, dcs_sc, bedarg))
    dcs_sc = sort_index(dcs_sc)
    sscs_sc_sing = sort_index('{}/dcs_sc/{}.sscs.sc.singleton.bam'.format(sample_dir, identifier))
    all_unique = '{}/dcs_sc/{}.all.unique.dcs.bam'.format(sample_dir, identifier)
    merge_bams(all_unique, [dcs_sc, sscs_sc_sing, moved["uncorrected"]])
    all_unique = sort_index(all_unique)
    os.rename('{}/dcs_sc/{}.stats.txt'.format(sample_dir, identifier), '{}/{}.stats.txt'.format(sample_dir, identifier))
    os.rename('{}/sscs/{}.read_families.txt'.format(sample_dir, identifier),
              '{}/{}.read_families.txt'.format(sample_dir, identifier))
    return dict(sscs=sscs, singleton=sing, badreads='{}/sscs/{}.badReads.bam'.format(sample_dir, identifier),
                dcs=dcs, sscs_singleton=sscs_sing, sscs_correction=moved["sscs.correction"],
                singleton_correction=moved["singleton.correction"], uncorrected=moved["uncorrected"],
                sscs_sc=sscs_sc, dcs_sc=dcs_sc, sscs_sc_singleton=sscs_sc_sing, all_unique=all_unique,
                stats='{}/{}.stats.txt'.format(sample_dir, identifier),
                read_families='{}/{}.read_families.txt'.format(sample_dir, identifier))


@pytest.mark.parametrize("case", ["basic", "bed_multi", "cutoff_delim", "hg19_bed"])
def test_stage_scripts_as_the_orchestrator_runs_them(case, tmp_path):
    d = os.path.join(GOLDEN, case)
    kw = dict(json.load(open(os.path.join(d, "params.json")))["run"])
    if kw.get("bedfile", "False") != "False":
        kw["bedfile"] = os.path.join(d, kw["bedfile"])
    bam = str(tmp_path / "sample.bam")
    shutil.copy(os.path.join(d, "input.bam"), bam)
    out = consensus_by_scripts(bam, str(tmp_path), **kw)
    exp = os.path.join(d, "expected")
    for f in sorted(os.listdir(exp)):
        if f.endswith(".bam"):
            assert_same_in_order(out[f[:-4]], os.path.join(exp, f), "%s/%s" % (case, f))
    assert open(out["stats"]).read() == open(os.path.join(exp, "stats.txt")).read()
    assert open(out["read_families"]).read() == open(os.path.join(exp, "read_families.txt")).read()
    for k in ("sscs", "dcs", "all_unique"):
        assert os.path.exists(out[k] + ".bai")


def test_orchestrator_rows(tmp_path):
    """genome=hg38 selects the bundled hg38_cytoBand.txt; cleanup='True' removes exactly the files of
    ConsensusCruncher.py:325-346; all.unique.sscs is SSCS + corrections + uncorrected, merged."""
    from consensuscruncher_amd import synth
    from consensuscruncher_amd.pipeline import consensus_pipeline
    from consensuscruncher_amd.stages import get_engine
    import samtools_shim
    contigs = synth.band_contigs("hg38_cytoBand.txt")
    batch = synth.generate(6000, seed=synth.SEED_BASE + 801, contigs=contigs, transloc_frac=0.02)
    bam = str(tmp_path / "s.bam")
    synth.write_bam_native(batch, bam)
    eng = get_engine()
    a = consensus_pipeline(bam, str(tmp_path / "a"), genome="hg38", engine=eng, all_unique_sscs=True)
    b = consensus_pipeline(bam, str(tmp_path / "b"), bedfile=os.path.join(synth.DATA, "hg38_cytoBand.txt"),
                           engine=eng)
    for k in b:
        if k.endswith("stats") or k == "read_families":
            continue
        assert pysam.sam_lines(a[k]) == pysam.sam_lines(b[k]), k
    # legacy all.unique.sscs: the merge the shell pipeline does, through the samtools stand-in
    cp = [str(tmp_path / ("c%d.bam" % i)) for i in range(4)]
    for src, dst in zip((a["sscs"], a["sscs_correction"], a["singleton_correction"], a["uncorrected"]), cp):
        shutil.copy(src, dst)
    exp = samtools_shim.samtools_sort_index(samtools_shim.samtools_merge(str(tmp_path / "m.bam"), *cp))
    assert pysam.sam_lines(a["all_unique_sscs"]) == pysam.sam_lines(exp)
    # cleanup
    c = consensus_pipeline(bam, str(tmp_path / "c"), genome="hg38", engine=eng, cleanup_files="True")
    sd = os.path.dirname(c["stats"])
    gone = ["s.time_tracker.txt", "sscs/s.badReads.bam", "dcs/s.sscs.singleton.sorted.bam",
            "dcs/s.sscs.singleton.sorted.bam.bai", "dcs_sc/s.sscs.sc.singleton.sorted.bam",
            "dcs_sc/s.sscs.sc.singleton.sorted.bam.bai"]
    for n in ("singleton.correction", "sscs.correction", "uncorrected"):
        gone += ["sscs_sc/s.%s.sorted.bam" % n, "sscs_sc/s.%s.sorted.bam.bai" % n]
    for f in gone:
        assert not os.path.exists(os.path.join(sd, f)), f
    for k in ("sscs", "dcs", "sscs_sc", "dcs_sc", "all_unique", "stats", "read_families"):
        assert os.path.exists(c[k]), k
