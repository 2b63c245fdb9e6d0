"""consensus mode orchestration (ConsensusCruncher.py:127-346) on the GPU stages.

Same directory layout, file names, stats/time-tracker moves and merge order as
the reference; samtools sort/merge/index are replaced by libccio's stable
coordinate sort, file-ordered merge and BAI writer (ConsensusCruncher.py:10-34,
262-266, 299-304).  Also mirrored: the genome=hg38/hg38_noAlt bed override
(:145-153, the bundled cytoband tables in consensuscruncher_amd/data), cleanup
(:325-346), and the legacy shell pipeline's all.unique.sscs product
(test/bash_scripts/ConsensusCruncher.sh:261-265), on request.
"""
import os
import time

from .engine import index_bam, merge_bams, sort_bam
from .stages import DCSRun, get_engine, run_dcs, run_sc, run_sscs

DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")


def sort_index(bam, level=6, index=True):
    """ConsensusCruncher.py:10-34: X.bam -> X.sorted.bam (+ X.sorted.bam.bai), X.bam removed."""
    out = '{}.sorted.bam'.format(bam.split('.bam', 1)[0])
    sort_bam(bam, out, level)
    os.remove(bam)
    if index:
        index_bam(out)
    return out


def genome_bedfile(genome, bedfile):
    """ConsensusCruncher.py:145-153: hg38 / hg38_noAlt replace the bed file with the bundled cytobands."""
    if genome == 'hg38':
        return os.path.join(DATA, 'hg38_cytoBand.txt')
    if genome == 'hg38_noAlt':
        return os.path.join(DATA, 'hg38_noAlt_cytoBand.txt')
    return bedfile


def cleanup(sd, identifier, scorrect):
    """ConsensusCruncher.py:325-346: remove the intermediate files (cleanup == 'True')."""
    os.remove('{}/{}.time_tracker.txt'.format(sd, identifier))
    os.remove('{}/sscs/{}.badReads.bam'.format(sd, identifier))
    os.remove('{}/dcs/{}.sscs.singleton.sorted.bam'.format(sd, identifier))
    os.remove('{}/dcs/{}.sscs.singleton.sorted.bam.bai'.format(sd, identifier))
    if scorrect != 'False':
        for name in ('singleton.correction', 'sscs.correction', 'uncorrected'):
            os.remove('{}/sscs_sc/{}.{}.sorted.bam'.format(sd, identifier, name))
            os.remove('{}/sscs_sc/{}.{}.sorted.bam.bai'.format(sd, identifier, name))
        os.remove('{}/dcs_sc/{}.sscs.sc.singleton.sorted.bam'.format(sd, identifier))
        os.remove('{}/dcs_sc/{}.sscs.sc.singleton.sorted.bam.bai'.format(sd, identifier))


def consensus_pipeline(bam, c_output, bedfile="False", cutoff=0.7, bdelim="|", scorrect="True", engine=None,
                       verbose=False, level=6, genome=None, cleanup_files="False", all_unique_sscs=False):
    bedfile = genome_bedfile(genome, bedfile)
    identifier = os.path.basename(bam).split('.bam', 1)[0]
    sd = '{}/{}'.format(c_output, identifier)
    os.makedirs(sd + '/sscs', exist_ok=True)
    bed = None if bedfile == "False" else bedfile
    sscs = '{}/sscs/{}.sscs.bam'.format(sd, identifier)
    sing = '{}/sscs/{}.singleton.bam'.format(sd, identifier)
    run_sscs(bam, sscs, cutoff, bedfile=bed, bdelim=bdelim, engine=engine, verbose=verbose, level=level)
    sscs = sort_index(sscs, level)
    sing = sort_index(sing, level)
    os.makedirs(sd + '/dcs', exist_ok=True)
    dcs = '{}/dcs/{}.dcs.bam'.format(sd, identifier)
    sscs_sing = '{}/dcs/{}.sscs.singleton.bam'.format(sd, identifier)
    os.rename('{}/sscs/{}.stats.txt'.format(sd, identifier), '{}/dcs/{}.stats.txt'.format(sd, identifier))
    os.rename('{}/sscs/{}.time_tracker.txt'.format(sd, identifier), '{}/dcs/{}.time_tracker.txt'.format(sd, identifier))
    # Singleton correction reads the same sorted SSCS file as DCS.  Without a bed file the SSCS side's
    # per-chromosome scope is one scope (singleton_correction.py:208-229 resets nothing), so its
    # read_bam grouping equals DCS's: the SC stage then joins against the DCS run's resident grouping
    # instead of decoding, uploading and grouping the file again (same results, stages.SCRun).
    share = scorrect != 'False' and bed is None
    t_dcs = time.time()
    dcs_run = DCSRun(engine or get_engine(), sscs, None if bed is None else bed)
    try:
        dcs_run.emit(dcs, level, verbose, t_dcs)
    finally:
        if not share:
            dcs_run.close()
    dcs = sort_index(dcs, level)
    sscs_sing = sort_index(sscs_sing, level)
    out = dict(sscs=sscs, singleton=sing, dcs=dcs, sscs_singleton=sscs_sing,
               badreads='{}/sscs/{}.badReads.bam'.format(sd, identifier))
    if scorrect != 'False':
        os.makedirs(sd + '/sscs_sc', exist_ok=True)
        os.rename('{}/dcs/{}.stats.txt'.format(sd, identifier), '{}/sscs/{}.stats.txt'.format(sd, identifier))
        os.rename('{}/dcs/{}.time_tracker.txt'.format(sd, identifier),
                  '{}/sscs/{}.time_tracker.txt'.format(sd, identifier))
        try:
            run_sc(sing, bedfile=bed, engine=engine, verbose=verbose, level=level,
                   sscs_run=dcs_run if share else None)
        finally:
            dcs_run.close()
        moved = {}
        for name in ("sscs.correction", "singleton.correction", "uncorrected"):
            dst = '{}/sscs_sc/{}.{}.bam'.format(sd, identifier, name)
            os.rename('{}/sscs/{}.{}.bam'.format(sd, identifier, name), dst)
            moved[name] = sort_index(dst, level)
        sscs_sc = '{}/sscs_sc/{}.sscs.sc.bam'.format(sd, identifier)
        merge_bams(sscs_sc, [sscs, moved["sscs.correction"], moved["singleton.correction"]], level)
        sscs_sc = sort_index(sscs_sc, level)
        os.makedirs(sd + '/dcs_sc', exist_ok=True)
        dcs_sc = '{}/dcs_sc/{}.dcs.sc.bam'.format(sd, identifier)
        os.rename('{}/sscs/{}.stats.txt'.format(sd, identifier), '{}/dcs_sc/{}.stats.txt'.format(sd, identifier))
        os.rename('{}/sscs/{}.time_tracker.txt'.format(sd, identifier),
                  '{}/dcs_sc/{}.time_tracker.txt'.format(sd, identifier))
        run_dcs(sscs_sc, dcs_sc, bedfile=bed, engine=engine, verbose=verbose, level=level)
        dcs_sc = sort_index(dcs_sc, level)
        sscs_sc_sing = sort_index('{}/dcs_sc/{}.sscs.sc.singleton.bam'.format(sd, identifier), level)
        all_unique = '{}/dcs_sc/{}.all.unique.dcs.bam'.format(sd, identifier)
        merge_bams(all_unique, [dcs_sc, sscs_sc_sing, moved["uncorrected"]], level)
        all_unique = sort_index(all_unique, level)
        if all_unique_sscs:
            # legacy shell pipeline (test/bash_scripts/ConsensusCruncher.sh:261-265): SSCS + corrected
            # singletons + uncorrected singletons
            aus = '{}/sscs_sc/{}.all.unique.sscs.bam'.format(sd, identifier)
            merge_bams(aus, [sscs, moved["sscs.correction"], moved["singleton.correction"], moved["uncorrected"]],
                       level)
            out["all_unique_sscs"] = sort_index(aus, level)
        os.rename('{}/dcs_sc/{}.stats.txt'.format(sd, identifier), '{}/{}.stats.txt'.format(sd, identifier))
        os.rename('{}/dcs_sc/{}.time_tracker.txt'.format(sd, identifier),
                  '{}/{}.time_tracker.txt'.format(sd, identifier))
        out.update(sscs_correction=moved["sscs.correction"], singleton_correction=moved["singleton.correction"],
                   uncorrected=moved["uncorrected"], sscs_sc=sscs_sc, dcs_sc=dcs_sc, sscs_sc_singleton=sscs_sc_sing,
                   all_unique=all_unique)
    else:
        os.rename('{}/dcs/{}.stats.txt'.format(sd, identifier), '{}/{}.stats.txt'.format(sd, identifier))
        os.rename('{}/dcs/{}.time_tracker.txt'.format(sd, identifier), '{}/{}.time_tracker.txt'.format(sd, identifier))
    os.rename('{}/sscs/{}_tag_fam_size.png'.format(sd, identifier), '{}/{}_tag_fam_size.png'.format(sd, identifier))
    os.rename('{}/sscs/{}.read_families.txt'.format(sd, identifier),
              '{}/{}.read_families.txt'.format(sd, identifier))
    out["stats"] = '{}/{}.stats.txt'.format(sd, identifier)
    out["read_families"] = '{}/{}.read_families.txt'.format(sd, identifier)
    if cleanup_files == 'True':
        cleanup(sd, identifier, scorrect)
    return out
