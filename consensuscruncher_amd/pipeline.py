"""consensus mode orchestration (ConsensusCruncher.py:127-346) on the GPU stages.

Same directory layout, file names, stats/time-tracker moves and merge order as
the reference; samtools sort/merge/index are replaced by libccio's stable
coordinate sort and file-ordered merge (ConsensusCruncher.py:10-34,262-266,
299-304).  No .bai is written (nothing downstream of the stages needs one).
"""
import os

from .engine import merge_bams, sort_bam
from .stages import run_dcs, run_sc, run_sscs


def sort_index(bam, level=6):
    """ConsensusCruncher.py:10-34: X.bam -> X.sorted.bam, X.bam removed."""
    out = '{}.sorted.bam'.format(bam.split('.bam', 1)[0])
    sort_bam(bam, out, level)
    os.remove(bam)
    return out


def consensus_pipeline(bam, c_output, bedfile="False", cutoff=0.7, bdelim="|", scorrect="True", engine=None,
                       verbose=False, level=6):
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
    run_dcs(sscs, dcs, bedfile=bed, engine=engine, verbose=verbose, level=level)
    dcs = sort_index(dcs, level)
    sscs_sing = sort_index(sscs_sing, level)
    out = dict(sscs=sscs, singleton=sing, dcs=dcs, sscs_singleton=sscs_sing,
               badreads='{}/sscs/{}.badReads.bam'.format(sd, identifier))
    if scorrect != 'False':
        os.makedirs(sd + '/sscs_sc', exist_ok=True)
        os.rename('{}/dcs/{}.stats.txt'.format(sd, identifier), '{}/sscs/{}.stats.txt'.format(sd, identifier))
        os.rename('{}/dcs/{}.time_tracker.txt'.format(sd, identifier),
                  '{}/sscs/{}.time_tracker.txt'.format(sd, identifier))
        run_sc(sing, bedfile=bed, engine=engine, verbose=verbose, level=level)
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
    return out
