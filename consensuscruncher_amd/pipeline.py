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

from .engine import Sink, flush_writes, index_bam, merge_bams, merge_kept, sort_bam
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
    """ConsensusCruncher.consensus (ConsensusCruncher.py:127-346).  Each stage output the reference
    writes and then sort_index-es (X.bam -> X.sorted.bam + .bai, X.bam removed) is written sorted and
    indexed at once (engine.Sink: the same files at the end), and a stage reading the file another
    stage just wrote takes its records from memory instead of inflating it again; the merges
    (samtools merge of sorted files, then sort_index) merge the sorted records in memory and write
    X.sorted.bam + .bai directly (a stable sort of a merge of sorted inputs changes nothing)."""
    bedfile = genome_bedfile(genome, bedfile)
    identifier = os.path.basename(bam).split('.bam', 1)[0]
    sd = '{}/{}'.format(c_output, identifier)
    os.makedirs(sd + '/sscs', exist_ok=True)
    bed = None if bedfile == "False" else bedfile
    sscs = '{}/sscs/{}.sscs.bam'.format(sd, identifier)
    sing = '{}/sscs/{}.singleton.bam'.format(sd, identifier)
    dcs = '{}/dcs/{}.dcs.bam'.format(sd, identifier)
    sscs_sing = '{}/dcs/{}.sscs.singleton.bam'.format(sd, identifier)
    corr = {name: '{}/sscs/{}.{}.bam'.format(sd, identifier, name)
            for name in ("sscs.correction", "singleton.correction", "uncorrected")}
    dcs_sc = '{}/dcs_sc/{}.dcs.sc.bam'.format(sd, identifier)
    sscs_sc_sing = '{}/dcs_sc/{}.sscs.sc.singleton.bam'.format(sd, identifier)
    sc_on = scorrect != 'False'
    sink = Sink(fused=[sscs, sing, dcs, sscs_sing, dcs_sc, sscs_sc_sing] + list(corr.values()),
                keep=[sscs] + ([sing] + list(corr.values()) + [dcs_sc, sscs_sc_sing] if sc_on else []),
                async_writes=True)
    try:
        out = _stages(bam, c_output, bed, cutoff, bdelim, scorrect, engine, verbose, level, identifier, sd, sink,
                      all_unique_sscs)
    finally:
        flush_writes()   # the fused outputs compressed and written in the background
    if cleanup_files == 'True':
        cleanup(sd, identifier, scorrect)
    return out


def _stages(bam, c_output, bed, cutoff, bdelim, scorrect, engine, verbose, level, identifier, sd, sink,
            all_unique_sscs):
    """consensus_pipeline's stages (ConsensusCruncher.py:155-322)."""
    srt = lambda p: '{}.sorted.bam'.format(p.split('.bam', 1)[0])  # noqa: E731
    sscs = '{}/sscs/{}.sscs.bam'.format(sd, identifier)
    sing = '{}/sscs/{}.singleton.bam'.format(sd, identifier)
    dcs = '{}/dcs/{}.dcs.bam'.format(sd, identifier)
    sscs_sing = '{}/dcs/{}.sscs.singleton.bam'.format(sd, identifier)
    corr = {name: '{}/sscs/{}.{}.bam'.format(sd, identifier, name)
            for name in ("sscs.correction", "singleton.correction", "uncorrected")}
    dcs_sc = '{}/dcs_sc/{}.dcs.sc.bam'.format(sd, identifier)
    sscs_sc_sing = '{}/dcs_sc/{}.sscs.sc.singleton.bam'.format(sd, identifier)
    sc_on = scorrect != 'False'
    run_sscs(bam, sscs, cutoff, bedfile=bed, bdelim=bdelim, engine=engine, verbose=verbose, level=level, sink=sink)
    sscs, sing = srt(sscs), srt(sing)
    sscs_h, sing_h = sink.take(sscs), sink.take(sing)
    os.makedirs(sd + '/dcs', exist_ok=True)
    os.rename('{}/sscs/{}.stats.txt'.format(sd, identifier), '{}/dcs/{}.stats.txt'.format(sd, identifier))
    os.rename('{}/sscs/{}.time_tracker.txt'.format(sd, identifier), '{}/dcs/{}.time_tracker.txt'.format(sd, identifier))
    # Singleton correction reads the same sorted SSCS file as DCS.  Without a bed file the SSCS side's
    # per-chromosome scope is one scope (singleton_correction.py:208-229 resets nothing), so its
    # read_bam grouping equals DCS's: the SC stage then joins against the DCS run's resident grouping
    # instead of decoding, uploading and grouping the file again (same results, stages.SCRun).
    share = sc_on and bed is None
    t_dcs = time.time()
    dcs_run = DCSRun(engine or get_engine(), sscs, None if bed is None else bed, bam=sscs_h)
    try:
        dcs_run.emit(dcs, level, verbose, t_dcs, sink=sink)
    finally:
        if not share:
            dcs_run.close()
    dcs, sscs_sing = srt(dcs), srt(sscs_sing)
    out = dict(sscs=sscs, singleton=sing, dcs=dcs, sscs_singleton=sscs_sing,
               badreads='{}/sscs/{}.badReads.bam'.format(sd, identifier))
    if sc_on:
        os.makedirs(sd + '/sscs_sc', exist_ok=True)
        os.rename('{}/dcs/{}.stats.txt'.format(sd, identifier), '{}/sscs/{}.stats.txt'.format(sd, identifier))
        os.rename('{}/dcs/{}.time_tracker.txt'.format(sd, identifier),
                  '{}/sscs/{}.time_tracker.txt'.format(sd, identifier))
        try:
            run_sc(sing, bedfile=bed, engine=engine, verbose=verbose, level=level,
                   sscs_run=dcs_run if share else None, sink=sink, bam=sing_h, xbam=sscs_h)
        finally:
            dcs_run.close()
        sing_h = None
        moved, mh = {}, {}
        flush_writes()   # the corrected outputs move next
        for name, path in corr.items():
            # written sorted + indexed in sscs/ (the reference writes them there), moved like the
            # reference moves the unsorted files before sort_index
            dst = srt('{}/sscs_sc/{}.{}.bam'.format(sd, identifier, name))
            os.rename(srt(path), dst)
            os.rename(srt(path) + '.bai', dst + '.bai')
            moved[name] = dst
            mh[name] = sink.take(srt(path))
        sscs_sc = srt('{}/sscs_sc/{}.sscs.sc.bam'.format(sd, identifier))
        sscs_sc_h = merge_kept(sscs_sc, [sscs_h, mh["sscs.correction"], mh["singleton.correction"]], level,
                               async_writes=True)
        os.makedirs(sd + '/dcs_sc', exist_ok=True)
        os.rename('{}/sscs/{}.stats.txt'.format(sd, identifier), '{}/dcs_sc/{}.stats.txt'.format(sd, identifier))
        os.rename('{}/sscs/{}.time_tracker.txt'.format(sd, identifier),
                  '{}/dcs_sc/{}.time_tracker.txt'.format(sd, identifier))
        run_dcs(sscs_sc, dcs_sc, bedfile=bed, engine=engine, verbose=verbose, level=level, sink=sink, bam=sscs_sc_h)
        sscs_sc_h = None
        dcs_sc, sscs_sc_sing = srt(dcs_sc), srt(sscs_sc_sing)
        all_unique = srt('{}/dcs_sc/{}.all.unique.dcs.bam'.format(sd, identifier))
        merge_kept(all_unique, [sink.take(dcs_sc), sink.take(sscs_sc_sing), mh["uncorrected"]], level, keep=False,
                   async_writes=True)
        if all_unique_sscs:
            # legacy shell pipeline (test/bash_scripts/ConsensusCruncher.sh:261-265): SSCS + corrected
            # singletons + uncorrected singletons
            aus = srt('{}/sscs_sc/{}.all.unique.sscs.bam'.format(sd, identifier))
            merge_kept(aus, [sscs_h, mh["sscs.correction"], mh["singleton.correction"], mh["uncorrected"]], level,
                       keep=False, async_writes=True)
            out["all_unique_sscs"] = aus
        mh = None
        os.rename('{}/dcs_sc/{}.stats.txt'.format(sd, identifier), '{}/{}.stats.txt'.format(sd, identifier))
        os.rename('{}/dcs_sc/{}.time_tracker.txt'.format(sd, identifier),
                  '{}/{}.time_tracker.txt'.format(sd, identifier))
        out.update(sscs_correction=moved["sscs.correction"], singleton_correction=moved["singleton.correction"],
                   uncorrected=moved["uncorrected"], sscs_sc=sscs_sc, dcs_sc=dcs_sc, sscs_sc_singleton=sscs_sc_sing,
                   all_unique=all_unique)
    else:
        os.rename('{}/dcs/{}.stats.txt'.format(sd, identifier), '{}/{}.stats.txt'.format(sd, identifier))
        os.rename('{}/dcs/{}.time_tracker.txt'.format(sd, identifier), '{}/{}.time_tracker.txt'.format(sd, identifier))
    sscs_h = None
    os.rename('{}/sscs/{}_tag_fam_size.png'.format(sd, identifier), '{}/{}_tag_fam_size.png'.format(sd, identifier))
    os.rename('{}/sscs/{}.read_families.txt'.format(sd, identifier),
              '{}/{}.read_families.txt'.format(sd, identifier))
    out["stats"] = '{}/{}.stats.txt'.format(sd, identifier)
    out["read_families"] = '{}/{}.read_families.txt'.format(sd, identifier)
    return out
