"""Generate golden fixtures under tests/golden/ by running the REFERENCE.

TEST INFRASTRUCTURE, runs only in the build container (needs /root/reference).
For every case: a seeded synthetic input BAM (written through the pysam shim),
the reference consensus pipeline (oracle/refrun.py: the unmodified stage
scripts + a stable samtools stand-in, randint patched to pick the first tie),
and its outputs copied next to the input:
    tests/golden/<case>/input.bam [, regions.bed], params.json,
    expected/<output>.bam, expected/stats.txt, expected/read_families.txt,
    expected/error.txt (cases where the reference raises)
Usage: python oracle/make_golden.py [case ...]
"""
import json
import os
import shutil
import sys
import tempfile
import traceback

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402

import refrun  # noqa: E402
import synthbam  # noqa: E402
from consensuscruncher_amd import synth  # noqa: E402

GOLDEN = os.path.join(ROOT, "tests", "golden")

OUTPUTS = ["sscs", "singleton", "badreads", "dcs", "sscs_singleton", "sscs_correction", "singleton_correction",
           "uncorrected", "sscs_sc", "dcs_sc", "sscs_sc_singleton", "all_unique"]


# completed-stage outputs kept when the reference raises later in the pipeline
PARTIAL = {"sscs": "sscs/ID.sscs.sorted.bam", "singleton": "sscs/ID.singleton.sorted.bam",
           "badreads": "sscs/ID.badReads.bam", "dcs": "dcs/ID.dcs.sorted.bam",
           "sscs_singleton": "dcs/ID.sscs.singleton.sorted.bam",
           "sscs_correction": "sscs_sc/ID.sscs.correction.sorted.bam",
           "singleton_correction": "sscs_sc/ID.singleton.correction.sorted.bam",
           "uncorrected": "sscs_sc/ID.uncorrected.sorted.bam", "sscs_sc": "sscs_sc/ID.sscs.sc.sorted.bam"}


def hg19_contigs():
    ends = {}
    for line in open(os.path.join(refrun.REF_PKG, "hg19_cytoBand.txt")):
        c = line.split("\t")
        ends[c[0]] = max(ends.get(c[0], 0), int(c[2]))
    return list(ends.items())


def case_defs():
    return {
        # default C2-like model, -b False
        "basic": dict(gen=dict(n_pairs=1500, seed=synth.SEED_BASE + 2, contigs=(("chr1", 300_000),)),
                      run=dict(bedfile="False", cutoff=0.7)),
        # 126 bp reads, mostly singletons (C1 surrogate: bundled FASTQ length, low duplication)
        "c1_surrogate": dict(gen=dict(n_pairs=1200, seed=synth.SEED_BASE + 1, read_len=126, fam_mean=0.3,
                                      contigs=(("chr1", 400_000),)),
                             run=dict(bedfile="False", cutoff=0.7)),
        # several contigs, translocations, a bed with non-consecutive regions per contig and a contig
        # left out of the bed (reads dropped, translocated mates stuck in pair_dict)
        "bed_multi": dict(gen=dict(n_pairs=1500, seed=synth.SEED_BASE + 3, transloc_frac=0.05,
                                   contigs=(("chr1", 200_000), ("chr2", 150_000), ("chr3", 100_000))),
                          bed=[("chr1", 0, 90_000, "p1"), ("chr2", 0, 150_000, "p1"), ("chr1", 90_000, 200_000, "q1")],
                          run=dict(cutoff=0.7)),
        # variable-length barcode list, 70% singletons (C5)
        "c5_list": dict(gen=dict(n_pairs=1500, seed=synth.SEED_BASE + 5, barcode_mode="list", singleton_frac=0.7,
                                 contigs=(("chr1", 300_000),)),
                        run=dict(bedfile="False", cutoff=0.7)),
        # skewed family sizes on a few loci (C4 shape)
        "c4_skew": dict(gen=dict(n_pairs=500, seed=synth.SEED_BASE + 4, loci=4, zipf_s=1.5, max_fam=120,
                                 contigs=(("chr1", 400_000),)),
                        run=dict(bedfile="False", cutoff=0.7)),
        # other cutoff, custom delimiter
        "cutoff_delim": dict(gen=dict(n_pairs=1200, seed=synth.SEED_BASE + 6, contigs=(("chr1", 300_000),)),
                             delim="+", run=dict(bedfile="False", cutoff=0.51, bdelim="+")),
        # the bundled hg19 cytoband bed (genome hg19 default) over an hg19-named header
        "hg19_bed": dict(gen=dict(n_pairs=1500, seed=synth.SEED_BASE + 7, transloc_frac=0.02,
                                  contigs=None), hg19=True, run=dict(cutoff=0.7)),
        # read_bam dictionary quirks: shared consensus tags (NOT UNIQUE orphans), tag == mate tag drops
        "quirks": dict(gen=dict(n_pairs=1500, seed=synth.SEED_BASE + 9, quirk_frac=0.05,
                                contigs=(("chr1", 300_000),)), run=dict(bedfile="False", cutoff=0.7)),
        # odd-length barcodes without '.': duplex_tag is not an involution (consensus_helper.py:663-674), plus
        # chains t -> duplex(t) -> duplex(duplex(t)); several contigs, translocations, a bed (SC resets)
        "nonmutual": dict(gen=dict(n_pairs=2000, seed=synth.SEED_BASE + 10, barcode_mode="odd", chain_frac=0.2,
                                   transloc_frac=0.03, contigs=(("chr1", 200_000), ("chr2", 150_000))),
                          bed=[("chr1", 0, 100_000, "p1"), ("chr1", 100_000, 200_000, "q1"), ("chr2", 0, 150_000, "p1")],
                          run=dict(cutoff=0.7)),
        # qnames seen three and four times (a shifted third record, an interleaved second pair, exact
        # duplicate records): pair_dict pairs occurrences in stream order (consensus_helper.py:426-432)
        "dup_qname": dict(gen=dict(n_pairs=1500, seed=synth.SEED_BASE + 11, dupq_frac=0.05,
                                   contigs=(("chr1", 300_000),)), run=dict(bedfile="False", cutoff=0.7)),
        # records not coordinate-sorted (fetch(until_eof=True) order), no bed
        "unsorted": dict(gen=dict(n_pairs=1500, seed=synth.SEED_BASE + 12, shuffle=True, transloc_frac=0.02,
                                  contigs=(("chr1", 300_000), ("chr2", 100_000))),
                         run=dict(bedfile="False", cutoff=0.7)),
        # C1 surrogate from the bundled test FASTQ: the first 4000 pairs of
        # LargeMid_56, barcodes extracted per NNT by the reference's extract_barcodes.py, placed at
        # sequence-derived coordinates (synth.fastq_surrogate; no bwa or genome here)
        "c1_fastq": dict(fastq=("LargeMid_56_L005", 4000, "NNT"), gen=dict(seed=synth.SEED_BASE + 1),
                         run=dict(bedfile="False", cutoff=0.7)),
        # overlapping bed regions: reads in the overlap are fetched by both regions; a pair completed in
        # the first is completed again in the second, after its families were emitted and deleted
        # (read_dict[tag] KeyError, consensus_helper.py:490)
        "bed_overlap": dict(gen=dict(n_pairs=1200, seed=synth.SEED_BASE + 13, contigs=(("chr1", 300_000),)),
                            bed=[("chr1", 0, 130_000, "p1"), ("chr1", 100_000, 300_000, "q1")],
                            run=dict(cutoff=0.7)),
        # N at Q>=30 inside a family: the reference raises IndexError (SSCS_maker.py:129)
        "err_n_highq": dict(gen=dict(n_pairs=300, seed=synth.SEED_BASE + 8, contigs=(("chr1", 100_000),)),
                            inject_n_highq=True, run=dict(bedfile="False", cutoff=0.7)),
    }


def fastq_batch(sample, pairs, pattern, seed, tmp):
    """The reference's own UMI extraction on the first `pairs` pairs of a bundled FASTQ, then the
    sequence-derived placement of synth.fastq_surrogate."""
    src = os.path.join(refrun.REF_ROOT, "test", "fastq", sample + "_R%d.fastq")
    work = os.path.join(tmp, "fq_" + sample)
    os.makedirs(work)
    for k in (1, 2):
        with open(src % k) as f, open(os.path.join(work, "in_R%d.fastq" % k), "w") as g:
            for _ in range(4 * pairs):
                g.write(next(f))
    out = os.path.join(work, "tag", "s")
    os.makedirs(os.path.dirname(out))
    refrun.run_extract(["--read1", os.path.join(work, "in_R1.fastq"), "--read2", os.path.join(work, "in_R2.fastq"),
                        "--outfile", out, "--bpattern", pattern])
    return synth.fastq_surrogate(out + "_barcode_R1.fastq", out + "_barcode_R2.fastq", seed=seed)


def make_case(name, d, tmp):
    gen = dict(d["gen"])
    if d.get("fastq"):
        batch = fastq_batch(*d["fastq"], seed=gen["seed"], tmp=tmp)
        gen["fastq"] = d["fastq"]
    else:
        batch = None
    if d.get("hg19"):
        ctg = hg19_contigs()
        # reads on chr1/chr2/chr10 only, header lists every hg19 contig (fetch needs them all)
        gen["contigs"] = tuple((c, 600_000) for c, _ in ctg if c in ("chr1", "chr2", "chr10"))
    if batch is None:
        batch = synth.generate(**gen)
    if d.get("hg19"):
        keep = [n for n, _ in ctg]
        remap = np.array([keep.index(n) for n in batch.names], np.int32)
        for f in ("tid", "mtid"):
            v = getattr(batch, f)
            setattr(batch, f, np.where(v >= 0, remap[np.maximum(v, 0)], v).astype(np.int32))
        batch.names = keep
        batch.lens = [600_000 if n in ("chr1", "chr2", "chr10") else l for n, l in ctg]
        # re-sort: tids changed
        tkey = batch.tid.astype(np.int64)
        tkey[tkey < 0] = 1 << 40
        order = np.lexsort((np.arange(batch.n), (batch.flag & 0x10) > 0, batch.pos.astype(np.int64) + 1, tkey))
        for f in ("pair", "tid", "pos", "mtid", "mpos", "tlen", "flag", "mapq", "cig", "bc", "rg", "seq", "qual",
                  "spacer_bad"):
            setattr(batch, f, getattr(batch, f)[order])
    if d.get("inject_n_highq"):
        # a read of a multi-read family gets N at Q35 at position 10
        fam = {}
        for i in range(batch.n):
            if batch.flag[i] in (99, 147) and not batch.spacer_bad[i]:
                fam.setdefault((batch.tid[i], batch.pos[i], batch.cig[i], batch.bc[i], batch.flag[i]), []).append(i)
        big = [v for v in fam.values() if len(v) >= 3]
        i = big[0][1]
        batch.seq[i, 10] = ord("N")
        batch.qual[i, 10] = 35
    out = os.path.join(GOLDEN, name)
    if os.path.exists(out):
        shutil.rmtree(out)
    os.makedirs(os.path.join(out, "expected"))
    inp = os.path.join(out, "input.bam")
    synthbam.write_batch(batch, inp, level=9, delim=d.get("delim", "|"))
    run = dict(d["run"])
    if "bed" in d:
        bed = os.path.join(out, "regions.bed")
        with open(bed, "w") as f:
            for c, s, e, arm in d["bed"]:
                f.write("%s\t%d\t%d\t%s\tgneg\n" % (c, s, e, arm))
        run["bedfile"] = "regions.bed"
    if d.get("hg19"):
        # cytoband-like bed over the hg19 contigs in the bundled file's contig order (chrM, chr1, chr10, ...),
        # band boundaries drawn at random (the bundled file itself is not copied)
        rng = np.random.default_rng(gen["seed"])
        with open(os.path.join(out, "cytoband_like.bed"), "w") as f:
            for c, ln in [(n, 600_000 if n in ("chr1", "chr2", "chr10") else l) for n, l in hg19_contigs()]:
                s0, k = 0, 0
                while s0 < ln:
                    e0 = min(ln, s0 + int(rng.integers(20_000, 80_000)) if c in ("chr1", "chr2", "chr10")
                             else ln)
                    f.write("%s\t%d\t%d\t%s%d\tgneg\n" % (c, s0, e0, "p" if k % 2 == 0 else "q", k))
                    s0, k = e0, k + 1
        run["bedfile"] = "cytoband_like.bed"
    with open(os.path.join(out, "params.json"), "w") as f:
        json.dump(dict(run=run, gen={k: v for k, v in gen.items() if k != "contigs"}), f, indent=1, default=str)
    work = os.path.join(tmp, name)
    os.makedirs(work)
    shutil.copy(inp, os.path.join(work, "sample.bam"))
    kw = dict(run)
    if kw.get("bedfile", "False") != "False":
        kw["bedfile"] = os.path.join(out, kw["bedfile"])
    try:
        res = refrun.consensus_pipeline(os.path.join(work, "sample.bam"), work, **kw)
    except Exception as e:
        with open(os.path.join(out, "expected", "error.txt"), "w") as f:
            f.write("%s: %s\n" % (type(e).__name__, e))
            f.write(traceback.format_exc())
        # the outputs of the stages that completed before the raise (same file layout as the pipeline)
        got = []
        for k, rel in PARTIAL.items():
            src = os.path.join(work, "sample", rel.replace("ID", "sample"))
            if os.path.exists(src):
                shutil.copy(src, os.path.join(out, "expected", k + ".bam"))
                got.append(k)
        print(name, "-> reference raised", type(e).__name__, "; partial outputs:", got)
        return
    for k in OUTPUTS:
        if k in res:
            shutil.copy(res[k], os.path.join(out, "expected", k + ".bam"))
    shutil.copy(res["stats"], os.path.join(out, "expected", "stats.txt"))
    shutil.copy(res["read_families"], os.path.join(out, "expected", "read_families.txt"))
    print(name, open(res["stats"]).read().replace("\n", " | ")[:400])


def main(names):
    defs = case_defs()
    tmp = tempfile.mkdtemp()
    try:
        for n in (names or sorted(defs)):
            make_case(n, defs[n], tmp)
    finally:
        shutil.rmtree(tmp)


if __name__ == "__main__":
    main(sys.argv[1:])
