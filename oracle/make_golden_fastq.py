#!/usr/bin/env python3
"""Golden fixtures for fastq2bam's UMI extraction, made by running the
REFERENCE's extract_barcodes.py unmodified (oracle/refrun.run_extract, Biopython stand-in) on
read pairs from the reference's bundled test FASTQs (test/fastq/LargeMid_56_L005_R{1,2}.fastq,
data files).  TEST INFRASTRUCTURE, this container only.

tests/golden_fastq/
  inputs/R1.fastq.gz, R2.fastq.gz     the first PAIRS pairs of LargeMid_56 (gzip to keep them small)
  <case>/params.json                  argv (INPUT/OUTFILE/BLIST placeholders), input variant
  <case>/expected/*                   the reference's outputs (FASTQs gzipped), error.txt on a raise
"""
import gzip
import json
import os
import shutil
import sys
import tempfile
import traceback

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), HERE]
import refrun  # noqa: E402

SRC = "/root/reference/test/fastq/LargeMid_56_L005_R%d.fastq"
OUT = os.path.join(os.path.dirname(HERE), "tests", "golden_fastq")
PAIRS = 1000
BLIST = ["TGT", "CCT", "TCT", "CGT", "TGTT", "ACGT", "CCT", "GGAT", "TT"]

CASES = {
    "nnt": dict(argv=["--bpattern", "NNT"]),
    "spacer_mix": dict(argv=["--bpattern", "NCNT"]),
    "list_skip": dict(argv=["--blist", "BLIST", "--skipcheck"]),
    "list_nocheck": dict(argv=["--blist", "BLIST"]),
    "pattern_and_list": dict(argv=["--bpattern", "NNT", "--blist", "BLIST"]),
    "id_mismatch": dict(argv=["--bpattern", "NNT"], mutate_r2_id_at=300),
    "gz": dict(argv=["--bpattern", "NNT"], gz=True),
    # reads shorter than the longest list barcode (adapter-trimmed): read.seq[:blen] as it comes
    "list_short": dict(argv=["--blist", "BLIST", "--skipcheck"],
                       truncate={"5": [2, 126], "17": [126, 3], "40": [3, 4], "41": [1, 1], "77": [4, 2]}),
}


def variant_inputs(d, case, work):
    """The case's input pair in `work` (shared by this generator and tests/test_extract_barcodes.py)."""
    p = CASES[case] if isinstance(case, str) else case
    r = []
    for k in (1, 2):
        lines = gzip.open(os.path.join(d, "inputs", "R%d.fastq.gz" % k), "rt").read().split("\n")
        if k == 2 and p.get("mutate_r2_id_at"):
            i = 4 * (p["mutate_r2_id_at"] - 1)
            lines[i] = lines[i].replace(":", ";", 1)
        for pair, lens in sorted((p.get("truncate") or {}).items()):
            i = 4 * int(pair)
            lines[i + 1] = lines[i + 1][:lens[k - 1]]
            lines[i + 3] = lines[i + 3][:lens[k - 1]]
        text = "\n".join(lines)
        if p.get("gz"):
            path = os.path.join(work, "sample_R%d.fastq.gz" % k)
            with gzip.open(path, "wt") as f:
                f.write(text)
        else:
            path = os.path.join(work, "sample_R%d.fastq" % k)
            with open(path, "w") as f:
                f.write(text)
        r.append(path)
    return r


def argv_for(p, r1, r2, outfile, blist_path):
    argv = ["--read1", r1, "--read2", r2, "--outfile", outfile]
    return argv + [blist_path if a == "BLIST" else a for a in p["argv"]]


OUTPUTS = ("_barcode_R1.fastq", "_barcode_R2.fastq", "_r1_bad_barcodes.txt", "_r2_bad_barcodes.txt")


def main():
    os.makedirs(os.path.join(OUT, "inputs"), exist_ok=True)
    for k in (1, 2) if not sys.argv[1:] else ():
        with open(SRC % k) as f:
            lines = [next(f) for _ in range(4 * PAIRS)]
        with gzip.open(os.path.join(OUT, "inputs", "R%d.fastq.gz" % k), "wt", compresslevel=9) as g:
            g.write("".join(lines))
    if not sys.argv[1:]:
        with open(os.path.join(OUT, "inputs", "blist.txt"), "w") as f:
            f.write("\n".join(BLIST) + "\n")
    only = sys.argv[1:]   # case names: regenerate those only
    for case, p in CASES.items():
        if only and case not in only:
            continue
        work = tempfile.mkdtemp(prefix="ccfq_")
        try:
            r1, r2 = variant_inputs(OUT, case, work)
            os.makedirs(os.path.join(work, "fastq_tag"))
            outfile = os.path.join(work, "fastq_tag", "sample")
            err = None
            try:
                refrun.run_extract(argv_for(p, r1, r2, outfile, os.path.join(OUT, "inputs", "blist.txt")))
            except BaseException as e:   # noqa: B902 - the reference's raise is the expected outcome
                err = "%s: %s\n%s" % (type(e).__name__, e, traceback.format_exc())
            cd = os.path.join(OUT, case)
            shutil.rmtree(cd, ignore_errors=True)
            os.makedirs(os.path.join(cd, "expected"))
            json.dump(p, open(os.path.join(cd, "params.json"), "w"), indent=1)
            for suf in OUTPUTS:
                src = outfile + suf
                if os.path.exists(src):
                    with open(src, "rb") as f, gzip.open(os.path.join(cd, "expected", suf[1:] + ".gz"), "wb") as g:
                        g.write(f.read())
            st = os.path.join(work, "fastq_tag_barcode_stats.txt")
            if os.path.exists(st):
                shutil.copy(st, os.path.join(cd, "expected", "barcode_stats.txt"))
            if err:
                open(os.path.join(cd, "expected", "error.txt"), "w").write(err)
            print(case, "error" if err else "ok", sorted(os.listdir(os.path.join(cd, "expected"))))
        finally:
            shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    main()
