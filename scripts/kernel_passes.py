#!/usr/bin/env python3
"""Per-pass kernel breakdown of one bench step from a rocprofv3 kernel trace (--kernel-trace,
csv).  The last step's dispatches are split into the stage calls of the chain (each read_bam pass
starts with its k_fill + k_build_meta; the SSCS / DCS / SC stage calls follow their passes) and the
time of every kernel is summed per pass.

usage: kernel_passes.py KERNEL_TRACE_CSV [PASSES_PER_STEP=9] [OUT_JSON]
"""
import collections
import csv
import glob
import json
import sys


def load(path):
    rows = []
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0].split("<")[0].strip()
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    rows.sort()
    return rows


def main():
    path = sys.argv[1]
    if "*" in path:
        path = sorted(glob.glob(path, recursive=True))[-1]
    rows = load(path)
    # read_bam passes begin at k_build_meta; the bench step is 5 passes (SSCS, DCS, SC x2, DCS+SC)
    starts = [i for i, r in enumerate(rows) if r[2] == "k_build_meta"]
    per_step = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    last = starts[-per_step:]
    # SC joins the DCS grouping without a bed file (one read_bam pass for its singletons only)
    names = ["sscs", "dcs", "sc_singletons", "sc_sscs", "dcs_sc"] if per_step == 5 else ["sscs", "dcs", "sc", "dcs_sc"]
    out = collections.OrderedDict()
    for k, b in enumerate(last):
        e = last[k + 1] if k + 1 < len(last) else len(rows)
        acc = collections.OrderedDict()
        for s, t, n in rows[b - 1 if b > 0 and rows[b - 1][2] == "k_fill" else b:e]:
            acc[n] = acc.get(n, 0.0) + (t - s) / 1000.0
        out[names[k] if k < len(names) else "pass%d" % k] = dict(total_us=round(sum(acc.values()), 1),
                                                                 kernels={n: round(v, 1) for n, v in acc.items()})
    for p, d in out.items():
        print("%-14s %8.1f us" % (p, d["total_us"]))
        for n, v in sorted(d["kernels"].items(), key=lambda kv: -kv[1])[:14]:
            print("    %-28s %8.1f" % (n, v))
    if len(sys.argv) > 3:
        json.dump(out, open(sys.argv[3], "w"), indent=1)


if __name__ == "__main__":
    main()
