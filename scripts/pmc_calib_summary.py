#!/usr/bin/env python3
"""Summary of the counter calibration (scripts/calib/pmc_calib.hip under three rocprofv3 --pmc passes:
FETCH_SIZE, WRITE_SIZE, and TCC_EA0_RDREQ_32B/64B/128B) against the kernels' known byte counts.

usage: pmc_calib_summary.py FETCH_CSV WRITE_CSV SIZED_CSV OUT_JSON"""
import csv
import json
import sys

KNOWN = {"k_rd16": 2 ** 30, "k_rd8": 2 ** 30, "k_rd4": 2 ** 30, "k_gat16": 2 ** 24 * 16, "k_gat4": 2 ** 24 * 4,
         "k_wr16": 2 ** 30, "k_wr4": 2 ** 30}
ORDER = ["k_rd16", "k_rd8", "k_rd4", "k_gat16", "k_gat4", "k_wr16", "k_wr4"]
SIZE = {"TCC_EA0_RDREQ_32B_sum": 32, "TCC_EA0_RDREQ_64B_sum": 64, "TCC_EA0_RDREQ_128B_sum": 128}


def dispatches(path):
    d = {}
    for r in csv.DictReader(open(path)):
        if not r["Kernel_Name"].startswith("void k_"):
            continue
        d.setdefault(int(r["Dispatch_Id"]), {})[r["Counter_Name"]] = float(r["Counter_Value"])
    return [d[k] for k in sorted(d)][-len(ORDER):]   # the second round (warm code)


def main():
    f, w, s = (dispatches(p) for p in sys.argv[1:4])
    out = {}
    for i, k in enumerate(ORDER):
        sized = sum(SIZE[c] * v for c, v in s[i].items() if c in SIZE)
        out[k] = dict(known_bytes=KNOWN[k], fetch_x2_over_known=round(2048 * f[i]["FETCH_SIZE"] / KNOWN[k], 4),
                      sized_reads_over_known=round(sized / KNOWN[k], 4),
                      write_over_known=round(1024 * w[i]["WRITE_SIZE"] / KNOWN[k], 4),
                      requests={c: int(v) for c, v in s[i].items()})
    out["_note"] = ("1 GiB buffer (4x the Infinity Cache), 2^24 random gathers; every read request on gfx950 is "
                    "a 128-B request (FETCH_SIZE tallies it at 64 B: x2 is exact for 4/8/16-B lanes alike); a "
                    "random 4-B or 16-B gather costs a whole 128-B line; WRITE_SIZE is exact for 4- and 16-B "
                    "stores")
    json.dump(out, open(sys.argv[4], "w"), indent=1)
    print(json.dumps({k: (v["fetch_x2_over_known"], v["sized_reads_over_known"], v["write_over_known"])
                      for k, v in out.items() if not k.startswith("_")}))


if __name__ == "__main__":
    main()
