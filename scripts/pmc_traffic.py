#!/usr/bin/env python3
"""Per-launch HBM traffic of the profiled kernels from the rocprofv3 PMC passes of gpurun_prof.sh.

FETCH_SIZE and WRITE_SIZE come from separate passes (they do not fit one TCC pass on gfx950) and
are reported in KiB (converted to bytes here).  MI355X_MICROARCH.md (HBM section): on gfx950 FETCH_SIZE counts exactly half
the bytes of a wide coalesced streaming read (16 B per lane), so it is doubled here; WRITE_SIZE is
exact for 16-B-per-lane stores.  The vote kernels read 16 B + 8 B per lane and member and write
16 B + 8 B per lane, so the 8-B parts are uncalibrated (see the guide).

usage: pmc_traffic.py FETCH_CSV WRITE_CSV OUT_JSON [PASSES [BENCH_JSON]]

PASSES: pipeline passes the profiled bench run made (setup + warmup + profiling + timed steps);
stored as _meta.passes so that bench.py can turn launches into launches per step.  BENCH_JSON: the
profiled run's own output line; its workload and input reads are stored so that bench.py only
quotes the traffic for the same workload.
"""
import csv
import json
import sys


def per_kernel(path, counter):
    out = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        out.setdefault(r["Kernel_Name"].split("(")[0], []).append(float(r["Counter_Value"]) * 1024.0)
    return out


def main():
    fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
    write = per_kernel(sys.argv[2], "WRITE_SIZE")
    res = {}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, [0.0])
        w = write.get(k, [0.0])
        fb = 2.0 * sum(f) / len(f)
        wb = sum(w) / len(w)
        res[k] = dict(fetch_bytes_per_launch=fb, write_bytes_per_launch=wb, traffic_bytes_per_launch=fb + wb,
                      launches=len(f), raw_fetch_bytes=f, raw_write_bytes=w,
                      note="FETCH_SIZE x2 (gfx950 half-count on 16-B streaming reads), WRITE_SIZE as reported")
    if len(sys.argv) > 4:
        res["_meta"] = dict(passes=int(sys.argv[4]))
    if len(sys.argv) > 5:
        b = json.loads(open(sys.argv[5]).read().strip().splitlines()[-1])
        res["_meta"].update(workload=b["config"]["workload"], input_reads=b["config"]["input_reads_per_rank"])
    json.dump(res, open(sys.argv[3], "w"), indent=1)
    print(json.dumps({k: round(v["traffic_bytes_per_launch"] / 1e9, 4) for k, v in res.items() if k != "_meta"}))


if __name__ == "__main__":
    main()
