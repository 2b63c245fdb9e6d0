#!/usr/bin/env python3
"""Per-launch HBM traffic of the profiled kernels from the rocprofv3 PMC passes of gpurun_prof.sh.

FETCH_SIZE and WRITE_SIZE come from separate passes (they do not fit one TCC pass on gfx950) and
are reported in KiB (converted to bytes here).  MI355X_MICROARCH.md (HBM section): on gfx950 FETCH_SIZE counts exactly half
the bytes of a wide coalesced streaming read (16 B per lane), so it is doubled here; WRITE_SIZE is
exact for 16-B-per-lane stores.  The vote kernels read 16 B + 8 B per lane and member and write
16 B + 8 B per lane, so the 8-B parts are uncalibrated (see the guide).

usage: pmc_traffic.py FETCH_CSV WRITE_CSV OUT_JSON [PASSES [BENCH_JSON]] [--sized SIZED_CSV]

SIZED_CSV: a third pass over TCC_EA0_RDREQ_32B_sum, TCC_EA0_RDREQ_64B_sum and TCC_EA0_RDREQ_128B_sum
(3 TCC counters, one pass).  Those count the memory-side read requests by size, so their byte sum
is the read traffic whatever the access width (FETCH_SIZE's gfx950 formula tallies the 128-B requests
at 64 B, which the x2 above undoes only for pure 16-B streams: a gather kernel's 32/64-B requests
would be doubled too).  When given, fetch_bytes_per_launch is the size-resolved figure and the x2
figure stays beside it (fetch_x2_bytes_per_launch).  scripts/calib/pmc_calib.hip checks both
against known byte counts (profiles/r04_pmc_calib.json).

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


SIZES = {"TCC_EA0_RDREQ_32B_sum": 32.0, "TCC_EA0_RDREQ_64B_sum": 64.0, "TCC_EA0_RDREQ_128B_sum": 128.0,
         "TCC_EA0_RDREQ_32B": 32.0, "TCC_EA0_RDREQ_64B": 64.0, "TCC_EA0_RDREQ_128B": 128.0}


def sized_reads(path):
    """Per kernel, per dispatch: read bytes from the size-resolved request counts."""
    per = {}
    for r in csv.DictReader(open(path)):
        sz = SIZES.get(r["Counter_Name"])
        if sz is None:
            continue
        k = r["Kernel_Name"].split("(")[0]
        d = per.setdefault(k, {})
        d[r["Dispatch_Id"]] = d.get(r["Dispatch_Id"], 0.0) + sz * float(r["Counter_Value"])
    return {k: [v[i] for i in sorted(v, key=int)] for k, v in per.items()}


def main():
    argv = list(sys.argv)
    sized = None
    if "--sized" in argv:
        i = argv.index("--sized")
        sized = sized_reads(argv[i + 1])
        del argv[i:i + 2]
    fetch = per_kernel(argv[1], "FETCH_SIZE")
    write = per_kernel(argv[2], "WRITE_SIZE")
    res = {}
    for k in sorted(set(fetch) | set(write) | set(sized or ())):
        f = fetch.get(k, [0.0])
        w = write.get(k, [0.0])
        fb = 2.0 * sum(f) / len(f)
        wb = sum(w) / len(w)
        row = dict(fetch_bytes_per_launch=fb, write_bytes_per_launch=wb, traffic_bytes_per_launch=fb + wb,
                   launches=len(f), raw_fetch_bytes=f, raw_write_bytes=w,
                   note="FETCH_SIZE x2 (gfx950 half-count on 16-B streaming reads), WRITE_SIZE as reported")
        if sized is not None:
            s_ = sized.get(k, [0.0])
            sb = sum(s_) / len(s_)
            row.update(fetch_x2_bytes_per_launch=fb, fetch_bytes_per_launch=sb, traffic_bytes_per_launch=sb + wb,
                       raw_sized_read_bytes=s_,
                       note="reads: TCC_EA0_RDREQ_32B/64B/128B x their sizes; WRITE_SIZE as reported; "
                            "fetch_x2: FETCH_SIZE x2")
        res[k] = row
    if len(argv) > 4:
        res["_meta"] = dict(passes=int(argv[4]), reads="sized requests" if sized is not None else "FETCH_SIZE x2")
    if len(argv) > 5:
        b = json.loads(open(argv[5]).read().strip().splitlines()[-1])
        res["_meta"].update(workload=b["config"]["workload"], input_reads=b["config"]["input_reads_per_rank"])
    json.dump(res, open(argv[3], "w"), indent=1)
    print(json.dumps({k: round(v["traffic_bytes_per_launch"] / 1e9, 4) for k, v in res.items() if k != "_meta"}))


if __name__ == "__main__":
    main()
