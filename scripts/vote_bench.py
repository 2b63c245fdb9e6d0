#!/usr/bin/env python3
"""Kernel-level timing of the SSCS stage (read_bam + consensus_maker) on one synthetic BAM, for
tuning variants of libccamd (CCAMD_LIB=<variant .so>).  Prints one JSON line: per-kernel mean
milliseconds per launch over --steps re-runs of the resident stage.

  python scripts/vote_bench.py --bam /tmp/c2.bam --pairs 3000000      # writes the BAM if missing
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bam", required=True)
    ap.add_argument("--pairs", type=int, default=3_000_000)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--cutoff", type=float, default=0.7)
    args = ap.parse_args()
    from consensuscruncher_amd import synth
    from consensuscruncher_amd.engine import Engine
    from consensuscruncher_amd.stages import SSCSRun
    if not os.path.exists(args.bam):
        cfg = dict(synth.CONFIGS["c2"])
        cfg["n_pairs"] = args.pairs
        t = time.time()
        batch = synth.generate(seed=synth.SEED_BASE + 2, **cfg)
        synth.write_bam_native(batch, args.bam, level=1)
        print("wrote %s (%d reads) in %.1fs" % (args.bam, batch.n, time.time() - t), file=sys.stderr, flush=True)
    eng = Engine(0)
    run = SSCSRun(eng, args.bam, args.cutoff)
    run.step(1)
    eng.synchronize()
    eng.set_profiling(True)
    t = time.perf_counter()
    for i in range(args.steps):
        run.step(100 + i)
    eng.synchronize()
    el = time.perf_counter() - t
    kt = eng.kernel_times()
    eng.set_profiling(False)
    out = dict(lib=os.environ.get("CCAMD_LIB", "default"), reads=run.n_input, ms_per_step=1000 * el / args.steps,
               kernels={k: round(v[0] / max(v[1], 1), 4) for k, v in sorted(kt.items(), key=lambda kv: -kv[1][0])})
    print(json.dumps(out), flush=True)
    run.close()
    eng.close()


if __name__ == "__main__":
    main()
