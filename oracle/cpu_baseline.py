#!/usr/bin/env python3
"""CPU baseline worker (TEST INFRASTRUCTURE, bench.py's cpu_baseline leg): one sample of a bench
configuration through the C++ oracle's consensus pipeline (oracle/cc_oracle.cpp, the reference's
dictionary program in C++, pinned to the reference by tests/test_oracle_native.py) on one core.

Prints one JSON line: input reads, the consensus-only seconds (the four stages from decoded records
to output records; BAM decode/encode and the samtools stand-in excluded, as the GPU figure
excludes them) and the wall seconds of the whole pipeline.

usage: cpu_baseline.py CONFIG PAIRS SEED
"""
import json
import os
import shutil
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), HERE]

import cc_oracle_native as O  # noqa: E402
from consensuscruncher_amd import synth  # noqa: E402


def sample(config, pairs, seed):
    """A bounded sample of the configuration with its read density (c2: the contig scaled with the
    pair count; c3: rank 0's share of the cytoband blocks at the per-GPU density)."""
    cfg, bed = synth.config(config)
    full = cfg["n_pairs"]
    cfg["n_pairs"] = pairs
    if bed is None:
        name, ln = cfg["contigs"][0]
        cfg["contigs"] = ((name, max(100_000, int(ln * pairs / full))),)
    else:
        # the first cytoband regions up to the sample's share of the genome
        keep, acc, total = [], 0, sum(e - s for _, s, e in cfg["windows"])
        for w in cfg["windows"]:
            keep.append(w)
            acc += w[2] - w[1]
            if acc >= total * pairs / full:
                break
        cfg["windows"] = keep
    return synth.generate(seed=seed, **cfg), bed


def main():
    config, pairs, seed = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    d = tempfile.mkdtemp(prefix="cccpu_")
    try:
        batch, bed = sample(config, pairs, seed)
        bam = os.path.join(d, "sample.bam")
        synth.write_bam_native(batch, bam, level=1, nthreads=1)
        times = {}
        t = time.time()
        O.consensus_pipeline(bam, d, bedfile=bed or "False", times=times)
        print(json.dumps(dict(reads=int(batch.n), consensus_s=sum(times.values()), wall_s=time.time() - t,
                              stages=times)))
    finally:
        shutil.rmtree(d, ignore_errors=True)


if __name__ == "__main__":
    main()
