#!/usr/bin/env python3
"""Time the REFERENCE's own consensus stages on a sample of a bench configuration (SURVEY.md
§8d(i)), beside the C++ oracle on the same BAM.  TEST INFRASTRUCTURE, this container only: the
reference does not travel to the GPU box, so bench.py's cpu_baseline uses the C++ oracle and
DESIGN.md §5 quotes this script's output next to it.

The reference runs unmodified through oracle/refrun.py (the pure-Python pysam stand-in injected,
randint -> first).  Its stage times therefore include that stand-in's pure-Python BGZF/BAM codec;
the line also reports how long the stand-in alone takes to iterate the input once, so the
dictionary work can be told apart from the I/O.

usage: time_reference.py [CONFIG] [PAIRS] [SEED]      (default c2 20000 1)
"""
import json
import os
import shutil
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), HERE]

import refrun  # noqa: E402
import cc_oracle_native as O  # noqa: E402
from cpu_baseline import sample  # noqa: E402
from consensuscruncher_amd import synth  # noqa: E402


def main():
    config = sys.argv[1] if len(sys.argv) > 1 else "c2"
    pairs = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
    seed = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    d = tempfile.mkdtemp(prefix="ccref_")
    try:
        batch, bed = sample(config, pairs, seed)
        bam = os.path.join(d, "sample.bam")
        synth.write_bam_native(batch, bam, level=1, nthreads=1)
        m = refrun.load_reference()
        # the stand-in's cost of reading the input once (pysam.AlignmentFile iteration)
        import pysam
        t = time.time()
        with pysam.AlignmentFile(bam, "rb") as f:
            n_iter = sum(1 for _ in f.fetch(until_eof=True))
        read_s = time.time() - t
        stage_s = {}
        real = refrun.run_main

        def timed(module, argv):
            t0 = time.time()
            out = real(module, argv)
            name = {m["sscs"]: "sscs", m["dcs"]: "dcs", m["sc"]: "sc"}[module]
            if name == "dcs" and "dcs" in stage_s:
                name = "dcs_sc"
            stage_s[name] = time.time() - t0
            return out

        refrun.run_main = timed
        try:
            t = time.time()
            refrun.consensus_pipeline(bam, os.path.join(d, "ref"), bedfile=bed or "False")
            ref_wall = time.time() - t
        finally:
            refrun.run_main = real
        times = {}
        t = time.time()
        O.consensus_pipeline(bam, os.path.join(d, "oracle"), bedfile=bed or "False", times=times)
        ora_wall = time.time() - t
        ref_stages = sum(stage_s.values())
        print(json.dumps(dict(
            config=config, pairs=pairs, input_reads=int(batch.n), cores=1,
            reference=dict(stages_s=stage_s, stages_total_s=round(ref_stages, 3), wall_s=round(ref_wall, 3),
                           reads_per_s=round(batch.n / ref_stages, 1),
                           shim_read_once_s=round(read_s, 3), shim_records=n_iter),
            cpp_oracle=dict(consensus_s=round(sum(times.values()), 4), wall_s=round(ora_wall, 3),
                            reads_per_s=round(batch.n / sum(times.values()), 1)))))
    finally:
        shutil.rmtree(d, ignore_errors=True)


if __name__ == "__main__":
    main()
