"""Search for the input the engine fences with CC_E_AMBIGUOUS: one consensus tag (csn_pair_dict key)
created in two bed regions by different pairs (consensus_helper.py:455-489 with the SSCS region loop,
SSCS_maker.py:265-339, which emits and deletes the first region's entry).

TEST INFRASTRUCTURE ONLY (CPU, the pinned Python oracle).  Small seeded samples with overlapping random
bed regions on one contig, qnames seen three and four times (synth dupq_frac) and shared consensus
tags (synth quirk_frac); for each, the SSCS stage of oracle/cc_oracle.py runs with its FamilyBuilder
instrumented to record, per consensus tag, the regions in which families were added to its entry.

usage: python oracle/fuzz_csn_regions.py FIRST_SEED LAST_SEED
prints one line per hit and a summary: seeds run, seeds where the reference raises KeyError, hits.
"""
import collections
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), HERE, os.path.join(HERE, "shim")]

import numpy as np  # noqa: E402

import cc_oracle  # noqa: E402
import synthbam  # noqa: E402
from consensuscruncher_amd import synth  # noqa: E402

_feed = cc_oracle.FamilyBuilder.feed


def run(seed, tmp):
    rng = np.random.default_rng(seed)
    gen = dict(n_pairs=int(rng.integers(60, 300)), seed=seed, contigs=(("chr1", 20000),),
               dupq_frac=float(rng.choice([0, 0.1, 0.3])), quirk_frac=float(rng.choice([0, 0.1, 0.3])))
    bam = os.path.join(tmp, "in%d.bam" % seed)
    synthbam.write_batch(synth.generate(**gen), bam)
    bed = os.path.join(tmp, "r%d.bed" % seed)
    with open(bed, "w") as f:
        for k in range(int(rng.integers(2, 5))):
            s = int(rng.integers(0, 18000))
            f.write("chr1\t%d\t%d\tr%d\tgneg\n" % (s, s + int(rng.integers(500, 8000)), k))
    state = {"region": -1}
    created = collections.defaultdict(set)

    def feed(self, records, region=None, **kw):
        state["region"] += 1
        before = {k: len(v) for k, v in self.entries.items()}
        out = _feed(self, records, region, **kw)
        for k, v in self.entries.items():
            if len(v) > before.get(k, 0):
                created[k].add(state["region"])
        return out
    cc_oracle.FamilyBuilder.feed = feed
    try:
        cc_oracle.sscs_stage(bam, os.path.join(tmp, "o%d.sscs.bam" % seed), 0.7, bed)
        raised = False
    except cc_oracle.OracleError:
        raised = True
    finally:
        cc_oracle.FamilyBuilder.feed = _feed
    return {k: v for k, v in created.items() if len(v) > 1}, raised


def main(a, b):
    n = raised = hits = 0
    with tempfile.TemporaryDirectory() as tmp:
        for seed in range(a, b):
            multi, r = run(seed, tmp)
            n += 1
            raised += r
            if multi:
                hits += 1
                print("hit seed %d (reference raises: %s): %s" % (seed, r, list(multi.items())[:2]), flush=True)
    print("seeds %d, reference raised KeyError %d, consensus tags created in two regions %d" % (n, raised, hits))


if __name__ == "__main__":
    main(int(sys.argv[1]), int(sys.argv[2]))
