"""Multi-GPU sharding over bed regions.

A family, its duplex partner and its SC complement share coordinates, so they
all complete in one region.  Work is therefore split along the bed regions in
their iteration order: each rank owns a contiguous block of regions and
processes the stream positions of those regions exactly as the single-GPU
path does.  Concatenating the per-rank outputs in rank order gives the
reference's emission order (region-major).

The only cross-shard dependency is a read pair whose two ends lie in regions
owned by different ranks (translocations, pairs straddling a block edge). The
reference pairs by qname across regions (pair_dict persists,
consensus_helper.py:426-432): the pair completes at the later-streamed mate.
The host moves the first-streamed mate to the rank of the completing region
as a *foreign* stream entry.  It goes before that rank's own positions, carries
region ``-(r+1)``, pairs by coordinates and is counted there; the sender keeps
its entry marked ``CC_REGION_MOVED`` (never paired there; counted and listed
there only when it is a bad read of the SSCS pass, which lists them).  The mate's region comes from its (mtid, mpos)
fields, i.e. the aligner's mate coordinates.

Stats are summed over ranks (the one RCCL all-reduce of the multi-GPU driver).
"""
import numpy as np

from . import native as N
from .engine import Stream


def plan_blocks(region_counts, world):
    """Contiguous blocks of regions with near-equal read counts: list of (lo, hi)."""
    counts = np.asarray(region_counts, np.int64)
    n = len(counts)
    cum = np.concatenate([[0], np.cumsum(counts)])
    total = cum[-1]
    bounds = [0]
    for k in range(1, world):
        target = total * k / world
        b = int(np.searchsorted(cum, target, "left"))
        b = min(max(b, bounds[-1]), n)
        bounds.append(b)
    bounds.append(n)
    return [(bounds[i], bounds[i + 1]) for i in range(world)]


def overlap_safe_blocks(blocks, regions):
    """The block plan with every boundary moved forward past any pair of overlapping bed regions
    (same contig, [start, end) intersecting) that it would split.  A record in two overlapping
    regions is streamed by both (pysam's fetch per region, consensus_helper.py:377-396), and the
    reference then raises KeyError or pairs it twice depending on the order of the two regions'
    loops (consensus_helper.py:475-500): both regions must run in one rank, in bed order.  Blocks
    emptied by a moved boundary stay as empty (lo, lo) ranges.  Cytoband tables have no overlaps."""
    n = len(regions)
    if n == 0:
        return [tuple(b) for b in blocks]
    chrom = np.array([c for _, c, _, _ in regions])
    start = np.array([max(s, 0) for _, _, s, _ in regions], np.int64)
    end = np.array([e for _, _, _, e in regions], np.int64)
    # reach[i]: the last region (bed order) overlapping region i or an earlier one
    reach = np.arange(n)
    for i in range(n):
        ov = np.nonzero((chrom == chrom[i]) & (start < end[i]) & (start[i] < end) & (end > start))[0]
        if len(ov) and end[i] > start[i]:
            reach[i] = max(i, int(ov.max()))
    reach = np.maximum.accumulate(reach)
    out, lo = [], 0
    for k, (_, hi) in enumerate(blocks):
        hi = max(int(hi), lo)
        while 0 < hi < n and reach[hi - 1] >= hi:   # a cut at hi splits an overlapping pair
            hi += 1
        if k == len(blocks) - 1:
            hi = n
        out.append((lo, hi))
        lo = hi
    return out


def region_of_positions(regions, names, tid, pos):
    """Bed region index containing each (tid, pos) with start <= pos < end (the first such region in
    bed order), or -1.  Non-overlapping regions (cytoband tables): one binary search per position."""
    tid = np.asarray(tid, np.int64)
    pos = np.asarray(pos, np.int64)
    out = np.full(len(tid), -1, np.int64)
    iv = [(names[c], max(s, 0), e, r) for r, (_, c, s, e) in enumerate(regions) if c in names and e > max(s, 0)]
    if not iv or not len(tid):
        return out
    iv.sort()
    t = np.array([x[0] for x in iv], np.int64)
    lo = (t << 32) + np.array([x[1] for x in iv], np.int64)
    hi = (t << 32) + np.array([x[2] for x in iv], np.int64)
    if np.any(lo[1:] < hi[:-1]):   # overlapping regions: bed order decides, region by region
        for r, (_, chrom, start, end) in enumerate(regions):
            tt = names.get(chrom, -2)
            m = (tid == tt) & (pos >= start) & (pos < end) & (out < 0)
            out[m] = r
        return out
    key = np.where(tid < 0, np.int64(-1), (tid << 32) + pos)
    j = np.searchsorted(lo, key, "right") - 1
    ok = (j >= 0) & (tid >= 0)
    jj = np.maximum(j, 0)
    ok &= key < hi[jj]
    out[ok] = np.array([x[3] for x in iv], np.int64)[jj[ok]]
    return out


def shard_streams(records, refs, regions, global_stream, world, blocks=None):
    """Per-rank Streams for the regions plan.  global_stream is engine.bed_stream(...).  blocks: the
    sample's region plan (every stage of one sample must use the same one: a family, its duplex
    partner and its SC complement live in one region); default: balanced on this file's reads."""
    names = {name: i for i, (name, _) in enumerate(refs)}
    nreg = len(regions)
    if blocks is None:
        counts = np.bincount(global_stream.region, minlength=nreg)
        blocks = plan_blocks(counts, world)
    owner = np.zeros(nreg, np.int64)
    for k, (lo, hi) in enumerate(blocks):
        owner[lo:hi] = k
    rec = global_stream.rec
    reg = global_stream.region.astype(np.int64)
    mate_reg = region_of_positions(regions, names, records.mtid[rec], records.mpos[rec])
    # first-streamed end of a cross-shard pair: its mate's region comes later and is owned elsewhere
    send = (mate_reg >= 0) & (mate_reg > reg) & (owner[np.maximum(mate_reg, 0)] != owner[reg])
    out = []
    for k, (lo, hi) in enumerate(blocks):
        own = (reg >= lo) & (reg < hi)
        foreign = send & (owner[np.maximum(mate_reg, 0)] == k)
        srec = np.concatenate([rec[foreign], rec[own]]).astype(np.int32)
        # the own entries moved to their completing rank (cc_read_bam: CC_REGION_MOVED)
        oreg = np.where(send[own], reg[own] | N.REGION_MOVED, reg[own])
        sreg = np.concatenate([-(reg[foreign] + 1), oreg]).astype(np.int32)
        out.append(Stream(srec, sreg, global_stream.region_run, global_stream.region_keys))
    return out, blocks


def allreduce_stats(counters, elapsed_s, group=None):
    """The one collective of the multi-GPU path: sum the per-rank counters (stats.txt
    quantities, input reads, family-size histogram bins) and take the max of the per-rank step times.
    Over RCCL (backend "nccl") on GPUs, over gloo on CPU.  Returns (summed dict, max elapsed)."""
    import torch
    import torch.distributed as dist
    keys = sorted(counters)
    dev = torch.device("cuda", torch.cuda.current_device()) if (
        dist.get_backend(group) == "nccl") else torch.device("cpu")
    v = torch.tensor([float(counters[k]) for k in keys], dtype=torch.float64, device=dev)
    t = torch.tensor([float(elapsed_s)], dtype=torch.float64, device=dev)
    dist.all_reduce(v, op=dist.ReduceOp.SUM, group=group)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    vals = v.cpu().tolist()
    return {k: vals[i] for i, k in enumerate(keys)}, float(t.item())
