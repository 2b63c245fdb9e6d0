"""The multi-GPU path on CPU: two processes over gloo (world size 2), as the driver launches bench.py
with torch.distributed (one rank per GPU, RCCL there).  Checks
  * the shard plan (consensuscruncher_amd/shard.py): every bed region belongs to one
    rank, ranks own disjoint parts of the read_bam stream that together are the whole stream, and
    every read pair whose two ends fall to different ranks has its first-streamed end routed to
    the rank that completes it (the rank owning the later end), so pair_dict completes there;
  * allreduce_stats, the one collective: per-rank counters summed, step times max-reduced.
The GPU-side equality of sharded and single-pass outputs is tests/test_gpu_shard.py."""
import json
import os
import socket

import numpy as np
import pytest

from parity import GOLDEN

WORLD = 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _plan(case):
    from consensuscruncher_amd.consensus_helper import region_list
    from consensuscruncher_amd.engine import MODE_SSCS, Bam, Interner, bed_stream
    d = os.path.join(GOLDEN, case)
    bed = os.path.join(d, json.load(open(os.path.join(d, "params.json")))["run"]["bedfile"])
    bam = Bam(os.path.join(d, "input.bam"))
    rec = bam.decode(Interner(), MODE_SSCS, "|")
    return bam, rec, bed, region_list(bed), bed_stream(rec, bam.refs, bed)


def _worker(rank, port, case, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(WORLD))
    import torch.distributed as dist
    from consensuscruncher_amd.shard import allreduce_stats, shard_streams
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        bam, rec, bed, regions, st = _plan(case)
        streams, blocks = shard_streams(rec, bam.refs, regions, st, WORLD)
        mine = streams[rank]
        own = mine.rec[mine.region >= 0]
        foreign = mine.rec[mine.region < 0]
        sums, tmax = allreduce_stats({"own": len(own), "foreign": len(foreign), "rank": rank}, 1.5 + rank)
        parts = [None] * WORLD
        dist.all_gather_object(parts, (own.tolist(), foreign.tolist(), (-mine.region[mine.region < 0] - 1).tolist()))
        if rank == 0:
            json.dump(dict(sums=sums, tmax=tmax, parts=parts, blocks=blocks), open(os.path.join(out_dir, "r0.json"), "w"))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case,routed", [("bed_multi", False), ("hg19_bed", True)])
def test_two_rank_shard_plan_and_stats_reduction(case, routed, tmp_path):
    import torch.multiprocessing as mp
    port = _free_port()
    mp.start_processes(_worker, args=(port, case, str(tmp_path)), nprocs=WORLD, join=True, start_method="spawn")
    r = json.load(open(str(tmp_path / "r0.json")))
    bam, rec, bed, regions, st = _plan(case)
    owns = [np.array(p[0], np.int64) for p in r["parts"]]
    # the collective
    assert r["sums"]["own"] == st.n
    assert r["sums"]["foreign"] == sum(len(p[1]) for p in r["parts"])
    assert r["sums"]["rank"] == sum(range(WORLD))
    assert r["tmax"] == 1.5 + (WORLD - 1)
    # regions: contiguous blocks in bed order covering every region once
    blocks = [tuple(b) for b in r["blocks"]]
    assert blocks[0][0] == 0 and blocks[-1][1] == len(regions)
    assert all(blocks[k][1] == blocks[k + 1][0] for k in range(WORLD - 1))
    # ownership: a partition of the whole stream, in stream order within each rank
    allown = np.concatenate(owns)
    assert sorted(allown.tolist()) == sorted(st.rec.tolist())
    assert len(set(allown.tolist())) == len(allown)
    pos_in_stream = {int(x): i for i, x in enumerate(st.rec)}
    owner = {}
    for k, o in enumerate(owns):
        for x in o:
            owner[int(x)] = k
    # pairs: the later-streamed end's rank must hold the earlier end (own or routed in)
    by_name = {}
    for x in st.rec:
        by_name.setdefault(bam.qname(int(x)), []).append(int(x))
    held = [set(p[0]) | set(p[1]) for p in r["parts"]]
    cross = 0
    for name, xs in by_name.items():
        if len(xs) != 2:
            continue
        a, b = sorted(xs, key=lambda x: pos_in_stream[x])
        k = owner[b]
        if owner[a] != k:
            cross += 1
            assert a in held[k], "first mate of %s not routed to rank %d" % (name, k)
    # every routed record is a first-streamed end owned elsewhere
    for k, p in enumerate(r["parts"]):
        for x in p[1]:
            assert owner[int(x)] != k
    if routed:   # hg19_bed at two ranks has pairs (translocations) spanning the shards
        assert cross > 0, "no pair spans the two shards; the routing is untested"


def _part(rank):
    fams = {0: [(3, 5), (1, 2), (12, 1)], 1: [(1, 4), (7, 1), (3, 1), (40, 2)]}[rank]
    return dict(counters={"COUNTER": 10 + rank, "UNMAPPED_MATE": rank, "FAMILIES": 7 * (rank + 1)},
                sscs=3 + rank, singletons=2 * rank, never_emitted=0, families=fams, mapped=99)


def _reduce_worker(rank, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(WORLD))
    import torch.distributed as dist
    from consensuscruncher_amd.sharded import TorchComm
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        comm = TorchComm()
        got = comm.reduce_part(_part(rank))
        plan = comm.broadcast_obj([(0, 3), (3, 9)] if rank == 0 else None)
        if rank == 1:
            json.dump(dict(got=got, plan=plan), open(os.path.join(out_dir, "r1.json"), "w"))
    finally:
        dist.destroy_process_group()


def test_two_rank_stage_reduction_matches_combine(tmp_path):
    """The sharded pipeline's one collective (sharded.TorchComm.reduce_part: counters summed, the
    read_families Counter merged in first-seen order over the ranks' creation orders) equals the
    in-process combine_parts; the region plan broadcast reaches every rank."""
    import torch.multiprocessing as mp
    from consensuscruncher_amd.sharded import combine_parts
    mp.start_processes(_reduce_worker, args=(_free_port(), str(tmp_path)), nprocs=WORLD, join=True,
                       start_method="spawn")
    r = json.load(open(str(tmp_path / "r1.json")))
    exp = combine_parts([_part(0), _part(1)])
    assert r["got"]["counters"] == exp["counters"]
    for k in ("sscs", "singletons", "never_emitted", "mapped"):
        assert r["got"][k] == exp[k]
    assert [tuple(x) for x in r["got"]["families"]] == exp["families"] == [(3, 6), (1, 6), (12, 1), (7, 1), (40, 2)]
    assert [tuple(x) for x in r["plan"]] == [(0, 3), (3, 9)]


def test_concat_parts_in_rank_order(tmp_path):
    """Stage parts joined in rank order (engine.concat_bams): records in file order, first header."""
    import pysam
    from consensuscruncher_amd.engine import concat_bams
    src = os.path.join(GOLDEN, "basic", "expected")
    parts = [os.path.join(src, f) for f in ("sscs.bam", "singleton.bam", "dcs.bam")]
    out = str(tmp_path / "joined.bam")
    concat_bams(out, parts)
    assert pysam.sam_lines(out) == sum((pysam.sam_lines(p) for p in parts), [])


def _phase_worker(rank, port, out_dir):
    """TorchComm's exchange (all_to_all of record payloads) and its failure path: a raise on one rank
    inside a phase must raise on every rank instead of leaving the others in a collective."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(WORLD))
    import torch.distributed as dist
    from consensuscruncher_amd.sharded import RankFailed, TorchComm
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        comm = TorchComm()
        sends = {rank: [(np.arange(3 + d + 10 * rank, dtype=np.uint8), np.array([rank, d], np.int32))
                        for d in range(WORLD)]}
        got = comm.exchange(sends)[rank]
        res = {"got": [[a.tolist() for a in g] for g in got]}

        def boom(r):
            if r == 1:
                raise ZeroDivisionError("rank 1 fails (singleton_correction.py's empty-file ZeroDivisionError)")
            return r
        try:
            comm.each(boom)
            res["raised"] = None
        except RankFailed:
            res["raised"] = "RankFailed"
        except ZeroDivisionError:
            res["raised"] = "ZeroDivisionError"
        res["after"] = comm.each(lambda r: r * 10)[rank]   # the group is still usable
        json.dump(res, open(os.path.join(out_dir, "r%d.json" % rank), "w"))
    finally:
        dist.destroy_process_group()


def test_two_rank_exchange_and_failure_propagation(tmp_path):
    import torch.multiprocessing as mp
    mp.start_processes(_phase_worker, args=(_free_port(), str(tmp_path)), nprocs=WORLD, join=True,
                       start_method="spawn")
    r0 = json.load(open(str(tmp_path / "r0.json")))
    r1 = json.load(open(str(tmp_path / "r1.json")))
    for me, r in ((0, r0), (1, r1)):
        for src in range(WORLD):
            assert r["got"][src] == [list(range(3 + me + 10 * src)), [src, me]]
    assert r0["raised"] == "RankFailed" and r1["raised"] == "ZeroDivisionError"
    assert r0["after"] == 0 and r1["after"] == 10


def test_overlap_safe_blocks():
    """No block boundary splits two overlapping bed regions (same contig, intersecting [start, end));
    plans without overlaps are unchanged."""
    from consensuscruncher_amd.shard import overlap_safe_blocks
    regs = [("a", "chr1", 0, 100), ("b", "chr1", 100, 200), ("c", "chr2", 0, 50), ("d", "chr1", 150, 250),
            ("e", "chr2", 60, 70), ("f", "chr3", 0, 10)]
    # region d overlaps b: cuts at 2 and 3 would split (b, d)
    assert overlap_safe_blocks([(0, 2), (2, 4), (4, 6)], regs) == [(0, 4), (4, 4), (4, 6)]
    assert overlap_safe_blocks([(0, 1), (1, 3), (3, 6)], regs) == [(0, 1), (1, 4), (4, 6)]
    cyto = [("x%d" % i, "chr1", 100 * i, 100 * (i + 1)) for i in range(8)]
    assert overlap_safe_blocks([(0, 3), (3, 5), (5, 8)], cyto) == [(0, 3), (3, 5), (5, 8)]
    # the last block always ends at the last region
    assert overlap_safe_blocks([(0, 1), (1, 2)], [("p", "chr1", 0, 130000), ("q", "chr1", 100000, 300000)]) == \
        [(0, 2), (2, 2)]
