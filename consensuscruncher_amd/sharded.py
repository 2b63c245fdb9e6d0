"""One sample's consensus pipeline over several GPUs, split along the bed regions.

The reference processes its bed regions one after another (SSCS_maker.py:265-281,
DCS_maker.py:204-218, singleton_correction.py:203-229; consensus_helper.py:38-54), with pair_dict
persisting across regions.  A family, its duplex partner and its singleton-correction complement
share their coordinates, so they complete in one region; the regions therefore split into
contiguous blocks, one per rank, and every stage of the sample uses the same block plan.

Each rank holds only the records at its block's positions (its device tables are about 1/N of
the sample):
  * the input BAM is read through its BAI, only the block's regions (ccio_bam_open_regions);
  * a pair whose two ends fall to different ranks completes at its later-streamed end: the rank
    holding the first-streamed end moves that record (raw BAM bytes) to the completing rank, where
    it enters the stream as a foreign entry (region -(r+1)) before the rank's own entries and pairs
    by coordinates like the rest; the sender keeps its entry marked CC_REGION_MOVED (not paired
    there, counted once over the ranks, listed as a bad read only by the sender: cc_read_bam);
  * every stage output record goes to the rank owning its position (a consensus of a foreign end
    sits in another block), and each rank stably sorts what it receives in sender order: exactly
    its part of the whole-sample sorted file the next stage of the reference reads (the samtools
    stand-in's stable sort of the rank-order concatenation), without that file on the critical
    path.  The next stage runs on these rank-local inputs.
The exchanges are host-side and small (cross-block pairs only).  The stats.txt / read_families.txt
quantities are reduced once per stage (the path's one collective: over RCCL through
cc_reduce_stats on GPUs, gloo on CPU), rank 0 writes the side outputs, and at the end rank 0
merges the ranks' sorted parts into the reference's output files (ties in rank order, which is
the whole-sample sort's order).

Two drivers run the same code: LocalComm runs the ranks one after another in this process on one
GPU (tests: the outputs equal the single-pass pipeline's byte for byte); TorchComm is one process
per GPU under torch.distributed.
"""
import os
import shutil
import time

import numpy as np

from .consensus_helper import region_list, region_runs
from .engine import MODE_DUPLEX, MODE_SSCS, Bam, Interner, Stream, bed_stream, concat_bams, index_bam, merge_bams
from . import native as N
from .shard import overlap_safe_blocks, plan_blocks, region_of_positions
from .stages import DCSRun, SCRun, SSCSRun, dcs_side, sc_side, sscs_side

COUNTER_KEYS = ("COUNTER", "UNMAPPED", "UNMAPPED_MATE", "MULTIPLE_MAPPING", "BAD_SPACER", "PAIRS", "READ_ENDS",
                "FAMILIES", "ENTRIES", "UNPAIRED", "ORPHAN_TAGS", "DROPPED", "BAD_LISTED", "FOREIGN")
SCALARS = ("sscs", "singletons", "never_emitted", "dcs", "sscs_singletons", "processed", "sscs_correction",
           "singleton_correction", "uncorrected", "mapped_own")


def combine_parts(parts):
    """The reduction of the per-rank stage parts (rank order): counters and stage counts summed;
    read_families' Counter (SSCS_maker.py:401-408) merged in first-seen order over the ranks'
    creation orders, i.e. ordered by (first rank holding the size, its place in that rank's table)."""
    out = {"counters": {k: sum(p["counters"].get(k, 0) for p in parts) for k in parts[0]["counters"]}}
    for k in SCALARS:
        if k in parts[0]:
            out[k] = sum(p[k] for p in parts)
    if "families" in parts[0]:
        order, cnt = [], {}
        for p in parts:
            for size, n in p["families"]:
                if size not in cnt:
                    order.append(size)
                    cnt[size] = 0
                cnt[size] += n
        out["families"] = [(s, cnt[s]) for s in order]
    if "mapped" in parts[0]:
        out["mapped"] = parts[0]["mapped"]
    return out


class LocalComm(object):
    """world ranks run one after another in this process (one GPU)."""

    def __init__(self, world):
        self.world = world
        self.rank = 0
        self.ranks = list(range(world))

    def each(self, fn):
        return {r: fn(r) for r in self.ranks}

    def exchange(self, sends):
        """sends[r][d]: what rank r sends rank d -> received[d][s] from every rank s."""
        return {d: [sends[s][d] for s in range(self.world)] for d in self.ranks}

    def reduce(self, parts):
        return combine_parts([parts[r] for r in range(self.world)])

    def broadcast_obj(self, obj):
        return obj

    def barrier(self):
        pass

    def close(self):
        pass


_DT = {0: np.dtype(np.uint8), 1: np.dtype(np.int32), 2: np.dtype(np.int64)}


def _encode(arrays):
    """A tuple of uint8 / int32 / int64 arrays as bytes: count, then (dtype code, length, data) each."""
    code = {v: k for k, v in _DT.items()}
    parts = [np.array([len(arrays)], np.int64)]
    for a in arrays:
        a = np.ascontiguousarray(a)
        parts.append(np.array([code[a.dtype], a.nbytes], np.int64))
        parts.append(a)
    return np.concatenate([x.view(np.uint8) for x in parts])


def _decode(buf):
    n = int(buf[:8].view(np.int64)[0])
    out, o = [], 8
    for _ in range(n):
        c, nb = buf[o:o + 16].view(np.int64)
        o += 16
        out.append(buf[o:o + int(nb)].copy().view(_DT[int(c)]))
        o += int(nb)
    return tuple(out)


class RankFailed(RuntimeError):
    """Another rank raised inside a phase of the sharded pipeline."""


class TorchComm(object):
    """One process per GPU under torch.distributed (RCCL as backend "nccl" on ROCm, gloo on CPU).
    Every phase ends in a MAX-reduce of a failure flag, so an exception on one rank stops every rank
    instead of leaving the others blocked in a collective.  With an engine on a "nccl" group the
    stats reduction is cc_reduce_stats over the engine's own RCCL communicator."""

    def __init__(self, group=None, engine=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.ranks = [self.rank]
        self.engine = engine
        self.cc_comm = None
        if engine is not None and dist.get_backend(group) == "nccl":
            from .engine import comm_unique_id
            uid = self.broadcast_obj(comm_unique_id() if self.rank == 0 else None)
            self.cc_comm = engine.comm_init(self.world, self.rank, uid)

    def close(self):
        if self.cc_comm is not None:
            N.amd().cc_comm_destroy(self.cc_comm)
            self.cc_comm = None

    def _device(self):
        import torch
        if self.dist.get_backend(self.group) == "nccl":
            return torch.device("cuda", torch.cuda.current_device())
        return torch.device("cpu")

    def _any(self, flag):
        import torch
        t = torch.tensor([1 if flag else 0], dtype=torch.int64, device=self._device())
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX, group=self.group)
        return bool(t.item())

    def each(self, fn):
        err = None
        try:
            res = fn(self.rank)
        except BaseException as e:   # noqa: B902 -- re-raised below, after the other ranks learn of it
            err = e
        if self._any(err is not None):
            if err is not None:
                raise err
            raise RankFailed("another rank failed in this phase of the sharded pipeline")
        return {self.rank: res}

    def exchange(self, sends):
        """all_to_all of each rank's payloads (tuples of numpy arrays) over the process group."""
        import torch
        dev = self._device()
        blobs = [_encode(x) for x in sends[self.rank]]
        n_out = torch.tensor([len(b) for b in blobs], dtype=torch.int64, device=dev)
        n_in = torch.zeros(self.world, dtype=torch.int64, device=dev)
        self.dist.all_to_all_single(n_in, n_out, group=self.group)
        out = torch.from_numpy(np.concatenate(blobs)).to(dev)
        inp = torch.zeros(int(n_in.sum().item()), dtype=torch.uint8, device=dev)
        self.dist.all_to_all_single(inp, out, output_split_sizes=n_in.tolist(), input_split_sizes=n_out.tolist(),
                                    group=self.group)
        buf = inp.cpu().numpy()
        got, o = [], 0
        for k in n_in.tolist():
            got.append(_decode(buf[o:o + k]))
            o += k
        return {self.rank: got}

    def reduce(self, parts):
        return self.reduce_part(parts[self.rank])

    def reduce_part(self, part):
        """combine_parts over the ranks with collectives: one SUM of the counter/count vector, and for
        the family table a MAX of its length, a SUM of the per-size counts and a MIN of each size's
        first-seen key (rank << 40 | place)."""
        ckeys = sorted(part["counters"])
        skeys = [k for k in SCALARS if k in part]
        vec = np.array([part["counters"][k] for k in ckeys] + [part[k] for k in skeys], np.int64)
        fam = part.get("families")
        top = np.array([max([s for s, _ in fam], default=0) if fam is not None else 0], np.int64)
        self._allreduce(top, "max")
        n = int(top[0]) + 1 if fam is not None else 0
        cnt = np.zeros(n, np.int64)
        first = np.full(n, 1 << 62, np.int64)
        if fam:
            sizes = np.array([s for s, _ in fam], np.int64)
            cnt[sizes] = [c for _, c in fam]
            first[sizes] = (self.rank << 40) + np.arange(len(fam), dtype=np.int64)
        if self.cc_comm is not None:
            self.engine.reduce_stats(self.cc_comm, vec, cnt if n else None, first if n else None)
        else:
            self._allreduce(vec, "sum")
            if n:
                self._allreduce(cnt, "sum")
                self._allreduce(first, "min")
        out = {"counters": dict(zip(ckeys, vec[:len(ckeys)].tolist()))}
        out.update(zip(skeys, vec[len(ckeys):].tolist()))
        if fam is not None:
            present = np.nonzero(cnt)[0]
            out["families"] = [(int(s), int(cnt[s])) for s in present[np.argsort(first[present], kind="stable")]]
        if "mapped" in part:
            out["mapped"] = part["mapped"]
        return out

    def _allreduce(self, a, op):
        if self.cc_comm is not None and op == "max":
            self.engine.allreduce_max(self.cc_comm, a)
            return
        import torch
        t = torch.from_numpy(a).to(self._device())
        self.dist.all_reduce(t, op={"sum": self.dist.ReduceOp.SUM, "max": self.dist.ReduceOp.MAX,
                                    "min": self.dist.ReduceOp.MIN}[op], group=self.group)
        a[:] = t.cpu().numpy()

    def broadcast_obj(self, obj):
        lst = [obj]
        self.dist.broadcast_object_list(lst, src=0, group=self.group)
        return lst[0]

    def barrier(self):
        self.dist.barrier(group=self.group)


# ------------------------------------------------------------------ the sample's region geometry
class _Cores(object):
    """tid / pos columns of a record set (what bed_stream reads)."""

    def __init__(self, bam):
        self.tid, self.pos, self.mtid, self.mpos, _ = bam.cores()
        self.n = bam.n


class Geometry(object):
    """The bed regions of a sample, their owner ranks (a block plan of contiguous regions) and the
    per-rank streams and exchanges."""

    def __init__(self, refs, bedfile, blocks):
        self.bedfile = bedfile
        self.refs = refs
        self.regions = region_list(bedfile)
        self.names = {n: i for i, (n, _) in enumerate(refs)}
        # overlapping regions stay in one block (shard.overlap_safe_blocks)
        self.blocks = overlap_safe_blocks(blocks, self.regions)
        self.world = len(self.blocks)
        self.owner = np.zeros(len(self.regions), np.int64)
        for k, (lo, hi) in enumerate(self.blocks):
            self.owner[lo:hi] = k
        self.run = np.array(region_runs(self.regions), np.int32)
        self.keys = [x[0] for x in self.regions]

    def block(self, rank):
        """(tids, begs, ends) of rank's regions (an unknown contig raises, as pysam's fetch does)."""
        lo, hi = self.blocks[rank]
        out = []
        for _, chrom, start, end in self.regions[lo:hi]:
            if chrom not in self.names:
                raise ValueError("invalid contig `%s`" % chrom)
            out.append((self.names[chrom], start, end))
        return ([x[0] for x in out], [x[1] for x in out], [x[2] for x in out])

    def own_stream(self, cores, rank):
        """The rank's own stream over its record set: its regions in bed order, start <= pos < end."""
        st = bed_stream(cores, self.refs, self.bedfile)
        lo, hi = self.blocks[rank]
        keep = (st.region >= lo) & (st.region < hi)
        return st.rec[keep], st.region[keep]

    def sent(self, cores, own, rank):
        """Which of rank's own stream entries are first-streamed ends of pairs completing in another
        rank's block (shard_streams' rule, the mate's region from the record's mate coordinates), and
        each one's destination rank."""
        rec, reg = own
        mate_reg = region_of_positions(self.regions, self.names, cores.mtid[rec], cores.mpos[rec])
        to = np.where(mate_reg >= 0, self.owner[np.maximum(mate_reg, 0)], -1)
        return (mate_reg > reg) & (to >= 0) & (to != rank), to

    def routes(self, bam, cores, own, rank):
        """What rank sends each rank: the first-streamed ends of its pairs completing in the other's
        block (raw records, their regions), in stream order.  They are moved: the receiver pairs and
        counts them, the sender's entries carry CC_REGION_MOVED (stage_input)."""
        rec, reg = own
        send, to = self.sent(cores, own, rank)
        out = []
        for d in range(self.world):
            m = send & (to == d)
            out.append((bam.pack(rec[m]) if m.any() else np.zeros(0, np.uint8), reg[m].astype(np.int32)))
        return out

    def stage_input(self, bam, own, received, mode, delim, it, moved=None):
        """The rank's table (its records and the foreign ends, sorted by position) decoded, and its
        stream: the foreign entries in global stream order (sender rank, then the sender's stream
        order), then its own entries (those moved to another rank marked CC_REGION_MOVED)."""
        blobs = [b for b, _ in received if len(b)]
        fregs = np.concatenate([r for _, r in received]).astype(np.int64) if received else np.zeros(0, np.int64)
        if blobs:
            table = Bam.combine([bam], blobs, key=0)
            inv = np.empty(table.n, np.int64)
            inv[table.origin()] = np.arange(table.n, dtype=np.int64)
        else:
            table, inv = bam, np.arange(bam.n, dtype=np.int64)
        rec, reg = own
        foreign = inv[bam.n + np.arange(len(fregs), dtype=np.int64)]
        srec = np.concatenate([foreign, inv[rec]]).astype(np.int32)
        oreg = reg.astype(np.int64)
        if moved is not None:
            oreg = np.where(moved, oreg | N.REGION_MOVED, oreg)
        sreg = np.concatenate([-(fregs + 1), oreg]).astype(np.int32)
        records = table.decode(it, mode, delim)
        return table, records, Stream(srec, sreg, self.run, self.keys)

    def split_by_position(self, path):
        """A rank's emitted stage output (file order), split by the rank owning each record's position
        (records at no region's position go to rank 0)."""
        b = Bam(path)
        t, p, _, _, _ = b.cores()
        reg = region_of_positions(self.regions, self.names, t, p)
        to = np.where(reg >= 0, self.owner[np.maximum(reg, 0)], 0)
        return [(b.pack(np.nonzero(to == d)[0]) if (to == d).any() else np.zeros(0, np.uint8),)
                for d in range(self.world)], b


def _part(path, rank):
    d, b = os.path.split(path)
    return os.path.join(d, ".shard%d" % rank, b)


def _indexed_input(bam, workdir):
    """The path to read `bam` through, with a current BAI: its own index when one exists and is not
    older than the BAM (htslib warns about an older one; a stale index names the wrong blocks),
    else a new one written next to it, else (a read-only input directory) a link to the BAM in the
    output directory indexed there."""
    bai = bam + ".bai"
    if os.path.exists(bai) and os.path.getmtime(bai) >= os.path.getmtime(bam):
        return bam
    try:
        index_bam(bam)
        return bam
    except (IOError, OSError):
        os.makedirs(workdir, exist_ok=True)
        link = os.path.join(workdir, ".input." + os.path.basename(bam))
        if os.path.lexists(link):
            os.remove(link)
        os.symlink(os.path.abspath(bam), link)
        index_bam(link)
        return link


def region_plan(bam_path, bedfile, world):
    """The sample's block plan: contiguous region blocks with near-equal compressed bytes, from the
    input's BAI (no decode)."""
    hdr = Bam.open_regions(bam_path, [], [], [])
    names = {n: i for i, (n, _) in enumerate(hdr.refs)}
    regions = region_list(bedfile)
    t = np.array([names.get(c, -1) for _, c, _, _ in regions], np.int32)
    b = np.array([s for _, _, s, _ in regions], np.int64)
    e = np.array([x for _, _, _, x in regions], np.int64)
    w = np.zeros(len(regions), np.int64)
    if N.io().ccio_bai_region_bytes(bam_path.encode(), len(regions), N.ptr(t), N.ptr(b), N.ptr(e), N.ptr(w)) != 0:
        raise IOError(N.io_error())
    return plan_blocks(w, world)


def to_owners(comm, geo, paths):
    """Stage outputs by position owner: each rank's emitted part (paths[r]) split by the rank owning
    each record's position, exchanged, and stably sorted in sender order with the samtools stand-in
    key: each rank's part of the whole-sample sorted file."""
    split = comm.each(lambda r: geo.split_by_position(paths[r]))
    recv = comm.exchange({r: split[r][0] for r in split})
    return comm.each(lambda r: Bam.combine([], [x[0] for x in recv[r]], key=1, tmpl=split[r][1]))


def sharded_pipeline(bam, c_output, bedfile, comm, engine, cutoff=0.7, bdelim="|", scorrect="True", level=6,
                     verbose=False, blocks=None, held=None, refs=None, keep=None, finalize=True):
    """ConsensusCruncher.py:127-346 with every stage split over comm.world region shards.  Same files
    and contents as pipeline.consensus_pipeline; rank 0 returns the output paths.

    held / refs / blocks: the ranks' record sets are given (bench.py: per-rank generated samples, already
    at their owners) instead of read from bam through its BAI; keep: a dict that receives the stage runs
    ({stage: {rank: run}}) resident on the GPU instead of closing them; finalize=False skips the
    merge of the ranks' parts into the whole-sample output files."""
    if bedfile in (None, "False"):
        raise ValueError("sharding needs the bed regions (-b / genome)")
    world = comm.world
    root = comm.rank == 0
    identifier = os.path.basename(bam).split('.bam', 1)[0]
    sd = '{}/{}'.format(c_output, identifier)
    subs = ("sscs", "dcs", "sscs_sc", "dcs_sc")
    for sub in subs:
        for r in comm.ranks:
            os.makedirs(os.path.join(sd, sub, ".shard%d" % r), exist_ok=True)
    if held is None:
        # the ranks read their regions through the input's BAI (rank 0 indexes it when needed)
        got = comm.each(lambda r: _indexed_input(bam, c_output) if r == 0 else None)
        bam = comm.broadcast_obj(got[0] if root else None)
        refs = Bam.open_regions(bam, [], [], []).refs
        if blocks is None:
            blocks = comm.broadcast_obj(region_plan(bam, bedfile, world) if root else None)
    geo = Geometry(refs, bedfile, blocks)
    start = time.time()
    P = lambda sub, name: '{}/{}/{}.{}'.format(sd, sub, identifier, name)  # noqa: E731

    def done(stage, runs, r, run):
        """a stage run after its emit: kept resident (bench) or closed"""
        if keep is not None:
            keep.setdefault(stage, {})[r] = run
        else:
            run.close()

    def routed(helds, mode, delim, it_of):
        """Each rank's stage tables and streams for the record sets helds[k][r] (k: the stage's inputs)."""
        cores = comm.each(lambda r: [_Cores(h[r]) for h in helds])
        own = comm.each(lambda r: [geo.own_stream(c, r) for c in cores[r]])
        out = []
        for k, h in enumerate(helds):
            recv = comm.exchange(comm.each(lambda r: geo.routes(h[r], cores[r][k], own[r][k], r)))
            out.append(comm.each(lambda r: geo.stage_input(h[r], own[r][k], recv[r], mode, delim, it_of[r],
                                                           geo.sent(cores[r][k], own[r][k], r)[0])))
        return out

    def save(local, sub, name):
        comm.each(lambda r: local[r].write_all(_part(P(sub, name), r), level))

    def on_root(fn):
        """rank 0's host work between stages; a raise there reaches every rank (comm.each)"""
        comm.each(lambda r: fn() if r == 0 else None)

    def move(a, b):   # the stats / time-tracker moves of ConsensusCruncher.py:200-203,225-228,275-278
        os.rename(P(a, "stats.txt"), P(b, "stats.txt"))
        os.rename(P(a, "time_tracker.txt"), P(b, "time_tracker.txt"))

    # ---- SSCS
    if held is None:
        held = comm.each(lambda r: Bam.open_regions(bam, *geo.block(r)))
    its = comm.each(lambda r: Interner())
    (inp,) = routed([held], MODE_SSCS, bdelim, its)
    sscs = P("sscs", "sscs.bam")
    prefix = sscs.split('.sscs')[0]

    def sscs1(r):
        table, rec, stream = inp[r]
        run = SSCSRun(engine, None, cutoff, bedfile, bdelim, src=(table, its[r], rec, stream))
        try:
            return run.emit(_part(sscs, r), level, verbose=False, side=False, plot=False)
        finally:
            done("sscs", keep, r, run)
    tot = comm.reduce(comm.each(sscs1))
    del inp, held

    def sscs2():
        concat_bams(prefix + '.badReads.bam', [_part(prefix + '.badReads.bam', r) for r in range(world)], level)
        # AlignmentFile.mapped from the BAI's pseudo-bins; without them (an index that does not write
        # them), the mapped records the ranks streamed (records outside every region not counted)
        tot["mapped"] = int(N.io().ccio_bai_mapped(bam.encode())) if os.path.exists(bam + ".bai") else -1
        if tot["mapped"] < 0:
            tot["mapped"] = tot.get("mapped_own", -1)
        sscs_side(prefix, tot, geo.keys, start, verbose)
    on_root(sscs2)
    sscs_loc = to_owners(comm, geo, {r: _part(sscs, r) for r in comm.ranks})
    sing_loc = to_owners(comm, geo, {r: _part(prefix + '.singleton.bam', r) for r in comm.ranks})
    save(sscs_loc, "sscs", "sscs.sorted.bam")
    save(sing_loc, "sscs", "singleton.sorted.bam")
    on_root(lambda: move("sscs", "dcs"))

    # ---- DCS (and DCS+SC below)
    def dcs_stage(src_loc, outfile):
        its_d = comm.each(lambda r: Interner())
        (din,) = routed([src_loc], MODE_DUPLEX, None, its_d)
        single = ('{}.sscs.sc.singleton.bam'.format(outfile.split('.dcs.sc')[0]) if '.dcs.sc' in outfile
                  else '{}.sscs.singleton.bam'.format(outfile.split('.dcs')[0]))

        def p1(r):
            table, rec, stream = din[r]
            run = DCSRun(engine, None, bedfile, src=(table, its_d[r], rec, stream))
            try:
                return run.emit(_part(outfile, r), level, verbose=False, side=False)
            finally:
                done("dcs_sc" if '.dcs.sc' in outfile else "dcs", keep, r, run)
        t = comm.reduce(comm.each(p1))
        on_root(lambda: dcs_side(outfile, t, start, verbose))
        dloc = to_owners(comm, geo, {r: _part(outfile, r) for r in comm.ranks})
        sloc = to_owners(comm, geo, {r: _part(single, r) for r in comm.ranks})
        return dloc, sloc

    dcs_loc, ss_loc = dcs_stage(sscs_loc, P("dcs", "dcs.bam"))
    save(dcs_loc, "dcs", "dcs.sorted.bam")
    save(ss_loc, "dcs", "sscs.singleton.sorted.bam")
    del dcs_loc, ss_loc
    finals = [("sscs", "sscs.sorted.bam"), ("sscs", "singleton.sorted.bam"), ("dcs", "dcs.sorted.bam"),
              ("dcs", "sscs.singleton.sorted.bam")]
    out = dict(badreads=prefix + '.badReads.bam')
    if scorrect != 'False':
        on_root(lambda: move("dcs", "sscs"))
        # ---- SC: singletons against the SSCS, both rank-local
        its_c = comm.each(lambda r: Interner())
        s_in, x_in = routed([sing_loc, sscs_loc], MODE_DUPLEX, None, its_c)
        base = P("sscs", "singleton.sorted.bam").split('.singleton')[0]

        def sc1(r):
            d = os.path.join(os.path.dirname(base), ".shard%d" % r)
            b = os.path.join(d, os.path.basename(base))
            (st, sr, ss), (xt, xr, xs) = s_in[r], x_in[r]
            run = SCRun(engine, b + '.singleton.sorted.bam', bedfile, src=(its_c[r], (st, sr, ss), (xt, xr, xs)))
            try:
                return run.emit(level, verbose=False, side=False)
            finally:
                done("sc", keep, r, run)
        t = comm.reduce(comm.each(sc1))
        del s_in, x_in
        on_root(lambda: sc_side(base, t, verbose))
        sc_loc = {}
        for name in ("sscs.correction", "singleton.correction", "uncorrected"):
            sc_loc[name] = to_owners(comm, geo, {r: _part('{}.{}.bam'.format(base, name), r) for r in comm.ranks})
            save(sc_loc[name], "sscs_sc", name + ".sorted.bam")
            finals.append(("sscs_sc", name + ".sorted.bam"))
        # merge(sscs.sorted, sscs.correction.sorted, singleton.correction.sorted) + sort, per rank
        sscs_sc_loc = comm.each(lambda r: Bam.combine([sscs_loc[r], sc_loc["sscs.correction"][r],
                                                       sc_loc["singleton.correction"][r]], [], key=1))
        save(sscs_sc_loc, "sscs_sc", "sscs.sc.sorted.bam")
        finals.append(("sscs_sc", "sscs.sc.sorted.bam"))
        del sscs_loc, sing_loc
        on_root(lambda: move("sscs", "dcs_sc"))
        dsc_loc, ssc_loc = dcs_stage(sscs_sc_loc, P("dcs_sc", "dcs.sc.bam"))
        save(dsc_loc, "dcs_sc", "dcs.sc.sorted.bam")
        save(ssc_loc, "dcs_sc", "sscs.sc.singleton.sorted.bam")
        au = comm.each(lambda r: Bam.combine([dsc_loc[r], ssc_loc[r], sc_loc["uncorrected"][r]], [], key=1))
        save(au, "dcs_sc", "all.unique.dcs.sorted.bam")
        finals += [("dcs_sc", "dcs.sc.sorted.bam"), ("dcs_sc", "sscs.sc.singleton.sorted.bam"),
                   ("dcs_sc", "all.unique.dcs.sorted.bam")]
        del dsc_loc, ssc_loc, au, sc_loc, sscs_sc_loc

    def finish():
        # the reference's output files: the ranks' sorted parts merged (ties in rank order)
        for sub, name in finals:
            merge_bams(P(sub, name), [_part(P(sub, name), r) for r in range(world)], level)
            index_bam(P(sub, name))
        if scorrect != 'False':
            os.rename(P("dcs_sc", "stats.txt"), '{}/{}.stats.txt'.format(sd, identifier))
            os.rename(P("dcs_sc", "time_tracker.txt"), '{}/{}.time_tracker.txt'.format(sd, identifier))
        else:
            os.rename(P("dcs", "stats.txt"), '{}/{}.stats.txt'.format(sd, identifier))
            os.rename(P("dcs", "time_tracker.txt"), '{}/{}.time_tracker.txt'.format(sd, identifier))
        png = '{}/sscs/{}_tag_fam_size.png'.format(sd, identifier)
        if os.path.exists(png):
            os.rename(png, '{}/{}_tag_fam_size.png'.format(sd, identifier))
        os.rename(P("sscs", "read_families.txt"), '{}/{}.read_families.txt'.format(sd, identifier))
        for sub in subs:
            for r in range(world):
                shutil.rmtree(os.path.join(sd, sub, ".shard%d" % r), ignore_errors=True)
    if finalize:
        on_root(finish)
    out.update(sscs=P("sscs", "sscs.sorted.bam"), singleton=P("sscs", "singleton.sorted.bam"),
               dcs=P("dcs", "dcs.sorted.bam"), sscs_singleton=P("dcs", "sscs.singleton.sorted.bam"))
    if scorrect != 'False':
        out.update(sscs_correction=P("sscs_sc", "sscs.correction.sorted.bam"),
                   singleton_correction=P("sscs_sc", "singleton.correction.sorted.bam"),
                   uncorrected=P("sscs_sc", "uncorrected.sorted.bam"), sscs_sc=P("sscs_sc", "sscs.sc.sorted.bam"),
                   dcs_sc=P("dcs_sc", "dcs.sc.sorted.bam"), sscs_sc_singleton=P("dcs_sc", "sscs.sc.singleton.sorted.bam"),
                   all_unique=P("dcs_sc", "all.unique.dcs.sorted.bam"))
    out["stats"] = '{}/{}.stats.txt'.format(sd, identifier)
    out["read_families"] = '{}/{}.read_families.txt'.format(sd, identifier)
    return out if root else None


def main(argv=None):
    """`ConsensusCruncher.py consensus` (its argv :461-518; consensus() :127-346) on the GPUs of one
    node: one process per GPU under torch.distributed.run (RCCL), the stages split over the bed regions;
    a single process runs pipeline.consensus_pipeline on GPU 0.

        python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
            -m consensuscruncher_amd.sharded -i sample.sorted.bam -o out -g hg38
    """
    import argparse
    from .pipeline import cleanup, consensus_pipeline, genome_bedfile
    from .stages import get_engine
    p = argparse.ArgumentParser(prog="consensuscruncher_amd.sharded")
    p.add_argument('-i', '--input', dest='bam', required=True, type=str)
    p.add_argument('-o', '--output', dest='c_output', required=True, type=str)
    p.add_argument('--scorrect', choices=['True', 'False'], default='True')
    p.add_argument('-g', '--genome', dest='genome', choices=['hg19', 'hg38', 'hg38_noAlt'], default='hg19')
    # the reference's default bed is its bundled hg19 cytobands (ConsensusCruncher.py:413-433)
    p.add_argument('-b', '--bedfile', type=str, default=os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                                     "data", "hg19_cytoBand.txt"))
    p.add_argument('--cutoff', type=float, default=0.7)
    p.add_argument('-d', '--bdelim', type=str, default='|')
    p.add_argument('--cleanup', choices=['True', 'False'], default='False')
    args = p.parse_args(argv)
    bedfile = genome_bedfile(args.genome, args.bedfile)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        eng = get_engine()
        consensus_pipeline(args.bam, args.c_output, bedfile=bedfile, cutoff=args.cutoff, bdelim=args.bdelim,
                           scorrect=args.scorrect, engine=eng, cleanup_files=args.cleanup)
        return
    import torch
    import torch.distributed as dist
    from .engine import Engine
    # CC_DIST_BACKEND=gloo with CC_DEVICE=k: every rank on GPU k, the reduction on the CPU (a one-GPU
    # rehearsal of the multi-GPU run; tests/test_gpu_shard.py)
    backend = os.environ.get("CC_DIST_BACKEND", "nccl")
    dev = int(os.environ["CC_DEVICE"]) if "CC_DEVICE" in os.environ else int(os.environ.get("LOCAL_RANK", "0"))
    if backend == "nccl":
        torch.cuda.set_device(dev)
    dist.init_process_group(backend)
    comm = None
    try:
        eng = Engine(dev)
        comm = TorchComm(engine=eng)
        out = sharded_pipeline(args.bam, args.c_output, bedfile, comm, eng, cutoff=args.cutoff,
                               bdelim=args.bdelim, scorrect=args.scorrect)
        if out is not None and args.cleanup == 'True':
            identifier = os.path.basename(args.bam).split('.bam', 1)[0]
            cleanup('{}/{}'.format(args.c_output, identifier), identifier, args.scorrect)
        dist.barrier()
        comm.close()
        eng.close()
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
