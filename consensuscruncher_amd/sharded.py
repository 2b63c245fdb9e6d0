"""One sample's consensus pipeline over several GPUs, split along the bed regions.

The reference processes its bed regions one after another (SSCS_maker.py:265-281,
DCS_maker.py:204-218, singleton_correction.py:203-229; consensus_helper.py:38-54).  A family, its
duplex partner and its singleton-correction complement share their coordinates, so they complete
in one region; the regions therefore split into contiguous blocks, one per GPU, and every stage of
the sample uses the same block plan (shard.plan_blocks over the input's reads per region).

Per stage, every rank runs the stage on its block (shard.shard_streams: its regions, plus the
first-streamed mates of pairs that complete in its block, routed in as foreign entries) and writes
its part of each output BAM.  The parts joined in rank order are the reference's region-major
emission order, so rank 0 concatenates them (engine.concat_bams) into the stage's output file.  The
stats.txt / read_families.txt quantities of the parts are reduced over the ranks (the multi-GPU
path's one collective: a sum of counters and a merge of the family-size tables, over RCCL on GPUs)
and rank 0 writes the side outputs.  Sorts and merges between the stages are the single-GPU
pipeline's (pipeline.py, ConsensusCruncher.py:127-346), on rank 0; the next stage reads the
whole-sample file, as the reference's next script does.

Two drivers run the same stage code: LocalComm runs the ranks one after another in this process on
one GPU (tests: the joined outputs must equal the single-pass pipeline's byte for byte); TorchComm
is one process per GPU under torch.distributed.
"""
import os
import shutil
import time

import numpy as np

from .consensus_helper import region_list
from .engine import Bam, Interner, MODE_SSCS, bed_stream, concat_bams, merge_bams
from .pipeline import sort_index
from .shard import plan_blocks, shard_streams
from .stages import DCSRun, SCRun, SSCSRun, dcs_side, sc_side, sscs_side

COUNTER_KEYS = ("COUNTER", "UNMAPPED", "UNMAPPED_MATE", "MULTIPLE_MAPPING", "BAD_SPACER", "PAIRS", "READ_ENDS",
                "FAMILIES", "ENTRIES", "UNPAIRED", "ORPHAN_TAGS", "DROPPED", "BAD_LISTED", "FOREIGN")
SCALARS = ("sscs", "singletons", "never_emitted", "dcs", "sscs_singletons", "processed", "sscs_correction",
           "singleton_correction", "uncorrected")


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
        out["mapped"] = parts[0]["mapped"]   # a whole-file count (every rank decodes the whole file)
    return out


class LocalComm(object):
    """world ranks run one after another in this process (one GPU)."""

    def __init__(self, world):
        self.world = world
        self.rank = 0

    def run_stage(self, phase1, phase2):
        parts = [phase1(r) for r in range(self.world)]
        return phase2(combine_parts(parts))

    def broadcast_obj(self, obj):
        return obj

    def barrier(self):
        pass


class TorchComm(object):
    """One process per GPU under torch.distributed (RCCL as backend "nccl" on ROCm, gloo on CPU)."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)

    def _device(self):
        import torch
        if self.dist.get_backend(self.group) == "nccl":
            return torch.device("cuda", torch.cuda.current_device())
        return torch.device("cpu")

    def reduce_part(self, part):
        """combine_parts over the ranks with collectives: one SUM of the counter/count vector, and for
        the family table a MAX of its length, a SUM of the per-size counts and a MIN of each size's
        first-seen key (rank << 40 | place)."""
        import torch
        dev = self._device()
        ckeys = sorted(part["counters"])
        skeys = [k for k in SCALARS if k in part]
        vec = torch.tensor([part["counters"][k] for k in ckeys] + [part[k] for k in skeys], dtype=torch.int64,
                           device=dev)
        self.dist.all_reduce(vec, op=self.dist.ReduceOp.SUM, group=self.group)
        v = vec.cpu().tolist()
        out = {"counters": dict(zip(ckeys, v[:len(ckeys)]))}
        out.update(zip(skeys, v[len(ckeys):]))
        if "families" in part:
            fam = part["families"]
            top = torch.tensor([max([s for s, _ in fam], default=0)], dtype=torch.int64, device=dev)
            self.dist.all_reduce(top, op=self.dist.ReduceOp.MAX, group=self.group)
            n = int(top.item()) + 1
            cnt = torch.zeros(n, dtype=torch.int64, device=dev)
            first = torch.full((n,), 1 << 62, dtype=torch.int64, device=dev)
            if fam:
                sizes = torch.tensor([s for s, _ in fam], dtype=torch.int64, device=dev)
                cnt[sizes] = torch.tensor([c for _, c in fam], dtype=torch.int64, device=dev)
                first[sizes] = (self.rank << 40) + torch.arange(len(fam), dtype=torch.int64, device=dev)
            self.dist.all_reduce(cnt, op=self.dist.ReduceOp.SUM, group=self.group)
            self.dist.all_reduce(first, op=self.dist.ReduceOp.MIN, group=self.group)
            c, f = cnt.cpu().numpy(), first.cpu().numpy()
            present = np.nonzero(c)[0]
            out["families"] = [(int(s), int(c[s])) for s in present[np.argsort(f[present], kind="stable")]]
        if "mapped" in part:
            out["mapped"] = part["mapped"]
        return out

    def run_stage(self, phase1, phase2):
        combined = self.reduce_part(phase1(self.rank))
        self.barrier()
        res = phase2(combined) if self.rank == 0 else None
        self.barrier()
        return res

    def broadcast_obj(self, obj):
        lst = [obj]
        self.dist.broadcast_object_list(lst, src=0, group=self.group)
        return lst[0]

    def barrier(self):
        self.dist.barrier(group=self.group)


def region_plan(bam_path, bedfile, world, delim="|"):
    """The sample's block plan: contiguous region blocks with near-equal input reads."""
    b = Bam(bam_path)
    try:
        st = bed_stream(b.decode(Interner(), MODE_SSCS, delim), b.refs, bedfile)
        return plan_blocks(np.bincount(st.region, minlength=len(region_list(bedfile))), world)
    finally:
        b.close()


def _shard_fn(bedfile, world, rank, blocks):
    regions = region_list(bedfile)

    def fn(bam, rec):
        st = bed_stream(rec, bam.refs, bedfile)
        streams, _ = shard_streams(rec, bam.refs, regions, st, world, blocks)
        return streams[rank]
    return fn


def _part(path, rank):
    d, b = os.path.split(path)
    return os.path.join(d, ".shard%d" % rank, b)


def _join(path, world, level):
    concat_bams(path, [_part(path, r) for r in range(world)], level)


def sharded_pipeline(bam, c_output, bedfile, comm, engine, cutoff=0.7, bdelim="|", scorrect="True", level=6,
                     verbose=False, blocks=None):
    """ConsensusCruncher.py:127-346 with every stage split over comm.world region shards.  Same files
    and contents as pipeline.consensus_pipeline; rank 0 returns the output paths."""
    if bedfile in (None, "False"):
        raise ValueError("sharding needs the bed regions (-b / genome)")
    world = comm.world
    identifier = os.path.basename(bam).split('.bam', 1)[0]
    sd = '{}/{}'.format(c_output, identifier)
    if blocks is None:
        blocks = comm.broadcast_obj(region_plan(bam, bedfile, world, bdelim) if comm.rank == 0 else None)
    for sub in ("sscs", "dcs", "sscs_sc", "dcs_sc"):
        for r in range(world):
            os.makedirs(os.path.join(sd, sub, ".shard%d" % r), exist_ok=True)
    comm.barrier()
    start = time.time()
    regions = region_list(bedfile)
    shard = lambda r: _shard_fn(bedfile, world, r, blocks)  # noqa: E731

    # ---- SSCS
    sscs = '{}/sscs/{}.sscs.bam'.format(sd, identifier)
    prefix = sscs.split('.sscs')[0]

    def sscs1(r):
        run = SSCSRun(engine, bam, cutoff, bedfile, bdelim, shard=shard(r))
        try:
            return run.emit(_part(sscs, r), level, verbose=False, side=False)
        finally:
            run.close()

    def sscs2(tot):
        for f in (sscs, prefix + '.singleton.bam', prefix + '.badReads.bam'):
            _join(f, world, level)
        sscs_side(prefix, tot, [k for k, _, _, _ in regions], start, verbose)
    comm.run_stage(sscs1, sscs2)
    out = dict(badreads='{}/sscs/{}.badReads.bam'.format(sd, identifier))
    if comm.rank == 0:
        out["sscs"] = sort_index(sscs, level)
        out["singleton"] = sort_index(prefix + '.singleton.bam', level)
        os.rename('{}/sscs/{}.stats.txt'.format(sd, identifier), '{}/dcs/{}.stats.txt'.format(sd, identifier))
        os.rename('{}/sscs/{}.time_tracker.txt'.format(sd, identifier),
                  '{}/dcs/{}.time_tracker.txt'.format(sd, identifier))
    comm.barrier()
    out["sscs"] = '{}/sscs/{}.sscs.sorted.bam'.format(sd, identifier)
    out["singleton"] = '{}/sscs/{}.singleton.sorted.bam'.format(sd, identifier)

    # ---- DCS (and DCS+SC below)
    def dcs_stage(infile, outfile):
        single = ('{}.sscs.sc.singleton.bam'.format(outfile.split('.dcs.sc')[0]) if '.dcs.sc' in outfile
                  else '{}.sscs.singleton.bam'.format(outfile.split('.dcs')[0]))

        def p1(r):
            run = DCSRun(engine, infile, bedfile, shard=shard(r))
            try:
                return run.emit(_part(outfile, r), level, verbose=False, side=False)
            finally:
                run.close()

        def p2(tot):
            _join(outfile, world, level)
            _join(single, world, level)
            dcs_side(outfile, tot, start, verbose)
        comm.run_stage(p1, p2)
        return single

    dcs = '{}/dcs/{}.dcs.bam'.format(sd, identifier)
    single = dcs_stage(out["sscs"], dcs)
    if comm.rank == 0:
        sort_index(dcs, level)
        sort_index(single, level)
    comm.barrier()
    out["dcs"] = '{}/dcs/{}.dcs.sorted.bam'.format(sd, identifier)
    out["sscs_singleton"] = '{}/dcs/{}.sscs.singleton.sorted.bam'.format(sd, identifier)
    if scorrect != 'False':
        if comm.rank == 0:
            os.rename('{}/dcs/{}.stats.txt'.format(sd, identifier), '{}/sscs/{}.stats.txt'.format(sd, identifier))
            os.rename('{}/dcs/{}.time_tracker.txt'.format(sd, identifier),
                      '{}/sscs/{}.time_tracker.txt'.format(sd, identifier))
        comm.barrier()
        # ---- SC: every rank reads the whole singleton/SSCS files through its own part paths
        base = out["singleton"].split('.singleton')[0]
        rest = out["singleton"].split('.singleton')[1]

        def sc1(r):
            d = os.path.join(os.path.dirname(base), ".shard%d" % r)
            b = os.path.join(d, os.path.basename(base))
            for src, dst in ((out["singleton"], b + '.singleton' + rest), ('{}.sscs{}'.format(base, rest),
                                                                            b + '.sscs' + rest)):
                if not os.path.exists(dst):
                    os.symlink(os.path.abspath(src), dst)
            run = SCRun(engine, b + '.singleton' + rest, bedfile, shard=shard(r))
            try:
                return run.emit(level, verbose=False, side=False)
            finally:
                run.close()

        def sc2(tot):
            for name in ("sscs.correction", "singleton.correction", "uncorrected"):
                _join('{}.{}.bam'.format(base, name), world, level)
            sc_side(base, tot, verbose)
        comm.run_stage(sc1, sc2)
        moved = {}
        for name in ("sscs.correction", "singleton.correction", "uncorrected"):
            dst = '{}/sscs_sc/{}.{}.bam'.format(sd, identifier, name)
            if comm.rank == 0:
                os.rename('{}/sscs/{}.{}.bam'.format(sd, identifier, name), dst)
                sort_index(dst, level)
            moved[name] = '{}.sorted.bam'.format(dst.split('.bam', 1)[0])
        sscs_sc = '{}/sscs_sc/{}.sscs.sc.bam'.format(sd, identifier)
        if comm.rank == 0:
            merge_bams(sscs_sc, [out["sscs"], moved["sscs.correction"], moved["singleton.correction"]], level)
            sort_index(sscs_sc, level)
            os.rename('{}/sscs/{}.stats.txt'.format(sd, identifier), '{}/dcs_sc/{}.stats.txt'.format(sd, identifier))
            os.rename('{}/sscs/{}.time_tracker.txt'.format(sd, identifier),
                      '{}/dcs_sc/{}.time_tracker.txt'.format(sd, identifier))
        comm.barrier()
        sscs_sc = '{}/sscs_sc/{}.sscs.sc.sorted.bam'.format(sd, identifier)
        dcs_sc = '{}/dcs_sc/{}.dcs.sc.bam'.format(sd, identifier)
        single = dcs_stage(sscs_sc, dcs_sc)
        all_unique = '{}/dcs_sc/{}.all.unique.dcs.bam'.format(sd, identifier)
        if comm.rank == 0:
            dcs_sc = sort_index(dcs_sc, level)
            single = sort_index(single, level)
            merge_bams(all_unique, [dcs_sc, single, moved["uncorrected"]], level)
            all_unique = sort_index(all_unique, level)
            os.rename('{}/dcs_sc/{}.stats.txt'.format(sd, identifier), '{}/{}.stats.txt'.format(sd, identifier))
            os.rename('{}/dcs_sc/{}.time_tracker.txt'.format(sd, identifier),
                      '{}/{}.time_tracker.txt'.format(sd, identifier))
        out.update(sscs_correction=moved["sscs.correction"], singleton_correction=moved["singleton.correction"],
                   uncorrected=moved["uncorrected"], sscs_sc=sscs_sc,
                   dcs_sc='{}/dcs_sc/{}.dcs.sc.sorted.bam'.format(sd, identifier),
                   sscs_sc_singleton='{}/dcs_sc/{}.sscs.sc.singleton.sorted.bam'.format(sd, identifier),
                   all_unique='{}/dcs_sc/{}.all.unique.dcs.sorted.bam'.format(sd, identifier))
    elif comm.rank == 0:
        os.rename('{}/dcs/{}.stats.txt'.format(sd, identifier), '{}/{}.stats.txt'.format(sd, identifier))
        os.rename('{}/dcs/{}.time_tracker.txt'.format(sd, identifier), '{}/{}.time_tracker.txt'.format(sd, identifier))
    if comm.rank == 0:
        if os.path.exists('{}/sscs/{}_tag_fam_size.png'.format(sd, identifier)):
            os.rename('{}/sscs/{}_tag_fam_size.png'.format(sd, identifier),
                      '{}/{}_tag_fam_size.png'.format(sd, identifier))
        os.rename('{}/sscs/{}.read_families.txt'.format(sd, identifier),
                  '{}/{}.read_families.txt'.format(sd, identifier))
        for sub in ("sscs", "dcs", "sscs_sc", "dcs_sc"):
            for r in range(world):
                shutil.rmtree(os.path.join(sd, sub, ".shard%d" % r), ignore_errors=True)
    comm.barrier()
    out["stats"] = '{}/{}.stats.txt'.format(sd, identifier)
    out["read_families"] = '{}/{}.read_families.txt'.format(sd, identifier)
    return out if comm.rank == 0 else None


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
    try:
        eng = Engine(dev)
        out = sharded_pipeline(args.bam, args.c_output, bedfile, TorchComm(), eng, cutoff=args.cutoff,
                               bdelim=args.bdelim, scorrect=args.scorrect)
        if out is not None and args.cleanup == 'True':
            identifier = os.path.basename(args.bam).split('.bam', 1)[0]
            cleanup('{}/{}'.format(args.c_output, identifier), identifier, args.scorrect)
        dist.barrier()
        eng.close()
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
