#!/usr/bin/env python3
"""bench.py — input reads/s through SSCS+DCS+SC consensus on MI355X (BASELINE.json metric).

One step = the whole consensus chain of ConsensusCruncher's `consensus` mode on
the GPU over one rank's synthetic sample, with every input already resident in
HBM: SSCS read_bam + consensus_maker, DCS (on the sorted SSCS), singleton
correction (singletons vs SSCS) and DCS+SC (on the merged SSCS+SC), i.e. four
read_bam passes (filter, qname pairing, tag grouping, csn entries) plus the
votes and duplex/SC joins.  The inputs of the later stages are the earlier
stages' real outputs, produced once in setup through the product's host path
(BAM encode, sort, merge, decode) — that setup pass is also timed and reported
as the end-to-end rate.

Workloads: N=1 runs C2 (BASELINE.json configs[1]: 10 M pairs, one contig, -b False).  N>1
(`--gpus N`: one process per GPU, spawned here through torch.distributed.run when WORLD_SIZE is
unset) runs C3 (configs[2]): ONE hg38 sample of 25 M pairs per GPU (N = 8: BASELINE's 200 M pairs;
weak scaling), split along the bundled hg38_cytoBand.txt into N blocks of consecutive regions
(SURVEY.md §8e), through the product's multi-GPU driver (consensuscruncher_amd/sharded.py): each
rank generates its block's molecules (0.1% translocated mates anywhere on the genome, 0.5% pairs
straddling a region boundary), the records go to the ranks owning their positions, and every
stage runs on the rank-local record sets with the cross-block first mates routed in as foreign
entries.  A step re-runs each stage's device chain on every rank plus the stage's one collective
(the stats counters, cc_reduce_stats over RCCL); the records exchanges and the host I/O are the
setup pass, outside the timed region as at N = 1.

cpu_baseline (rank 0, N=1, before the GPU is touched): the C++ oracle (oracle/cc_oracle.cpp, the
reference's dictionary program restated in C++ and pinned to the reference's outputs) on a bounded
sample of the same model, consensus-only time, one core and one process per core.
"""
import argparse
import json
import os
import shutil
import socket
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E peak (MI355X_MICROARCH.md)


def log(*a):
    print("[bench r%s]" % os.environ.get("RANK", "0"), *a, file=sys.stderr, flush=True)


def build_stages(eng, work, input_bam, cutoff, bed=None):
    """First pass through the product path (pipeline.consensus_pipeline's flow: stage outputs written
    sorted + indexed at once, the next stage reading them from memory); returns the resident runs +
    timings (each host and device piece of the end-to-end pass timed on its own)."""
    from consensuscruncher_amd.engine import Sink, flush_writes, merge_kept
    from consensuscruncher_amd.stages import DCSRun, SCRun, SSCSRun
    t = {}
    p = lambda n: os.path.join(work, "sample." + n)  # noqa: E731
    clock = [time.time()]

    def lap(name):
        now = time.time()
        t[name] = round(t.get(name, 0.0) + now - clock[0], 3)
        clock[0] = now

    t0 = clock[0]
    outs = ["sscs", "singleton", "dcs", "sscs.singleton", "sscs.correction", "singleton.correction", "uncorrected",
            "dcs.sc", "sscs.sc.singleton"]
    sink = Sink(fused=[p(n + ".bam") for n in outs],
                keep=[p(n + ".bam") for n in ("sscs", "singleton", "sscs.correction", "singleton.correction")],
                async_writes=True)
    sscs = SSCSRun(eng, input_bam, cutoff, bedfile=bed)
    lap("sscs_run")
    t.update({"sscs_run." + k: round(v, 3) for k, v in sscs.times.items()})
    sscs.emit(p("sscs.bam"), level=1, verbose=False, plot=False, sink=sink)
    lap("sscs_emit")
    t.update({"sscs_emit." + k[5:]: round(v, 3) for k, v in sscs.times.items() if k.startswith("emit_")})
    sscs_h, sing_h = sink.take(p("sscs.sorted.bam")), sink.take(p("singleton.sorted.bam"))
    dcs = DCSRun(eng, p("sscs.sorted.bam"), bedfile=bed, bam=sscs_h)
    lap("dcs_run")
    t.update({"dcs_run." + k: round(v, 3) for k, v in dcs.times.items()})
    dcs.emit(p("dcs.bam"), level=1, verbose=False, sink=sink)
    lap("dcs_emit")
    t.update({"dcs_emit." + k[5:]: round(v, 3) for k, v in dcs.times.items() if k.startswith("emit_")})
    # the product pipeline's SC joins the DCS run's grouping of the same sorted SSCS file without a bed
    # (pipeline.consensus_pipeline; stages.SCRun sscs_run)
    sc = SCRun(eng, p("singleton.sorted.bam"), bedfile=bed, sscs_run=dcs if bed is None else None, bam=sing_h,
               xbam=sscs_h)
    lap("sc_run")
    sc.emit(level=1, verbose=False, sink=sink)
    lap("sc_emit")
    sscs_sc_h = merge_kept(p("sscs.sc.sorted.bam"), [sscs_h, sink.take(p("sscs.correction.sorted.bam")),
                                                     sink.take(p("singleton.correction.sorted.bam"))], 1,
                           async_writes=True)
    lap("merge")
    dcssc = DCSRun(eng, p("sscs.sc.sorted.bam"), bedfile=bed, bam=sscs_sc_h)
    lap("dcs_sc_run")
    t.update({"dcs_sc_run." + k: round(v, 3) for k, v in dcssc.times.items()})
    dcssc.emit(p("dcs.sc.bam"), level=1, verbose=False, sink=sink)
    lap("dcs_sc_emit")
    t.update({"dcs_sc_emit." + k[5:]: round(v, 3) for k, v in dcssc.times.items() if k.startswith("emit_")})
    flush_writes()   # every output compressed and on disk (the writes ran in the background)
    lap("flush")
    t["e2e"] = time.time() - t0
    return [("sscs", sscs), ("dcs", dcs), ("sc", sc), ("dcs_sc", dcssc)], t


C3_PAIRS_PER_GPU = 25_000_000


def build_sharded(eng, comm, work, rank_bam, cutoff, bed):
    """Setup of the multi-GPU workload: this rank's generated records go to the ranks owning their
    positions (sharded.to_owners), then the product's sharded pipeline runs every stage once with the
    stage runs kept resident on the GPU; returns them + timings."""
    from consensuscruncher_amd.engine import Bam
    from consensuscruncher_amd.sharded import Geometry, sharded_pipeline, to_owners
    from consensuscruncher_amd.consensus_helper import region_list
    from consensuscruncher_amd.shard import plan_blocks
    t0 = time.time()
    b = Bam(rank_bam)
    refs = b.refs
    del b
    # the plan the sample was generated on (regions by bp, synth.c3_windows)
    blocks = plan_blocks([max(e - s, 0) for _, _, s, e in region_list(bed)], comm.world)
    geo = Geometry(refs, bed, blocks)
    held = to_owners(comm, geo, {comm.rank: rank_bam})
    t1 = time.time()
    keep = {}
    # the stage parts and side outputs live in one directory all ranks see (rank 0 joins parts there)
    shared = comm.broadcast_obj(tempfile.mkdtemp(prefix="ccbench_shared_") if comm.rank == 0 else None)
    try:
        sharded_pipeline(os.path.join(work, "sample.bam"), shared, bed, comm, eng, cutoff=cutoff, level=1,
                         blocks=blocks, held=held, refs=refs, keep=keep, finalize=False)
    finally:
        comm.barrier()
        if comm.rank == 0:
            shutil.rmtree(shared, ignore_errors=True)
    t2 = time.time()
    runs = [(k, keep[k][comm.rank]) for k in ("sscs", "dcs", "sc", "dcs_sc")]
    return runs, {"to_owners": t1 - t0, "stages": t2 - t1, "e2e": t2 - t0}


def stage_reduce(eng, comm, run):
    """A stage's one collective in the timed step: its stats counters summed over the ranks (RCCL
    through cc_reduce_stats, or gloo in a one-GPU rehearsal)."""
    import numpy as np
    g = run.g if hasattr(run, "g") else run.gs
    c = eng.counters(g)
    vec = np.array([c[k] for k in sorted(c)], np.int64)
    if comm.cc_comm is not None:
        eng.reduce_stats(comm.cc_comm, vec)
    else:
        comm._allreduce(vec, "sum")


def algorithmic_bytes(name, runs, L):
    """Algorithmic HBM bytes of ONE launch of `name`:
    votes read every voted base+qual once (L/2 + L per read) and write each
    consensus once; a radix sort of n (u64 key, u32 value) pairs must read and
    write them once (24 B per element); the other kernels stream their SoA
    fields once."""
    rd = L // 2 + L
    per = {}
    for tag, r in runs:
        eng = r.eng
        if tag == "sscs":
            g = r.g
            n = eng.fetch(g, "emit_n", np.int32)
            vs = eng.fetch(g, "emit_vslot", np.int32)
            nv_all = n[vs >= 0]
            small = nv_all <= 63      # VOTE_BIGN: larger families go to the split vote
            per.setdefault("k_sscs_vote_swar", []).append(int(nv_all[small].sum()) * (rd + 16)
                                                             + int(small.sum()) * (rd + 20))
            if (~small).any():
                # k_big_swar reads every member once; k_big_final writes the consensus (and reads the
                # items' 4 x L count planes, not algorithmic)
                per.setdefault("k_big_swar", []).append(int(nv_all[~small].sum()) * (rd + 16))
                per.setdefault("k_big_final", []).append(int((~small).sum()) * (rd + 20))
        if tag in ("dcs", "dcs_sc"):
            nv = int((eng.fetch(r.g, "dec", np.int32) == 0).sum())
            per.setdefault("k_duplex_vote_dcs", []).append(nv * (2 * rd + 16 + rd + 20))
        if tag == "sc":
            dec = eng.fetch(r.gs, "dec", np.int32)
            nv = int(((dec == 0) | (dec == 1)).sum())
            per.setdefault("k_duplex_vote_sc", []).append(nv * (2 * rd + 16 + rd + 20))
        # per-pass table preparation (k_build_meta: 28 B of SoA columns read, the 16-B member record
        # written; one launch per table)
        for rec in ([r.rec] if tag != "sc" else [r.srec, r.xrec]):
            per.setdefault("k_build_meta", []).append(rec.n * (28 + 16))
        groups = [r.g] if tag != "sc" else [r.gs, r.gx]
        for g in groups:
            c = eng.counters(g)
            S = r.n_input if tag != "sc" else (r.sstream.n if g == r.gs else r.xstream.n)
            per.setdefault("sort_qname", []).append(24 * S)
            per.setdefault("sort_tags", []).append(24 * c["READ_ENDS"])
            per.setdefault("sort_csn", []).append(24 * c["FAMILIES"])
            per.setdefault("k_classify", []).append(S * (4 + 4 + 2 + 1 + 8 + 2 + 24 + 8 + 4 + 1 + 4))
            per.setdefault("k_pair_keys", []).append(c["PAIRS"] * (8 + 2 * 40 + 48 + 8 + 12 + 2 * 44))
            # one-sided mate search: every stream entry reads skey, stream_rec, mtid, mpos, rkey (28 B);
            # each pair's searcher adds its bucket bounds (8), the candidate's rq (8), both cores'
            # qname fields (32), both qnames (2 x 24: ~19-char synthetic qnames in 8-B words), spos,
            # partner, claims (read+write) and mate_of (20)
            per.setdefault("k_pair_coord", []).append(S * 28 + c["PAIRS"] * (8 + 8 + 32 + 48 + 20))
            per.setdefault("k_fam_mark", []).append(c["READ_ENDS"] * (12 + 64 + 8 + 12))
    return {k: float(np.mean(v)) for k, v in per.items()}


# The engine's timing scopes (ProfScope in csrc/cc_engine.hip) that are not one kernel of the same
# name: the "k_pair_coord" scope is the whole coordinate pairing pass, "k_pair_resid" the residual
# keys' table and probe, and so on.  A scope's event time, its algorithmic bytes and its PMC traffic
# all cover these kernels together.  Kernels that run only on some passes (k_scatter_stream: bed
# streams; the residual kernels: passes with residual reads) are weighted by their launches.
SCOPE_KERNELS = {
    "k_pair_coord": ["k_scatter_stream", "k_pair_coord_tile", "k_pair_resid"],
    "k_pair_resid": ["k_resid_probe", "k_resid_probe_sorted"],
    "k_group": ["k_group_flags"],
    "k_fam_mark": ["k_fam_mark", "k_fam_dedup"],
    "k_csn": ["k_csn_mark", "k_csn_entries"],
    "k_duplex_vote_dcs": ["k_duplex_vote_swar"],
    "k_duplex_vote_sc": ["k_duplex_vote_swar"],
}


_WORKLOAD = {}


def _pmc_file():
    """profiles/pmc_latest.json holds the C2 passes; other configs' passes are pmc_<config>_latest.json."""
    c = _WORKLOAD.get("config", "c2")
    return "profiles/pmc_latest.json" if c == "c2" else "profiles/pmc_%s_latest.json" % c


def _pmc():
    """The committed PMC passes, if they were taken on this run's workload (same config, same reads)."""
    try:
        d = json.load(open(os.path.join(ROOT, _pmc_file())))
    except Exception:
        return None
    m = d.get("_meta", {})
    if _WORKLOAD and (m.get("workload") != _WORKLOAD.get("workload") or m.get("input_reads") != _WORKLOAD.get("n")):
        return None
    return d


def scope_traffic(d, scope, scope_launches_per_pass):
    """HBM bytes per launch of the timing scope `scope` from PMC passes `d` (pmc_traffic.py's JSON):
    the bytes of every kernel of the scope per pipeline pass (bytes per launch x launches / passes)
    over the scope's launches per pipeline pass.  None when no kernel of the scope was profiled."""
    passes = d["_meta"]["passes"]
    ks = [k for k in SCOPE_KERNELS.get(scope, [scope]) if k in d]
    if not ks or not scope_launches_per_pass:
        return None
    per_pass = sum(d[k]["traffic_bytes_per_launch"] * d[k]["launches"] / passes for k in ks)
    return per_pass / scope_launches_per_pass


def pmc_traffic(kernel, launches_per_step):
    """HBM bytes per launch of the scope `kernel` (its SCOPE_KERNELS, weighted by their launches) from
    the last rocprofv3 PMC passes (size-resolved read requests, or FETCH_SIZE x2, + WRITE_SIZE;
    scripts/pmc_traffic.py), committed as
    profiles/pmc_latest.json (pmc_<config>_latest.json for other configs); (None, None) without a
    PMC file for this workload or with no kernel of the scope in it."""
    d = _pmc()
    try:
        t = scope_traffic(d, kernel, launches_per_step)
        if t is None:
            return None, None
        return round(t, 1), _pmc_file() + " (rocprofv3 --pmc, same workload; kernels %s)" % ",".join(
            k for k in SCOPE_KERNELS.get(kernel, [kernel]) if k in d)
    except Exception:
        return None, None


# Kernels of cc_table_upload (the table's packed columns, built once per table in the setup, before
# the first pass): their bytes are not part of a step.
UPLOAD_KERNELS = ("k_qn_pack", "k_core_pack", "k_table_cols")


def step_traffic(d):
    """HBM bytes of one whole step from PMC passes `d` (pmc_traffic.py's JSON): every kernel's mean
    bytes per launch times its launches per pipeline pass (the PMC run's launches over its passes: the
    setup pass, the profiling steps and the timed steps each run every stage once), the upload
    kernels left out."""
    passes = d["_meta"]["passes"]
    return sum(v["traffic_bytes_per_launch"] * v["launches"] / passes
               for k, v in d.items() if not k.startswith("_") and k not in UPLOAD_KERNELS)


def pmc_step_traffic():
    d = _pmc()
    try:
        return round(step_traffic(d), 1)
    except Exception:
        return None


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(cfg_name, seed):
    """The C++ oracle (oracle/cpu_baseline.py) on bounded samples of the same model: one process on one
    core, then one process per core at once (independent samples, aggregate reads/s).  Runs before
    anything touches the GPU; its children are plain CPU processes.  Cores: this process's CPU
    affinity, bounded by the pool's per-job CPU share when one is set (OMP_NUM_THREADS: the GPU boxes
    give a one-GPU job 16 of the host's CPUs); both are reported."""
    pairs = int(os.environ.get("CC_CPU_SAMPLE_PAIRS", "250000"))
    affinity = len(os.sched_getaffinity(0))
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    cores = int(os.environ.get("CC_CPU_CORES", str(min(affinity, share) if share > 0 else affinity)))
    worker = [sys.executable, os.path.join(ROOT, "oracle", "cpu_baseline.py"), cfg_name, str(pairs)]
    env = dict(os.environ, OMP_NUM_THREADS="1", CC_ORACLE_THREADS="1")
    one = json.loads(subprocess.check_output(worker + [str(seed)], env=env).decode().strip().splitlines()[-1])
    procs = [subprocess.Popen(worker + [str(seed + 1 + i)], stdout=subprocess.PIPE, env=env) for i in range(cores)]
    many = [json.loads(pr.communicate()[0].decode().strip().splitlines()[-1]) for pr in procs]
    if any(pr.returncode for pr in procs):
        raise RuntimeError("cpu_baseline worker failed")
    agg = sum(m["reads"] for m in many) / max(m["consensus_s"] for m in many)
    out = dict(value=round(agg, 1), unit="reads/s", cores=cores, kind="port",
               cpu_model=_cpu_model(), affinity_cpus=affinity, cpu_share=share or None,
               single_core=round(one["reads"] / one["consensus_s"], 1),
               sample="oracle/cc_oracle.cpp (C++ restatement of the reference's dictionary program) on %d-read "
                      "samples of the %s model (%d pairs target each), consensus stages only (BAM decode/encode "
                      "and the sort/merge stand-in excluded, as in the GPU figure); value: %d concurrent processes, "
                      "one core each, on independent samples (%.1f s); single_core: one process (%.1f s)"
                      % (one["reads"], cfg_name, pairs, cores, max(m["consensus_s"] for m in many),
                         one["consensus_s"]))
    try:   # the reference itself, timed in the build container (it cannot travel to this box)
        ref = json.load(open(os.path.join(ROOT, "profiles", "r02_reference_cpu_c2_20kpairs.json")))
        out["reference_in_container"] = dict(
            value=ref["reference"]["reads_per_s"], unit="reads/s", cores=ref["cores"], kind="reference",
            sample="the unmodified reference stage scripts (pysam stand-in) on a %d-read c2 sample, one core, "
                   "timed in the build container (oracle/time_reference.py), not on this box" % ref["input_reads"],
            source="profiles/r02_reference_cpu_c2_20kpairs.json")
    except (OSError, KeyError, ValueError):
        pass
    return out


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default=None, help="c2 (default at 1 GPU), c3 (default at N > 1), c4, c5")
    ap.add_argument("--pairs", type=int, default=None, help="override the config's read-pair count (tests)")
    ap.add_argument("--cutoff", type=float, default=0.7)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--profile-steps", type=int, default=2, help="untimed steps for the per-kernel breakdown")
    args = ap.parse_args()
    args.profile_steps = max(1, args.profile_steps)

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one process per GPU: relaunch under torch.distributed.run as a child (nothing has touched
        # the GPU yet) and exit with its status
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
        sys.exit(subprocess.call(cmd))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world), file=sys.stderr)
        sys.exit(2)
    config = args.config or ("c2" if world == 1 else "c3")
    from consensuscruncher_amd import synth
    seed = synth.SEED_BASE + int(config[1:]) + 1000 * rank
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        t = time.time()
        cpu = cpu_baseline(config, seed + 17)
        log("cpu baseline in %.1fs: %s" % (time.time() - t, cpu))
    dist = None
    # rehearsal of the N-rank path on fewer GPUs (CC_BENCH_DEVICES=1: every rank on GPU 0, gloo for
    # the one reduction); the driver's multi-GPU runs leave it unset: rank k on GPU k, RCCL
    share = int(os.environ.get("CC_BENCH_DEVICES", "0"))
    device = local % share if share else local
    if world > 1:
        import torch
        import torch.distributed as dist
        backend = "gloo" if share or not torch.cuda.is_available() else "nccl"
        if backend == "nccl":
            torch.cuda.set_device(device)
        dist.init_process_group(backend)

    from consensuscruncher_amd.engine import Engine

    # C3 runs the multi-GPU driver at every N, N = 1 included (world 1: one block holding every
    # region), so that the 1/2/4/8-GPU points share code path and per-GPU workload
    sharded = world > 1 or config == "c3"
    cfg, bed = synth.config(config, world, rank)
    if sharded:
        # one sample over the ranks: 25 M pairs per GPU, translocated mates anywhere, region-straddling
        # pairs, disjoint qnames per rank
        cfg.update(n_pairs=C3_PAIRS_PER_GPU, mates_anywhere=True, straddle_frac=0.005, pair_offset=rank * 10 ** 9)
    if args.pairs:
        cfg["n_pairs"] = args.pairs
    work = tempfile.mkdtemp(prefix="ccbench_r%d_" % rank)
    comm = None
    try:
        t = time.time()
        batch = synth.generate(seed=seed, **cfg)
        L = batch.read_len
        log("generated %d reads in %.1fs" % (batch.n, time.time() - t))
        inp = os.path.join(work, "sample.bam")
        t = time.time()
        synth.write_bam_native(batch, inp, level=1)
        del batch
        log("wrote input BAM in %.1fs" % (time.time() - t))
        eng = Engine(device)
        if sharded:
            from consensuscruncher_amd.sharded import LocalComm, TorchComm
            comm = TorchComm(engine=eng) if world > 1 else LocalComm(1)
            runs, setup_t = build_sharded(eng, comm, work, inp, args.cutoff, bed)
            n_in = int((runs[0][1].stream.region >= 0).sum())   # own entries (foreign ends: another rank's)
        else:
            runs, setup_t = build_stages(eng, work, inp, args.cutoff, bed)
            n_in = runs[0][1].n_input
        log("setup (end-to-end product path) %.1fs: %s" % (setup_t["e2e"], setup_t))

        def step(i, reduce=True):
            # the stage calls of one step on resident groups run with their end-of-pass checks
            # deferred to one wait at the end of the step (Engine.deferred: exact replay when a
            # planned pass did not hold); then each stage's stats reduction over the ranks
            def calls():
                for _, r in runs:
                    r.step(0x5eed + 7919 * i)
            eng.deferred(calls)
            if comm is not None and world > 1 and reduce:
                for _, r in runs:
                    stage_reduce(eng, comm, r)

        def barrier():
            eng.synchronize()
            if dist is not None:
                import torch
                dist.barrier()
                if torch.cuda.is_available():
                    torch.cuda.synchronize()

        for i in range(args.warmup):
            step(i)
        barrier()
        # per-kernel breakdown: untimed steps with HIP events around every kernel scope (the events
        # add launch gaps, so these steps are not the timed ones)
        eng.set_profiling(True)
        # a rehearsal with several ranks on one GPU (CC_BENCH_DEVICES) profiles the ranks one after
        # another, so each rank's per-kernel times are its own and not shared with the other ranks'
        serial = bool(share) and world > 1
        for i in range(args.profile_steps):
            if serial:
                for k in range(world):
                    barrier()
                    if rank == k:
                        step(500 + i, reduce=False)
                        eng.synchronize()
                barrier()
            else:
                step(500 + i)
        eng.synchronize()
        ktimes = eng.kernel_times()
        eng.set_profiling(False)
        dom_name = max(ktimes.items(), key=lambda kv: kv[1][0])[0] if ktimes else None
        # the timed region: events only around the dominant kernel (its live launch duration)
        eng.profile_only([dom_name] if dom_name else [])
        eng.set_profiling(True)
        barrier()
        l0 = eng.launch_count()
        t0 = time.perf_counter()
        for i in range(args.steps):
            step(1000 + i)
        barrier()
        elapsed = time.perf_counter() - t0
        launches = (eng.launch_count() - l0) / float(args.steps)
        dtimes = eng.kernel_times()
        eng.set_profiling(False)
        eng.profile_only([])

        total_in, max_el = float(n_in), elapsed
        if dist is not None:
            # the single stats reduction (RCCL over xGMI): summed input reads, max step time
            from consensuscruncher_amd.shard import allreduce_stats
            sums, max_el = allreduce_stats({"input_reads": n_in}, elapsed)
            total_in = sums["input_reads"]
        ms_per_step = 1000.0 * max_el / args.steps
        value = total_in / (max_el / args.steps)

        _WORKLOAD.update(config=config, n=n_in, workload=("%s: SSCS+DCS+SC+DCS-SC consensus, %s, cutoff %.2f" % (
            config, "-b False" if bed is None else (
                "one hg38 sample over %d GPUs (hg38_cytoBand.txt region blocks, %d pairs per GPU, weak scaling)"
                % (world, cfg["n_pairs"]) if sharded else "hg38_cytoBand.txt regions"), args.cutoff)))
        # SURVEY.md §8(d), the headline: sum over the stages of B_s = N_in (L/2 + L + 16) + N_out (L/2 + L)
        # per step, over the honest step time (every kernel of every stage, table preparation
        # included, plus launch gaps and the end-of-pass readbacks)
        pipe_bytes = 0.0
        for tag, r in runs:
            if tag == "sc":
                n_out = int((eng.fetch(r.gs, "dec", np.int32) < 2).sum())
            else:
                n_out = len(eng.fetch(r.g, "emit_n" if tag == "sscs" else "dec", np.int32))
            pipe_bytes += r.n_input * (L // 2 + L + 16) + n_out * (L // 2 + L)
        step_s = max_el / args.steps
        pipe_ach = pipe_bytes / step_s / 1e9
        # secondary: the dominant kernel (HIP events on the engine's stream over the timed region)
        alg = algorithmic_bytes(None, runs, L)
        if dom_name is None:   # --profile-steps 0: the timed region's own scopes name it
            dom_name = max(dtimes.items(), key=lambda kv: kv[1][0])[0] if dtimes else None
        dom_ms, dom_n = dtimes.get(dom_name, (0.0, 0))
        avg_s = dom_ms / 1000.0 / max(dom_n, 1)
        bytes_per_launch = alg.get(dom_name)
        achieved = (bytes_per_launch / avg_s / 1e9) if bytes_per_launch else None
        traffic, traffic_src = pmc_traffic(dom_name, dom_n / float(args.steps))
        kernel_s = sum(v[0] for v in ktimes.values()) / 1000.0 / max(args.profile_steps, 1)
        out = {
            "metric": "input reads/sec through SSCS+DCS+SC consensus",
            "value": round(value, 1),
            "unit": "reads/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "launches_per_step": round(launches, 1),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (seeded %s model: %d input reads per rank, 2x%d bp, NNT UMIs)" % (
                config, n_in, L),
            "config": {"workload": _WORKLOAD["workload"],
                "input_reads_per_rank": n_in, "read_len": L,
                "pairs_per_gpu": cfg["n_pairs"],
                "parallelism": ("cytoband-block shards x%d (sharded.py: rank-local records, foreign first mates "
                                "routed, one RCCL stats reduction per stage)" % world) if sharded else
                               ("cytoband regions, one GPU" if bed else "single GPU, -b False")},
            "roofline": {"bound": "hbm", "scope": "pipeline: every stage of one step (SURVEY.md 8d)",
                         "achieved": round(pipe_ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(pipe_ach / HBM_PEAK_GBS, 4), "traffic": pmc_step_traffic(),
                         "traffic_source": _pmc_file() + ": all kernels but the upload's, bytes per step; reads: "
                         + str((_pmc() or {}).get("_meta", {}).get("reads", "FETCH_SIZE x2")),
                         "alg_bytes_per_step": pipe_bytes, "step_ms": round(step_s * 1000, 3),
                         "per_unit": "%d B per input read + %d B per emitted record" % (
                             L // 2 + L + 16, L // 2 + L)},
            "dominant_kernel": {"kernel": dom_name, "scope_kernels": SCOPE_KERNELS.get(dom_name, [dom_name]),
                                "achieved": round(achieved, 1) if achieved else None, "peak": HBM_PEAK_GBS,
                                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                                "traffic": traffic, "traffic_source": traffic_src,
                                "avg_launch_us": round(avg_s * 1e6, 2), "alg_bytes_per_launch": bytes_per_launch},
            "device_ms_per_step": round(kernel_s * 1000, 3),
            "kernels_ms_per_step": {k: round(v[0] / args.profile_steps, 4) for k, v in
                                    sorted(ktimes.items(), key=lambda kv: -kv[1][0])},
            "end_to_end": {"setup_s": round(setup_t["e2e"], 2),
                           "reads_per_s": round(n_in / setup_t["e2e"], 1),
                           "breakdown_s": {k: v for k, v in setup_t.items() if k != "e2e"},
                           "note": "decode+upload+GPU+encode+sort+merge, one pass, per rank"},
            "cpu_baseline": cpu,
        }
        if rank == 0:
            print(json.dumps(out), flush=True)
        for _, r in runs:
            r.close()
        if comm is not None:
            comm.close()
        eng.close()
    finally:
        shutil.rmtree(work, ignore_errors=True)
        if dist is not None:
            dist.destroy_process_group()


if __name__ == "__main__":
    main()
