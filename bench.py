"""bench.py -- pods scheduled/s + node-evaluations/s for the FGD replay of the
Alibaba openb trace on MI355X (BASELINE.json metric; configs[1] = C2).

Workload (one "step"): the C2 job -- openb GPU nodes (1213) x openb_pod_list_default,
FGD (gpuSelMethod FGD), tune 1.3, shuffled, seeds 42..51 -> 10 independent
simulated clusters replayed to completion on the device.  Per GPU the work is
fixed (rank k replays seeds 42+10k .. 51+10k): weak scaling, replicas only, no
collective on the data path.

One JSON line on rank 0.  Extra keys: node_evals_per_s, roofline (dominant
kernel: k_memo for FGD -- one persistent launch replays every replica with the
(pod class, node) keys memoised -- else k_replay; priced against HBM with SURVEY
§8(d)'s 32 B per node-evaluation + 56 B per pod), and cpu_baseline (the C oracle
-- a restatement of the Go path -- on the host cores).

Multi-GPU (torchrun, one rank per GPU): each rank replays its own seeds on its own
GPU; the only collectives are the timing barrier and the job reduction (max time,
summed events) -- see seeds_for_rank / reduce_job, tested with gloo on CPU.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-scheduler-simulator_amd"))

import ksim  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E peak 8.0 TB/s (spec)
BYTES_PER_NODE_EVAL = 32
BYTES_PER_POD = 56        # 16 B request + 8 B winner + 32 B scatter
# Counter passes of each bench configuration (scripts/profile_config.sh NAME ...): HBM bytes per
# dispatch of the dominant kernel (FETCH_SIZE x2 + WRITE_SIZE; MI355X_MICROARCH.md HBM section) and its
# VALU issue (SQ_INSTS_VALU with the fp64 split).  profiles/<round>/prof/<profile_key(args)>/pmc.json, the
# newest round that profiled the configuration first.
PROF_DIRS = [os.path.join(ROOT, "profiles", r, "prof") for r in ("r06", "r05", "r04", "r03", "r02")]
PROF_DIR = PROF_DIRS[0]
# MI355X_MICROARCH.md, persistent-kernel price list: handoff-1to1 = one producer -> one consumer
# granule hand-off between CUs, idle chip, 8 B: 0.8 us.  A pod step whose decision crosses CUs
# (k_memo, wide k_hmemo, k_replay at K > 1) pays at least one.
HANDOFF_FLOOR_US = 0.8


def profile_key(args):
    """The profiles/r02/prof/ directory of a bench configuration (scripts/profile_all.sh uses these names)."""
    k = args.config
    if args.policy != "FGD":
        k += "-" + args.policy.replace(" ", "_")
    if args.run_mode:
        k += "-rm%d" % args.run_mode
    if args.report and args.config != "c4":
        k += "-report"
    if args.sharded:
        k += "-sharded"
    if getattr(args, "random_stream", "hash") == "go":
        k += "-go"
    if getattr(args, "rank_share", ""):
        k += "-share%s" % args.rank_share.replace("/", "of")  # a share's own launches (no profile: traffic null)
    return k


def profile_file(key):
    """The newest round's counter summary of a bench configuration (PROF_DIRS order), or None."""
    return next((f for f in (os.path.join(d, key, "pmc.json") for d in PROF_DIRS) if os.path.exists(f)), None)


def profile_rooflines(args, kernels):
    """(traffic, traffic_source, valu) from this configuration's counter passes, if it was profiled and
    the profiled dominant kernel is one this run launched (`kernels`: Engine.last_run_kernels())."""
    pf = profile_file(profile_key(args))
    if pf is None:
        return None, None, None
    with open(pf) as f:
        pmc = json.load(f)
    dom = pmc.get("dominant") or {}
    fam = dom.get("kernel", "")  # scripts/pmc_summary.py kernel_of: k_memo, k_hmemo, k_scan1_mix, k_replay<1>, ...
    names = {{"k_hmemo_wide": "k_hmemo", "k_memo_hkeys": "k_memo"}.get(k, k) for k in kernels}
    if fam.split("<")[0] not in names:
        return None, None, None
    src = os.path.relpath(pf, ROOT)
    valu = None
    if dom.get("valu_insts_per_dispatch"):
        valu = {"bound": "valu", "kernel": dom["kernel"], "achieved": dom["valu_insts_per_s"],
                "peak": dom["valu_peak_insts_per_s"], "unit": "wave-instr/s", "frac": dom["valu_frac"],
                "insts_per_dispatch": dom["valu_insts_per_dispatch"], "f64_share": dom.get("f64_share"),
                "f64_frac": dom.get("f64_frac"), "nonf64_frac": dom.get("nonf64_frac"),
                "profiled_ms": dom["mean_duration_ns"] / 1e6, "source": src,
                "note": "rate over the profiled dispatch; peak = 256 CUs x 4 SIMDs x clock / 2 cycles per wave64 "
                        "instruction (SIMD-32), fp64 add/mul/FMA at 4 cycles (f64_frac + nonf64_frac = issue-slot share)"}
    traffic = dom.get("hbm_bytes_per_dispatch")
    return traffic, src, valu


def cpu_baseline(trace, seed, threads):
    """Oracle ("port") on the host: one full seed replay (~11k events), FGD, `threads` workers."""
    os.environ["KSIM_ORACLE_CACHE"] = "0"  # every timed replay runs (pyoracle memoises replays for the tests)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import helpers
    import pyoracle as O
    rp = trace.replay(seed=seed, tune_ratio=1.3, shuffle=True)
    nodes = helpers.oracle_nodes(trace, rp)
    ev = helpers.oracle_events(trace, rp)
    tp = helpers.oracle_typical(trace)
    t0 = time.perf_counter()
    O.run_events(nodes, tp, ev, policy=O.POL_FGD, gpu_sel=O.SEL_FGD, threads=threads)
    dt = time.perf_counter() - t0
    # one thread too, on a bounded prefix of the same stream (the first 1500 events)
    nodes1 = helpers.oracle_nodes(trace, rp)
    t1 = time.perf_counter()
    O.run_events(nodes1, tp, ev[:1500], policy=O.POL_FGD, gpu_sel=O.SEL_FGD, threads=1)
    one = 1500 / (time.perf_counter() - t1)
    return dict(value=len(ev) / dt, unit="pods/s", cores=threads, kind="port",
                node_evals_per_s=len(ev) * trace.num_nodes / dt,
                single_thread={"value": one, "unit": "pods/s", "cores": 1,
                               "sample": "the first 1500 events of the same stream"},
                sample="openb default, seed %d, full replay (%d events x %d nodes), FGD, %d worker threads "
                       "(parallelize.Until fan-out); host nproc=%d, cpu %s" % (seed, len(ev), trace.num_nodes, threads,
                                                                               os.cpu_count(), cpu_model()))


def _c2_worker(seed):
    """One C2 replica on the oracle, single-threaded, replayed to completion (cpu_baseline_replicas)."""
    os.environ["KSIM_ORACLE_CACHE"] = "0"
    sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
    import helpers
    import pyoracle as O
    t = ksim.Trace.openb("default")
    rp = t.replay(seed=seed, tune_ratio=1.3, shuffle=True)
    nodes, tp, ev = helpers.oracle_nodes(t, rp), helpers.oracle_typical(t), helpers.oracle_events(t, rp)
    t0 = time.perf_counter()
    O.run_events(nodes, tp, ev, policy=O.POL_FGD, gpu_sel=O.SEL_FGD, threads=1)
    return len(ev), time.perf_counter() - t0


def cpu_baseline_replicas(seeds):
    """SURVEY §8(d)(iii) for C2, like for like with the GPU line: the same seeds as independent
    single-threaded oracle processes, one core each (the reference runs replicas as separate simon
    processes), every replica replayed to completion."""
    import concurrent.futures as cf
    import multiprocessing as mp
    t0 = time.perf_counter()
    with cf.ProcessPoolExecutor(max_workers=len(seeds), mp_context=mp.get_context("spawn")) as ex:
        out = list(ex.map(_c2_worker, seeds))
    wall = time.perf_counter() - t0
    events = sum(o[0] for o in out)
    slowest = max(o[1] for o in out)
    return dict(value=events / slowest, unit="pods/s", cores=len(seeds), kind="port", wall_s=wall,
                sample="the bench's %d seeds (openb default, FGD, tune 1.3) replayed to completion (%d events) as %d "
                       "single-threaded oracle processes, one core each; value = events / the slowest replica's "
                       "replay time (process start-up and trace loads excluded); host nproc=%d, cpu %s"
                       % (len(seeds), events, len(seeds), os.cpu_count(), cpu_model()))


# paper-sweep policy directories -> the oracle's (policy, gpu selection) (tests/test_gpu_parity.py)
ORACLE_POLICY = {"01-Random": ("POL_RANDOM", "SEL_RANDOM"), "02-DotProd": ("POL_DOTPROD", "SEL_BEST"),
                 "03-GpuClustering": ("POL_CLUSTERING", "SEL_BEST"), "04-GpuPacking": ("POL_PACKING", "SEL_BEST"),
                 "05-BestFit": ("POL_BESTFIT", "SEL_BEST"), "06-FGD": ("POL_FGD", "SEL_FGD")}


def _c4_worker(job):
    """One paper-sweep experiment on the oracle, single-threaded, over its first `prefix` events."""
    os.environ["KSIM_ORACLE_CACHE"] = "0"
    sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
    import helpers
    import pyoracle as O
    trace_name, policy, seed, prefix = job
    t = ksim.Trace.openb(trace_name[len("openb_pod_list_"):])
    rp = t.replay(seed=seed, tune_ratio=1.3, shuffle=True)
    pol, sel = ORACLE_POLICY[policy]
    nodes, tp = helpers.oracle_nodes(t, rp), helpers.oracle_typical(t)
    ev = helpers.oracle_events(t, rp, prefix)
    t0 = time.perf_counter()
    O.run_events(nodes, tp, ev, policy=getattr(O, pol), gpu_sel=getattr(O, sel), seed=seed, threads=1)
    return len(ev), time.perf_counter() - t0, rp.n


def cpu_baseline_sweep(workers=16, per_worker=2, prefix=None):
    """SURVEY §8(d)(iii) for C4: the oracle as independent single-threaded experiments on `workers` host
    cores (the reference runs its sweep as parallel processes, one experiment each), on a bounded sample:
    workers x per_worker whole experiments (or their first `prefix` events) spread over the paper sweep's
    policies and traces.  Spawned before this process touches the GPU."""
    import concurrent.futures as cf
    import multiprocessing as mp
    import ksim.sweep as SW
    exps = SW.plan()
    step = max(1, len(exps) // (workers * per_worker))
    jobs = [(e[0], e[1], e[2], prefix) for e in exps[::step][:workers * per_worker]]
    t0 = time.perf_counter()
    with cf.ProcessPoolExecutor(max_workers=workers, mp_context=mp.get_context("spawn")) as ex:
        out = list(ex.map(_c4_worker, jobs))
    wall = time.perf_counter() - t0
    events = sum(o[0] for o in out)
    busy = sum(o[1] for o in out)
    full = sum(o[2] for o in out) / len(out)
    pods_s = events / busy * workers  # per-worker rate x workers (process start-up and trace loads excluded)
    return dict(value=pods_s, unit="pods/s", cores=workers, kind="port", experiments_per_s=pods_s / full,
                wall_s=wall,
                sample="%d of the 1020 paper-sweep experiments (every %dth: all 6 policies, 17 traces), %s, the oracle single-threaded in %d worker processes (SURVEY §8(d)(iii)); "
                       "experiments/s = pods/s / %.0f events per full experiment; host nproc=%d, cpu %s"
                       % (len(jobs), step, "the first %d events of each" % prefix if prefix else "replayed to completion", workers, full, os.cpu_count(), cpu_model()))


def cpu_baseline_c5(trace, rp, threads, prefix=400):
    """C5's CPU baseline: the oracle's FGD cycle over the 100 000-node cluster with `threads` workers per cycle
    (parallelize.Until's fan-out, generic_scheduler.go:274-346), on the first `prefix` events of the bench's own
    1M-event stream (a full replay would take days on the host)."""
    os.environ["KSIM_ORACLE_CACHE"] = "0"
    sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
    import helpers
    import pyoracle as O
    nodes, tp = helpers.oracle_nodes(trace, rp), helpers.oracle_typical(trace)
    ev = helpers.oracle_events(trace, rp, prefix)
    t0 = time.perf_counter()
    O.run_events(nodes, tp, ev, policy=O.POL_FGD, gpu_sel=O.SEL_FGD, threads=threads)
    dt = time.perf_counter() - t0
    return dict(value=len(ev) / dt, unit="pods/s", cores=threads, kind="port",
                node_evals_per_s=len(ev) * trace.num_nodes / dt,
                sample="C5's own stream (synthetic 100000 nodes, seed 1 draw), its first %d events, FGD, %d worker "
                       "threads per cycle (parallelize.Until fan-out); host nproc=%d, cpu %s"
                       % (len(ev), threads, os.cpu_count(), cpu_model()))


def cpu_model():
    """Host CPU model name (SURVEY §8(d) asks for it beside the thread count)."""
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def latency_block(kern_us, steps, wgs):
    """Per pod step of one replica: the dominant launch's duration over the steps it replays (replicas run
    concurrently, so this is the dependent-chain latency of one step), beside the measured floor of a
    cross-CU hand-off when a step's decision crosses CUs (wgs > 1)."""
    us = kern_us / steps if steps else None
    out = {"bound": "latency", "us_per_pod_step": us, "steps_per_launch": steps}
    if wgs and wgs > 1 and us:
        out.update(floor_us=HANDOFF_FLOOR_US, frac=HANDOFF_FLOOR_US / us,
                   floor="MI355X_MICROARCH.md handoff-1to1 (idle, 8 B): one cross-CU granule hand-off per pod step")
    return out


def seeds_for_rank(rank, replicas, base=42):
    """C2 seeds of one rank: rank k replays base + replicas*k .. base + replicas*(k+1) - 1."""
    return [base + replicas * rank + i for i in range(replicas)]


def reduce_job(dt, events, dist=None, device="cpu"):
    """Whole-job time (max over ranks) and events (sum over ranks)."""
    if dist is None:
        return dt, events
    import torch
    t = torch.tensor([dt], device=device, dtype=torch.float64)
    n = torch.tensor([events], device=device, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.all_reduce(n, op=dist.ReduceOp.SUM)
    return float(t.item()), int(n.item())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--replicas", type=int, default=10, help="seeds per GPU (C2: 10)")
    ap.add_argument("--nodes-per-block", type=int, default=0)
    ap.add_argument("--wgs", type=int, default=0, help="workgroups per replica (0 = auto)")
    ap.add_argument("--run-mode", type=int, default=0,
                    help="0 auto (FGD: k_memo), 1 k_step per pod, 2 k_replay only, 3 k_memo required")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--policy", default="FGD", help="FGD (headline) | BestFit | DotProd | GpuPacking | GpuClustering | Random | PWR | "
                         "'PWR 500 FGD 500' ...")
    ap.add_argument("--config", default="c2", choices=["c2", "c4", "c5"],
                    help="c2: openb x 10 seeds per GPU (headline); c4: the paper sweep, 17 traces x 6 policies "
                         "x 10 seeds split over the GPUs; c5: synthetic 100k nodes x 1M pods, one replica per GPU")
    ap.add_argument("--report", action="store_true", help="also compute the per-event cluster report")
    ap.add_argument("--sharded", action="store_true",
                    help="c5 only: ONE cluster node-sharded over the ranks (RCCL exchange per pod; strong "
                         "scaling) instead of one replica per rank")
    ap.add_argument("--rank-share", default="",
                    help="c4 only, 'k/N': time rank k's share of a world-N split of the sweep on this one GPU (the "
                         "1-GPU rehearsal of the N-GPU strong-scaling run: the max over k predicts its time)")
    ap.add_argument("--no-widen", action="store_true",
                    help="c4: every replica at one workgroup (no k_memo for a share's longest FGD chains)")
    ap.add_argument("--random-stream", default="hash", choices=["hash", "go"],
                    help="Random policy: the hash contract (default) or the reference's draw structure on Go's "
                         "math/rand stream (k_random_go)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # C4's CPU baseline first: its worker processes are spawned before anything here touches the GPU
    sweep_cpu = None
    if args.config == "c4" and rank == 0 and world == 1 and not args.no_cpu_baseline:
        sweep_cpu = cpu_baseline_sweep(workers=args.cpu_threads)
    # world 1 never imports torch: the process holds the one HIP runtime ksim binds (a profiler's, under
    # rocprofv3), and the engine's own run() synchronises and times the launch.  World > 1: torch.distributed
    # for the timing barrier and the job reduction only (no collective on the data path)
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        ndev = torch.cuda.device_count()  # (counting devices does not initialise the GPU)
        if ndev < world:
            # ranks sharing a device (a box with fewer GPUs than ranks rehearsing the N-GPU run, replicas or the
            # multi-process sharded mode): the launcher's own barrier / reductions go over gloo (RCCL refuses two
            # ranks on one device); the data path has no collective either way
            print("bench: %d ranks on %d device(s): ranks share devices, gloo for the barrier" % (world, ndev),
                  file=sys.stderr)
            local = local % max(ndev, 1)
            torch.cuda.set_device(local)
            dist.init_process_group("gloo")
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl")

    trace = ksim.Trace.openb("default")
    c5_rp = None
    if args.config == "c4":
        import ksim.sweep as SW
        items = SW.plan()
        share_k, share_n = rank, world
        if args.rank_share:
            share_k, share_n = (int(x) for x in args.rank_share.split("/"))
            assert world == 1 and 0 <= share_k < share_n, "--rank-share k/N runs one share on one GPU"
        # longest-processing-time split by the cost model (ksim.sweep.plan_costs): the long FGD replays spread
        # over the ranks, the totals balance
        exps = SW.shard(items, share_k, share_n, SW.plan_costs(items) if share_n > 1 else None)
        # one workgroup per replica unless asked: every policy group then runs concurrently (FGD on k_hmemo, the
        # cheap policies as one k_scan1_mix launch) whatever the share's size -- a share small enough for k_memo
        # or k_replay at K > 1 would run its groups back to back (profiles/r05/c4_shares/).  The share's longest
        # FGD chains take k_memo at 12-32 workgroups each on the CUs the share leaves free (SW.plan_widths)
        wide = {} if args.no_widen else SW.plan_widths(exps, SW.plan_costs(exps), SW.plan_wide_costs(exps))
        sweep = SW.Sweep(exps, device=local, report=True, wgs=args.wgs or 1, random_stream=args.random_stream,
                         wide=wide)
        eng = sweep.eng
        eng.total_events = sweep.total_events
        eng.memo_replicas = sweep.fgd_replicas()
        args.replicas = len(exps)
    elif args.config == "c5" and args.sharded:
        # one 100k-node cluster split by name rank over the ranks; every rank replays the same 1M events
        trace = trace.synthetic(100_000, 1_000_000, seed=0)
        args.replicas = 1
        eng = _sharded_engine(local, rank, world, trace, dist)
    elif args.config == "c5":
        # nodes i.i.d. from the openb node specs (seed 0), 1M pods i.i.d. from the
        # default-trace rows; rank k replays its own draw (seed 2k+1), no tuning, trace order
        trace = trace.synthetic(100_000, 1_000_000, seed=0)
        args.replicas = 1
        seeds = [2 * rank + 1]
        eng = _engine_on(local, trace, seeds, args.nodes_per_block, args.policy, args.wgs, args.run_mode,
                         tune=0.0, shuffle=False, report=args.report, random_stream=args.random_stream)
        c5_rp = trace.replay(seed=seeds[0], tune_ratio=0.0, shuffle=False)
    else:
        seeds = seeds_for_rank(rank, args.replicas)
        eng = _engine_on(local, trace, seeds, args.nodes_per_block, args.policy, args.wgs, args.run_mode,
                         report=args.report, random_stream=args.random_stream)
    total_events = eng.total_events

    for _ in range(args.warmup):
        eng.run()

    def barrier():
        # eng.run() returns after its stream synchronised, so the device is idle here
        if dist is not None:
            dist.barrier()

    barrier()
    t0 = time.perf_counter()
    dev_ms = 0.0
    for _ in range(args.steps):
        dev_ms += eng.run()
    barrier()
    dt = time.perf_counter() - t0
    dt, job_events = reduce_job(dt, total_events * args.steps, dist,
                                "cpu" if dist is not None and dist.get_backend() == "gloo" else "cuda")
    if args.sharded:
        job_events = total_events * args.steps  # one cluster: every rank processed the same events

    steps_per_run = eng.last_run_steps()
    kernel = eng.last_run_path()
    kernels = eng.last_run_kernels()  # what the run launched, in launch order
    gate, gate_timeouts = eng.last_run_gate()
    # roofline: the dominant kernel (k_memo / k_replay) is one launch per replay of all replicas; its
    # duration is the hipEvent pair around the launch on the engine stream (mean over the timed runs)
    kern_us = dev_ms / args.steps * 1000.0
    bytes_per_launch = total_events * (BYTES_PER_NODE_EVAL * trace.num_nodes + BYTES_PER_POD)
    achieved = bytes_per_launch / (kern_us * 1e-6) / 1e9

    value = job_events / dt
    # HBM traffic and the VALU issue fraction (FGD is fp64 VALU work) of the dominant kernel
    # from this configuration's counter passes (scripts/profile_config.sh -> profiles/r02/prof/)
    traffic, traffic_src, valu = profile_rooflines(args, kernels)
    # executed work (the memoised paths skip most node evaluations): feasible (pod, node) score evaluations
    # of the reference's Score phase, and the (class, node) keys the memoised FGD replicas recomputed
    score_evals, key_refreshes = eng.work(getattr(eng, "memo_replicas", None))
    # pods scheduled/s counts every pod event, failed ones included; report the failures
    failed = 0
    for r in range(eng.R):
        st = eng.results_array(r)["status"]
        failed += int(((st == ksim.UNSCHEDULABLE) | (st == ksim.ERROR)).sum())
    line = {
        "metric": "pods scheduled/sec + node-score evals/sec (FGD, openb trace) at 1/2/4/8 MI355X",
        "value": value,
        "unit": "pods/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt * 1000.0 / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32+f64",
        "data": "Alibaba openb trace (data/openb, from the reference's data/csv), the reference's own event order (Go math/rand replay)",
        "config": {"workload": "C2: openb 1213 GPU nodes x openb_pod_list_default, FGD, tune 1.3, shuffled, "
                               "%d seeds per GPU replayed to completion" % args.replicas,
                   "replicas_per_gpu": args.replicas, "events_per_gpu": total_events,
                   "parallelism": "replicas%d" % world},
        "node_evals_per_s": value * trace.num_nodes,
        "failed_pods_per_step": failed * (1 if args.sharded else world),
        "score_evals_per_s": score_evals * args.steps * world / dt,
        "key_refreshes_per_s": key_refreshes * args.steps * world / dt if "memo" in kernel else None,
        "device_ms_per_step": dev_ms / args.steps,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                     # what the counters saw the kernel move, as a fraction of peak over the same time
                     "traffic_frac": (traffic / (kern_us * 1e-6) / (HBM_PEAK_GBS * 1e9)) if traffic else None,
                     "kernel": "+".join(kernels), "path": kernel, "kernel_us": kern_us,
                     "bytes_per_launch": bytes_per_launch, "wgs_per_replica": eng.last_run_wgs()},
        # the bound that binds: every replica is a chain of dependent pod steps
        "latency": latency_block(kern_us, steps_per_run, eng.last_run_wgs()),
        "valu_roofline": valu,
    }
    if gate:
        line["residency_gate"] = {"opened": gate == 1, "timeouts": gate_timeouts}
    if args.config == "c4":
        # SURVEY's 32 B per node-evaluation prices node reads the LDS / VGPR-resident kernels never make (the
        # counters' traffic is ~0.2 % of it): the byte roofline is nominal here, the latency block binds
        line["roofline"]["nominal"] = True
        line["data"] = "Alibaba openb traces (data/openb: 17 pod lists), the reference's own event order (Go math/rand replay)"
        line["config"] = {"workload": "C4: paper sweep, 17 traces x 6 policies x seeds 42-51, tune 1.3, "
                                      "per-event cluster report", "replicas_per_gpu": args.replicas,
                          "events_per_gpu": total_events, "parallelism": "replicas%d" % world}
        # whole job: every rank's experiments per timed step (the reference: 1020 in ~10 h on 256 vCPU)
        line["experiments_per_s"] = args.replicas * world / (dt / args.steps)
        line["config"]["widened_fgd"] = len(wide)  # FGD replays on k_memo at several workgroups (plan_widths)
        line["config"]["wide_k"] = {str(k): sum(1 for v in wide.values() if v == k) for k in sorted(set(wide.values()))}
        if args.rank_share:
            line["config"]["rank_share"] = args.rank_share
            line["config"]["workload"] += " -- rank %s's share of the LPT split only (%d experiments)" % (
                args.rank_share, args.replicas)
    if args.config == "c5" and args.sharded:
        line["scaling"] = "strong"
        line["config"] = {"workload": "C5: synthetic 100000 nodes x 1000000 pods, FGD, ONE cluster node-sharded "
                                      "over %d shard process(es), k_hmemo slices with a device-to-device granule "
                                      "exchange per pod (IPC-mapped buffers, no collective)" % world,
                          "replicas_per_gpu": 1, "events_per_gpu": total_events,
                          "parallelism": "nodeshard%d" % world}
        line["data"] = "synthetic (SURVEY §8(d) C5): nodes and pods drawn i.i.d. from the openb default trace"
    elif args.config == "c5":
        line["data"] = "synthetic (SURVEY §8(d) C5): nodes and pods drawn i.i.d. from the openb default trace"
        line["config"] = {"workload": "C5: synthetic 100000 nodes x 1000000 pods, FGD, one replica per GPU",
                          "replicas_per_gpu": 1, "events_per_gpu": total_events, "parallelism": "replicas%d" % world}
    if args.policy != "FGD":
        line["config"]["workload"] = line["config"]["workload"].replace("FGD", args.policy)
    if args.report:
        line["config"]["report"] = True
    if args.random_stream == "go":
        line["config"]["random_stream"] = "go"  # Random replicas on Go's math/rand draw structure
        # the draws are the reference's; the feasible list they index is taken in node order (one filter
        # worker), while the reference's 16 workers order it by timing: a contract, not reference-equal
        line["config"]["parity"] = "unpinned (node-order contract, DESIGN.md §4)"
    if args.config == "c4" or args.report:
        line["report_ms_per_step"] = eng.last_report_ms()
    line["build_id"] = ksim.build_id()  # sha256 prefix of the library's sources (ksim.source_hash())
    line["hip_runtime"] = ksim.hip_runtimes()  # one HIP / HSA runtime per process
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.config == "c2":
        # like for like: the GPU line's seeds as single-threaded replicas on as many cores; beside it one
        # replica with `cpu_threads` workers per cycle (parallelize.Until) and one thread on a prefix
        one = cpu_baseline(trace, seeds[0], args.cpu_threads)
        line["cpu_baseline"] = cpu_baseline_replicas(seeds)
        line["cpu_baseline"]["one_replica_threaded"] = {k: one[k] for k in ("value", "unit", "cores", "sample")}
        line["cpu_baseline"]["single_thread"] = one["single_thread"]
    if sweep_cpu is not None:
        line["cpu_baseline"] = sweep_cpu
    if rank == 0 and world == 1 and not args.no_cpu_baseline and c5_rp is not None and args.policy == "FGD":
        line["cpu_baseline"] = cpu_baseline_c5(trace, c5_rp, args.cpu_threads)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if os.environ.get("KSIM_MAPS_OUT"):  # the process's mappings, to symbolise an exit-path fault
        with open("/proc/self/maps") as f, open(os.environ["KSIM_MAPS_OUT"], "w") as g:
            g.write(f.read())
    eng.close()
    if dist is not None:
        dist.destroy_process_group()
    elif os.environ.get("KSIM_DEVICE_RESET") == "1":
        ksim.device_reset()  # world 1 holds no torch state: release the device before the exit handlers run


def _sharded_engine(device, rank, world, trace, dist):
    """This rank's shard of the one C5 cluster (ksim.shard): FGD shards exchange each pod step's slice maxima
    device to device through IPC-mapped buffers (ksim_engine_set_shard_peers; the handles go over `dist`)."""
    import ksim.shard as SH
    rp = trace.replay(seed=1, tune_ratio=0.0, shuffle=False)
    parts = SH.partition(rp.nodes, world)
    off, local, idx = parts[rank]
    arr, n = trace.typical()
    eng = ksim.Engine(len(idx), 1, device=device)
    eng.set_shard(rank, world, off, trace.num_nodes, None)
    handles = [eng.shard_peer_handle()]
    if dist is not None:
        handles = [None] * world
        dist.all_gather_object(handles, eng.shard_peer_handle())
    eng.set_shard_peers(handles)
    eng.set_nodes(0, local)
    eng.set_typical(0, arr, n)
    eng.set_policy(0, "FGD")
    eng.load_events(0, rp.events, rp.n)
    eng.total_events = rp.n
    return eng


def _engine_on(device, trace, seeds, nodes_per_block, policy="FGD", wgs=0, run_mode=0, tune=1.3, shuffle=True,
               report=False, random_stream="hash"):
    arr, n = trace.typical()
    eng = ksim.Engine(trace.num_nodes, len(seeds), device=device, nodes_per_block=nodes_per_block,
                      wgs_per_replica=wgs, run_mode=run_mode)
    if report:
        eng.set_report(True)
    total = 0
    for r, s in enumerate(seeds):
        rp = trace.replay(seed=s, tune_ratio=tune, shuffle=shuffle)
        eng.set_nodes(r, rp.nodes)
        eng.set_typical(r, arr, n)
        eng.set_policy(r, policy)
        if ksim.parse_policy(policy)[0] in ("PWR", "PWR+FGD"):
            eng.set_power_model(r, trace.power_model())
        if policy == "Random" and random_stream == "go":
            eng.set_go_stream(r, trace.go_state(seed=s, tune_ratio=tune, shuffle=shuffle))
        eng.load_events(r, rp.events, rp.n)
        total += rp.n
    eng.total_events = total
    return eng


if __name__ == "__main__":
    main()
