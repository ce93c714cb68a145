#!/usr/bin/env python3
"""bench.py -- VaR dates solved/sec on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1]): 2-asset Student-t copula, MSM(k=4) marginals,
256x256 nested quadrature grid, 1000 out-of-sample dates per GPU (weak scaling:
rank r solves dates [r*1000, (r+1)*1000) of one synthetic series; the global
bisection coupling of the reference (Q2 iteration count, Q4 all-zero break) is
honoured with ONE all-gather of the per-rank solve headers + bisection snapshots,
after which every rank finalises the full VaR vector).

One "step" = the calc_var-equivalent scope (utils/calc_var_class.py:95-177) over
the batch, with the per-date forecast tables already resident in HBM:
  set per-date inputs (device copy) -> marginal/special-function tables (k_tables)
  -> per-date slab-on-the-fly bisection solve (k_compact; COMPACT strategy, the
  default; --strategy direct: k_direct) -> [all-gather] -> finalise.
  (--strategy prefix: k_tables -> joint-mass row prefixes k_mass -> k_solve_prefix.)

Prints ONE JSON line (rank 0).
  value        -- whole-job VaR-dates/s with `--inflight` independent batches in flight
                  (each its own plan + HIP stream; default 3), K timed steps.
  single_solve -- the SURVEY.md §8(d) figure: T / wall time of ONE calc_var-equivalent
                  solve (utils/calc_var_class.py:109-175), one batch at a time, K steps.
  roofline     -- dominant kernel (k_compact / k_sorted / k_mass), bound "fp64-valu":
                  algorithmic FP64 work (SURVEY.md §8d convention: FLOP per reachable
                  node x reachable nodes x dates per launch) / the kernel's average
                  duration, timed with HIP events on its stream in a separate one-batch
                  leg (one launch in flight, so the bracket is the kernel's own duration, as
                  rocprofv3's kernel trace gives it; profiles/ holds the trace split by
                  leg).  The legs that give value / single_solve carry no events.  Sub-object "hbm": 8 B x reachable nodes per date (the judged
                  algorithmic bytes of §8d) over the same duration, and the PMC traffic.
  cpu_baseline -- the joblib CPU path (oracle/joblib_port.py, scalar t.ppf),
                  timed on a bounded sample of the same workload, rank 0 at N=1.
  other_configs -- (default cfg-2 run, rank 0, N=1) configs 5 / 3 / 4 at full size, each a child
                  bench.py started after this run's timed legs (20 steps): in flight, single solve
                  (one batch at a time), kernel launch time, FP64 fraction, end to end;
                  `--other-configs`.

Multi-GPU: one process per GPU (torch.distributed, RCCL).  `python bench.py --gpus N` with no
launcher around it starts its N ranks itself (torch.distributed.run as a child process, before
anything touches the GPU, exiting with its return code); under a launcher WORLD_SIZE must equal
--gpus.  Default weak scaling
(--dates-per-gpu, default the config's T, per rank); --global-dates G solves G dates
split into contiguous blocks of ceil(G / N) (BASELINE configs 3/4/5: 5000 / 2000 / 5000
"sharded over 8"), strong scaling.  Both run every rank's block through
copula_var.distributed.device_sharded_var (local solve -> ONE all-gather -> finalize)
whenever N > 1 or --global-dates is given; each in-flight batch has its own process
group, so the batches' collectives never share a communicator.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "copula-msm-and-copula-garch-var_amd")
sys.path[:0] = [PKG, REPO]

# BASELINE.json metric (config 2); the other configs are labelled by their workload
METRICS = {2: "VaR dates solved/sec, 2-asset Student-copula MSM, 256x256 grid, 1/2/4/8 GPUs"}

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
FP64_PEAK_TFLOPS = 78.6        # MI355X FP64 vector (vendor figure)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="process group for N > 1 (nccl = RCCL over xGMI; gloo: the multi-rank path on "
                         "fewer GPUs than ranks, ranks sharing devices round-robin -- a test rehearsal)")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", type=int, default=2, help="BASELINE config number (1-5)")
    ap.add_argument("--dates-per-gpu", type=int, default=None)
    ap.add_argument("--global-dates", type=int, default=None,
                    help="total dates split over the ranks (strong scaling); default: --dates-per-gpu per rank")
    ap.add_argument("--single", type=int, default=1, help="also time the one-batch-at-a-time solve (single_solve)")
    ap.add_argument("--strategy", default="auto", choices=["auto", "prefix", "direct", "compact", "sorted", "sweep"],
                    help="auto: COMPACT for 2-asset MSM and integer-power Student, SORTED otherwise (engine.auto_strategy)")
    ap.add_argument("--cpu-baseline", type=int, default=1, help="time the joblib CPU path (rank 0, N=1)")
    ap.add_argument("--cpu-dates", type=int, default=0,
                    help="CPU sample size (0 = four per worker: ~15 s of joblib work on config 2)")
    ap.add_argument("--cpu-jobs", type=int, default=0)
    ap.add_argument("--e2e", type=int, default=1,
                    help="1 GPU: also time end-to-end steps (device forecast tables + solve, from returns)")
    ap.add_argument("--inflight", type=int, default=3,
                    help="independent batches in flight (one plan + HIP stream each); 1 = one batch at a time")
    ap.add_argument("--nu", type=float, default=None,
                    help="Student copula nu instead of the config's (e.g. 5.364, an IFM-fitted value: the "
                         "non-integer node power path)")
    ap.add_argument("--copula", default=None, choices=["gaussian", "student", "plackett"],
                    help="copula instead of the config's (same grid, model and dates; strategy studies)")
    ap.add_argument("--other-configs", default="auto",
                    help="after the main line, run these BASELINE configs' single solves as child processes and "
                         "attach their results (rank 0, N = 1): comma list, 'none', or 'auto' = 5,3,4 when the "
                         "main config is 2")
    ap.add_argument("--time-all", type=int, default=0,
                    help="HIP-event time every kernel kind (adds event records to the timed region)")
    return ap.parse_args()


def build_inputs(cfg, T_total, rank, world, device):
    """Synthetic returns for all dates; this rank's per-date tables via the device filters.
    Rank r holds the contiguous block distributed.shard gives it (ceil(T / world) dates)."""
    from copula_var import synthetic, tables
    from copula_var.distributed import shard
    c = cfg.with_(T=T_total)
    rets = synthetic.simulate_returns(c)
    mean, ptf_mean, centred, T = tables.insample_split(rets, c.n_in, c.weights)
    lo, hi, _ = shard(T_total, rank, world)
    per = hi - lo
    block = centred[lo: hi + c.n_in]                              # windows lo .. hi-1
    t0 = time.time()
    if c.model == "msm":
        ipt, uvs, ggp = tables.msm_integration_params(block, c.n_in, c.msm_params, c.k, c.num_points, device)
    else:
        ipt, uvs, ggp = tables.sigma_integration_params(block, c.n_in, c.model, c.model_params(), c.num_points, device)
    t_fc = time.time() - t0
    return c, ipt, uvs, ggp, ptf_mean, per, t_fc, block


def launch_ranks(a, argv):
    """`--gpus N` (N > 1) without a launcher: run this same command under torch.distributed.run
    with N ranks on this node (rendezvous on 127.0.0.1) as a child process and return its exit
    code.  Called before torch is imported, so this process never initialises the GPU.
    Under a launcher (WORLD_SIZE set) the world size must equal --gpus."""
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None:
        if int(env_world) != a.gpus:
            raise SystemExit(f"bench.py: WORLD_SIZE={env_world} (launcher) but --gpus {a.gpus}: "
                             "they must agree (n_gpus would misreport the run)")
        return None
    if a.gpus <= 1:
        return None
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)
    return subprocess.run(cmd, cwd=REPO).returncode


def main():
    a = parse()
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    import torch
    import torch.distributed as dist
    from copula_var import engine, synthetic

    if a.backend == "gloo":                           # rehearsal: ranks may share a device
        local = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    if world > 1:
        if a.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    cfg = synthetic.baseline_configs()[a.config]
    if a.nu is not None:
        if cfg.copula != "student":
            raise SystemExit(f"--nu applies to Student-copula configs; config {a.config} is {cfg.copula}")
        cfg = cfg.with_(nu=float(a.nu))
    if a.copula is not None and a.copula != cfg.copula:
        if cfg.dim == 3 and a.copula == "plackett":
            raise SystemExit("the Plackett copula is bivariate")
        corr = cfg.corr if cfg.corr is not None else np.full((cfg.dim, cfg.dim), 0.5) + 0.5 * np.eye(cfg.dim)
        cfg = cfg.with_(copula=a.copula, corr=corr)
    if a.strategy == "auto":
        a.strategy = engine.auto_strategy(cfg.model, cfg.dim, cfg.num_points, cfg.copula, cfg.copula_params())
    strong = a.global_dates is not None
    T_total = a.global_dates if strong else (a.dates_per_gpu or cfg.T) * world
    sharded = world > 1 or strong                 # local solve -> [all-gather] -> finalize
    c, ipt, uvs, ggp, ptf_mean, per, t_fc, block = build_inputs(cfg, T_total, rank, world, local)
    dens, x, step, combos = ggp
    dev = torch.device("cuda", local)
    d_a = torch.tensor(ipt[0], dtype=torch.float64, device=dev).contiguous()
    d_b = torch.tensor(ipt[1], dtype=torch.float64, device=dev).contiguous() if c.model == "msm" else None
    b_ptr = d_b.data_ptr() if d_b is not None else None
    args = engine.solve_args(ptf_mean)
    fast_ok = c.model == "msm" and bool(np.array_equal(                # the kernel's own rank-1 test, on the host
        ipt[1], (ipt[0][:, 0, :, None] * ipt[0][:, 1, None, :]).reshape(ipt[1].shape))) if c.dim == 2 else False
    if c.model != "msm" and c.dim == 2 and c.copula == "student":   # cvq_plan.hip fast_path_proven's Student rule
        fast_ok = bool(np.all(np.isfinite(ipt[0]) & (ipt[0] > 0.0)))
    # `inflight` batches in flight: plan i (its own HIP stream, scratch, output and, when
    # sharded, its own process group) solves steps i, i + inflight, ...  Consecutive
    # batches are independent, so the next one fills the CUs the current one's last
    # workgroups leave idle.
    nf = max(1, a.inflight)
    plans, streams, vars_, shardeds = [], [], [], []
    for _ in range(nf):
        p = engine.QuadraturePlan(c.model, c.copula, c.dim, x, step, dens, combos, c.weights,
                                  c.copula_params(), vol_states=uvs, device=local, strategy=a.strategy)
        s_ = torch.cuda.Stream(device=dev) if nf > 1 else torch.cuda.current_stream()
        p.set_stream(s_.cuda_stream)
        plans.append(p)
        streams.append(s_)
        vars_.append(torch.empty(T_total, dtype=torch.float64, device=dev))
        if sharded:
            from copula_var.distributed import device_sharded_var
            grp = dist.new_group(list(range(world))) if world > 1 else None
            with torch.cuda.stream(s_):
                shardeds.append(device_sharded_var(p, args, T_total, dev, group=grp))
    plan = plans[0]

    local_only = [False]                              # sharded: time this rank's local solve alone

    def step_fn(k):
        with torch.cuda.stream(streams[k]):
            # pi = outer product of the per-asset forecasts (compute_forecast_combinations), so the
            # fast path is asserted (a violating date would fail the solve status check below)
            plans[k].set_dates_device(per, d_a.data_ptr(), b_ptr, fast=fast_ok)   # forces tables recompute
            if not sharded:
                plans[k].solve_device(args, vars_[k].data_ptr())
            elif local_only[0]:
                shardeds[k].solve_local()
            else:
                shardeds[k].solve(check=False)

    def timed(n_batches, steps, warmup, timing=None, bracket=None):
        """Wall time of `steps` steps (batch i % n_batches), barrier + synchronize on both
        sides, max over ranks.  bracket: a list that receives the device time (ms) between
        two HIP events recorded on batch 0's stream before the first and after the last
        step (no events between launches)."""
        for i in range(warmup):
            step_fn(i % n_batches)
        torch.cuda.synchronize()
        for k in range(nf):
            plans[k].enable_timing(timing if (timing and k < n_batches) else False)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        if bracket is not None:
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record(streams[0])
        t0 = time.perf_counter()
        for i in range(steps):
            step_fn(i % n_batches)
        t_enq = time.perf_counter() - t0                  # host time to enqueue the K steps
        if bracket is not None:
            ev1.record(streams[0])
        torch.cuda.synchronize()
        if bracket is not None:
            bracket.append(ev0.elapsed_time(ev1))
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        if world > 1:
            tt = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            el = float(tt.item())
        kt = {}
        for kind in ("tables", "mass", "solve", "finalize"):
            ms_n = [plans[k].kernel_time(kind) for k in range(n_batches)]
            kt[kind] = (sum(m for m, _ in ms_n), sum(n_ for _, n_ in ms_n))
        for k in range(n_batches):       # convergence within the bisection budget (outside the timed region)
            plans[k].solve_status()
        enq_ms.append(t_enq / steps * 1e3)
        return el, kt

    enq_ms = []                                       # host enqueue time per step of each timed leg
    dom = "mass" if a.strategy == "prefix" else "solve"                      # dominant kernel
    # no HIP events between the timed legs' launches (an event record between two launches on
    # a stream delays the second: rocprofv3 saw ~10 us gaps in an event-timed one-batch leg)
    brk0 = []                                         # one batch in flight: the main leg's bracket
    elapsed, kt = timed(nf, a.steps, a.warmup, True if a.time_all else None, brk0 if nf == 1 else None)
    vals = (vars_[0] if not sharded else shardeds[0].var).cpu().numpy()
    ms_step = elapsed / a.steps * 1e3
    value = T_total * a.steps / elapsed
    # one batch at a time; its back-to-back launches bracketed by two HIP events on the stream
    # (the step is the one fused solve kernel for COMPACT / SORTED / SWEEP: the bracket over
    # K steps / K is the kernel's average duration, as rocprofv3's kernel trace gives it)
    one_kernel = a.strategy in ("compact", "sorted", "sweep") and not sharded
    brk = []
    if nf > 1 and a.single:
        el1, _ = timed(1, a.steps, a.warmup, None, brk)
        v1 = (vars_[0] if not sharded else shardeds[0].var).cpu().numpy()
        assert np.array_equal(v1, vals, equal_nan=True), "single-solve leg changed the VaR"
    else:
        el1 = elapsed
        brk = brk0
    single = {"value": T_total * a.steps / el1, "unit": "VaR-dates/s", "ms_per_step": el1 / a.steps * 1e3,
              "inflight": 1, "steps": a.steps,
              "scope": "one calc_var-equivalent solve per step (utils/calc_var_class.py:109-175), tables resident"}
    if sharded and a.single:
        # the step's two parts: every rank's local solve of its block (max over ranks), and the
        # rest -- the one all-gather of the packed blocks + the finalize
        local_only[0] = True
        el_loc, _ = timed(1, a.steps, a.warmup)
        local_only[0] = False
        single["local_solve_ms"] = el_loc / a.steps * 1e3
        single["allgather_finalize_ms"] = max(single["ms_per_step"] - single["local_solve_ms"], 0.0)
        single["split_note"] = ("local_solve_ms: the same one-batch leg without the exchange (barrier + synchronize "
                                "around K steps, max over ranks); allgather_finalize_ms: ms_per_step minus it")

    # roofline of the dominant kernel.  COMPACT / SORTED / SWEEP: the single-solve leg's event
    # bracket / K.  Otherwise (several kernels per step): one batch at a time with HIP events
    # around each launch of the dominant kernel.
    if one_kernel and brk:
        el_r, kt1 = el1, {dom: (brk[0], a.steps)}
        timing_note = ("two HIP events on the kernel's stream bracketing the single-solve leg's K back-to-back "
                       "launches (no events between launches); avg = bracket / K")
    else:
        el_r, kt1 = timed(1, a.steps, a.warmup, (dom,))
        timing_note = "HIP events around each launch on the kernel's stream, a separate one-batch leg"
    for p in plans:
        p.enable_timing(False)
    dom_ms, dom_n = kt1[dom]
    dom_avg_s = dom_ms / max(dom_n, 1) / 1e3
    # FP64 basis (SURVEY §8d convention): per node 14 FLOP + 1 pow (counted as 1) for Student,
    # over the nodes the solve evaluates -- counted on the device in one extra, untimed solve
    # (SORTED evaluates each node of its bisection path once: cfg 4 ~17% of the reachable set,
    # so the reachable-node basis would overstate the work), the reachable-node figure beside it
    flop_node = {"student": 15.0, "gaussian": 14.0, "plackett": 16.0}[c.copula] + (9.0 if c.dim == 3 else 0.0)
    nodes_eval = None
    if a.strategy in ("compact", "sorted", "sweep") and not sharded:
        plan.count_nodes(True)
        step_fn(0)
        torch.cuda.synchronize()
        nodes_eval = plan.nodes_evaluated()
        plan.count_nodes(False)
        v2 = vars_[0].cpu().numpy()
        assert np.array_equal(v2, vals, equal_nan=True), "node-count solve changed the VaR"
    flop_launch = flop_node * (nodes_eval if nodes_eval is not None else plan.reach_nodes * per)
    flop_reach = flop_node * plan.reach_nodes * per
    fp64_tflops = flop_launch / dom_avg_s / 1e12 if dom_avg_s > 0 else 0.0
    alg_bytes = 8.0 * plan.reach_nodes * per          # one f64 joint-mass word per reachable node
    achieved_gbs = alg_bytes / dom_avg_s / 1e9 if dom_avg_s > 0 else 0.0
    # PMC HBM bytes per launch (profiles/pmc_traffic_cfg<N>.json, tools/pmc_summary.py): attached only
    # when that pass measured THIS library build (sha of libcvq.so), the same strategy and launch size
    traffic, traffic_src = None, "no PMC pass of this library build (tools/pmc.sh)"
    lib_sha = _lib_sha16()
    pmc_path = os.path.join(REPO, "profiles", f"pmc_traffic_cfg{a.config}.json")
    if os.path.exists(pmc_path):
        try:
            pm = json.load(open(pmc_path))
            if (pm.get("lib_sha16") == lib_sha and pm.get("dates_per_launch") == per
                    and pm.get("strategy") == a.strategy):
                traffic = pm.get("hbm_bytes_per_launch")
                traffic_src = f"profiles/pmc_traffic_cfg{a.config}.json (FETCH_SIZE + WRITE_SIZE, lib {lib_sha})"
        except Exception:
            traffic = None
    pmc_gbs = traffic / dom_avg_s / 1e9 if (traffic is not None and dom_avg_s > 0) else None
    # the binding roofline: FP64 VALU unless the measured HBM traffic is the larger fraction of its
    # peak (the algorithmic bytes of SURVEY §8d are notional -- the solve never materialises the mass)
    fp64_frac = fp64_tflops / FP64_PEAK_TFLOPS
    hbm_bound = pmc_gbs is not None and pmc_gbs / HBM_PEAK_GBS > fp64_frac
    kernels = {k: {"avg_us": (v[0] / max(v[1], 1)) * 1e3, "launches": v[1]} for k, v in kt.items() if v[1]}
    kernels_single = {k: {"avg_us": (v[0] / max(v[1], 1)) * 1e3, "launches": v[1]} for k, v in kt1.items() if v[1]}

    e2e = None
    if a.e2e and world == 1 and not strong:
        e2e = end_to_end(a, c, block, per, plans, streams, vars_, args, vals, dev)

    cpu = None
    if rank == 0 and world == 1 and a.cpu_baseline:
        cpu = cpu_baseline(c, ipt, uvs, ggp, ptf_mean, vals, a)

    others = None
    if rank == 0 and world == 1 and not strong:
        others = other_configs(a)

    if rank == 0:
        kname = {"prefix": "k_mass (joint-mass row prefix)",
                 "direct": "k_direct (per-date slab-on-the-fly solve)",
                 "compact": "k_compact (per-date solve, block tail)",
                 "sorted": "k_sorted (per-date solve over the v*-sorted node list)",
                 "sweep": "k_sorted<SWEEP> (per-date solve, one pass per bisection cell)"}[a.strategy]
        out = {
            "metric": METRICS.get(a.config, f"VaR dates solved/sec, {c.name}"),
            "value": value,
            "unit": "VaR-dates/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": f"synthetic ({c.model} returns, seed {c.seed}; injected in-sample params; fixed copula)",
            "config": {"workload": f"cfg{a.config}: {c.name}" + (f", nu {c.nu}" if a.nu is not None else "")
                       + (f", copula {c.copula}" if a.copula is not None else ""),
                       "model": c.model, "copula": c.copula,
                       "dim": c.dim, "grid": f"{c.num_points}^{c.dim}", "dates_per_gpu": per,
                       "global_dates": T_total, "n_in": c.n_in, "parallelism": f"dates/dp{world}",
                       "strategy": a.strategy, "inflight": nf},
            "single_solve": single,
            "host_enqueue_ms_per_step": enq_ms[0] if enq_ms else None,
            "roofline": {"bound": "hbm" if hbm_bound else "fp64-valu",
                         "achieved": pmc_gbs if hbm_bound else fp64_tflops,
                         "peak": HBM_PEAK_GBS if hbm_bound else FP64_PEAK_TFLOPS,
                         "unit": "GB/s" if hbm_bound else "TFLOP/s",
                         "frac": pmc_gbs / HBM_PEAK_GBS if hbm_bound else fp64_frac,
                         "traffic": traffic, "traffic_source": traffic_src, "lib_sha16": lib_sha, "kernel": kname,
                         "flop_per_node": flop_node,
                         "flop_basis": "nodes evaluated (device count)" if nodes_eval is not None
                                       else "reachable nodes",
                         "nodes_evaluated_per_date": (nodes_eval / per) if nodes_eval is not None else None,
                         "reach_nodes_per_date": plan.reach_nodes,
                         "dates_per_launch": per, "flop_per_launch": flop_launch,
                         "avg_launch_us": dom_avg_s * 1e6, "launches": dom_n,
                         "timing": timing_note,
                         "event_leg_ms_per_step": el_r / a.steps * 1e3,
                         "reach_basis": {"flop_per_launch": flop_reach,
                                         "frac": flop_reach / dom_avg_s / 1e12 / FP64_PEAK_TFLOPS
                                         if dom_avg_s > 0 else 0.0},
                         "fp64": {"achieved": fp64_tflops, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                                  "frac": fp64_frac},
                         "hbm": {"pmc_bytes_per_launch": traffic, "pmc_achieved": pmc_gbs,
                                 "pmc_frac": pmc_gbs / HBM_PEAK_GBS if pmc_gbs is not None else None,
                                 "alg_bytes_per_launch": alg_bytes, "alg_achieved": achieved_gbs,
                                 "alg_frac": achieved_gbs / HBM_PEAK_GBS, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                 "note": "alg_*: 8 B x reachable nodes (SURVEY §8d), notional -- the solve never "
                                         "writes the joint mass; pmc_*: measured FETCH_SIZE + WRITE_SIZE"}},
            "kernels": kernels,
            "kernels_single": kernels_single,
            "forecast_stage_s": t_fc,
            "e2e": e2e,
            "var_checksum": float(np.nansum(vals)),
            "var_nan": int(np.isnan(vals).sum()),
            "cpu_baseline": cpu,
            "other_configs": others,
        }
        print(json.dumps(out), flush=True)
    for p in plans:
        p.close()
    if world > 1:
        dist.destroy_process_group()


def other_configs(a):
    """The other BASELINE configs at full size (auto strategy): batches in flight, the single solve
    (one batch at a time) and end to end -- each a fresh child `bench.py` process started after this
    run's own timed legs, so the default run's line also carries them (SURVEY.md §8d lists
    every config).  A child that fails or times out is recorded with its error, never raised."""
    import subprocess
    spec = a.other_configs
    if spec == "none" or (spec == "auto" and (a.config != 2 or a.dates_per_gpu is not None or a.nu is not None
                                              or a.copula is not None
                                              or a.strategy not in ("auto", "compact"))):
        return None
    cfgs = [5, 3, 4] if spec == "auto" else [int(v) for v in spec.split(",") if v.strip()]
    res = {}
    for cn in cfgs:
        cmd = [sys.executable, os.path.abspath(__file__), "--config", str(cn), "--steps", "20",
               "--warmup", "3", "--e2e", "1", "--cpu-baseline", "0", "--other-configs", "none"]
        try:
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
            line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
            if r.returncode != 0 or not line:
                res[f"cfg{cn}"] = {"error": f"exit {r.returncode}: {r.stderr.strip().splitlines()[-1:] }"}
                continue
            d = json.loads(line[-1])
            rf = d.get("roofline") or {}
            res[f"cfg{cn}"] = {"workload": d["config"]["workload"], "strategy": d["config"]["strategy"],
                               "dates": d["config"]["global_dates"], "in_flight": d["value"],
                               "inflight": d["config"]["inflight"],
                               "single_solve": (d.get("single_solve") or {}).get("value"),
                               "unit": d["unit"], "ms_per_step": d["ms_per_step"], "steps": d["steps"],
                               "kernel_avg_launch_us": rf.get("avg_launch_us"), "fp64_frac": rf.get("frac"),
                               "e2e": (d.get("e2e") or {}).get("value"), "var_checksum": d.get("var_checksum")}
        except subprocess.TimeoutExpired:
            res[f"cfg{cn}"] = {"error": "timed out after 300 s"}
    return res


def end_to_end(a, c, block, per, plans, streams, vars_, args, vals, dev):
    """End-to-end steps: centred returns resident in HBM -> every asset's
    rolling-window forecasts on the device -> the solve reading those tables in place.
    MSM: Hamilton filters, state collapse and forecast combinations (cvq_msm_tables);
    GARCH / UKF: sigma forecasts written as [T][dim] (cvq_sigma_tables).  Same batches in
    flight; the VaR must equal the main loop's (tables resident) bit for bit."""
    import torch
    from copula_var import engine, tables
    r_dev = torch.tensor(np.ascontiguousarray(block[:-1].T), dtype=torch.float64, device=dev)
    nf = len(plans)
    if c.model == "msm":
        vsa = np.array([tables.msm_vol_states(c.k, p["m_0"], p["sig"]) for p in c.msm_params])
        smap, uvs = tables.unique_vol_map(vsa)
        prm = [[p["m_0"], p["sig"], p["b"], p["gamma"]] for p in c.msm_params]
        mts = [engine.MsmTables(prm, c.k, smap, uvs.shape[1], c.n_in, per, dev.index or 0) for _ in range(nf)]
        ptrs = lambda m: (m.fbs.data_ptr(), m.pi.data_ptr())
        stage = "returns in HBM -> device MSM filters + tables (cvq_msm_tables) -> solve"
    else:
        mts = [engine.SigmaTables(c.model, c.model_params(), c.n_in, per, dev.index or 0) for _ in range(nf)]
        ptrs = lambda m: (m.sig.data_ptr(), None)
        stage = f"returns in HBM -> device {c.model} sigma forecasts (cvq_sigma_tables) -> solve"

    def step(i):
        k = i % nf
        with torch.cuda.stream(streams[k]):
            mts[k].run(r_dev, streams[k].cuda_stream)
            # cvq_msm_tables: rank-1 pi; GARCH / UKF Student: any finite sigma > 0 (a failed forecast
            # window is reported by the forecast stage, a violating date fails the solve loudly)
            plans[k].set_dates_device(per, *ptrs(mts[k]), fast=c.model == "msm" or (c.dim == 2 and c.copula == "student"))
            plans[k].solve_device(args, vars_[k].data_ptr())

    for i in range(a.warmup):
        step(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        step(i)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    for k, m in enumerate(mts):
        m.status(streams[k].cuda_stream)
        plans[k].solve_status()
    v = vars_[(a.steps - 1) % nf].cpu().numpy()
    return {"value": per * a.steps / el, "unit": "VaR-dates/s", "ms_per_step": el / a.steps * 1e3,
            "stage": stage, "var_matches_resident_tables": bool(np.array_equal(v, vals))}


def cpu_baseline(c, ipt, uvs, ggp, ptf_mean, gpu_var, a):
    """joblib CPU path on a bounded sample (first S dates of this workload)."""
    from oracle import quadrature as Q
    from oracle.joblib_port import JoblibPath
    jobs = a.cpu_jobs or min(16, os.cpu_count() or 1)
    S = a.cpu_dates or 4 * jobs
    dens, x, step, combos = ggp
    if c.model == "msm":
        per = (ipt[0][:S], ipt[1][:S])
    else:
        per = ipt[0][:S]
    P = Q.Problem(c.model, c.copula, c.dim, x, step, dens, combos, c.weights, c.copula_params(), per, uvs)
    J = JoblibPath(P, n_jobs=jobs)
    t0 = time.perf_counter()
    var, it, _ = J.calc_var(ptf_mean)
    wall = time.perf_counter() - t0
    # the sample's own global iteration count can differ from the full batch's (Q2)
    return {"value": S / wall, "unit": "VaR-dates/s", "cores": jobs, "kind": "port",
            "sample": f"first {S} dates of the same workload, full calc_var control flow "
                      f"({it} bisection iterations), joblib n_jobs={jobs}, scalar t.ppf; wall {wall:.1f}s",
            "cpu": _cpu_model()}


def _lib_sha16():
    """Build id of the loaded HIP library: the first 16 hex digits of sha256(libcvq.so)."""
    import hashlib
    from copula_var import _native
    h = hashlib.sha256()
    with open(_native.LIB_PATH, "rb") as f:
        for blk in iter(lambda: f.read(1 << 20), b""):
            h.update(blk)
    return h.hexdigest()[:16]


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except Exception:
        pass
    return None


if __name__ == "__main__":
    _rc = launch_ranks(parse(), sys.argv[1:])
    if _rc is not None:
        sys.exit(_rc)
    main()
