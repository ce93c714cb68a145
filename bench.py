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

Prints ONE JSON line (rank 0).  Extra objects:
  roofline     -- dominant kernel (k_direct, or k_mass for PREFIX), HIP-event timed
                  on the plan's stream; algorithmic bytes = 8 B x reachable nodes
                  x dates per launch, plus an FP64 sub-object.
  cpu_baseline -- the joblib CPU path (oracle/joblib_port.py, scalar t.ppf),
                  timed on a bounded sample of the same workload, rank 0 at N=1.
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
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=2, help="BASELINE config number (1-5)")
    ap.add_argument("--dates-per-gpu", type=int, default=None)
    ap.add_argument("--strategy", default="auto", choices=["auto", "prefix", "direct", "compact", "sorted", "sweep"],
                    help="auto: COMPACT for 2-asset MSM, SORTED otherwise (engine.auto_strategy)")
    ap.add_argument("--cpu-baseline", type=int, default=1, help="time the joblib CPU path (rank 0, N=1)")
    ap.add_argument("--cpu-dates", type=int, default=0,
                    help="CPU sample size (0 = four per worker: ~15 s of joblib work on config 2)")
    ap.add_argument("--cpu-jobs", type=int, default=0)
    ap.add_argument("--e2e", type=int, default=1,
                    help="1 GPU: also time end-to-end steps (device forecast tables + solve, from returns)")
    ap.add_argument("--inflight", type=int, default=3,
                    help="independent batches in flight (one plan + HIP stream each); 1 = one batch at a time")
    ap.add_argument("--time-all", type=int, default=0,
                    help="HIP-event time every kernel kind (adds event records to the timed region)")
    return ap.parse_args()


def build_inputs(cfg, T_total, rank, world, device):
    """Synthetic returns for all dates; this rank's per-date tables via the device filters."""
    from copula_var import synthetic, tables
    c = cfg.with_(T=T_total)
    rets = synthetic.simulate_returns(c)
    mean, ptf_mean, centred, T = tables.insample_split(rets, c.n_in, c.weights)
    per = T_total // world
    lo = rank * per
    block = centred[lo: lo + c.n_in + per]                       # windows lo .. lo+per-1
    t0 = time.time()
    if c.model == "msm":
        ipt, uvs, ggp = tables.msm_integration_params(block, c.n_in, c.msm_params, c.k, c.num_points, device)
    else:
        ipt, uvs, ggp = tables.sigma_integration_params(block, c.n_in, c.model, c.model_params(), c.num_points, device)
    t_fc = time.time() - t0
    return c, ipt, uvs, ggp, ptf_mean, per, t_fc, block


def main():
    a = parse()
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    import torch
    import torch.distributed as dist
    from copula_var import engine, synthetic
    from copula_var import _native as N

    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    cfg = synthetic.baseline_configs()[a.config]
    if a.strategy == "auto":
        a.strategy = engine.auto_strategy(cfg.model, cfg.dim)
    per_gpu = a.dates_per_gpu or cfg.T
    T_total = per_gpu * world
    c, ipt, uvs, ggp, ptf_mean, per, t_fc, block = build_inputs(cfg, T_total, rank, world, local)
    dens, x, step, combos = ggp
    dev = torch.device("cuda", local)
    if c.model == "msm":
        d_a = torch.tensor(ipt[0], dtype=torch.float64, device=dev).contiguous()
        d_b = torch.tensor(ipt[1], dtype=torch.float64, device=dev).contiguous()
        b_ptr = d_b.data_ptr()
    else:
        d_a = torch.tensor(ipt[0], dtype=torch.float64, device=dev).contiguous()
        d_b, b_ptr = None, None
    args = engine.solve_args(ptf_mean)
    fast_ok = c.model == "msm" and bool(np.array_equal(                # the kernel's own rank-1 test, on the host
        ipt[1], (ipt[0][:, 0, :, None] * ipt[0][:, 1, None, :]).reshape(ipt[1].shape))) if c.dim == 2 else False
    # `inflight` batches in flight: plan i (its own HIP stream, scratch and output)
    # solves steps i, i + inflight, ...  Consecutive batches are independent, so
    # the next one fills the CUs that the current one's last workgroups leave idle.
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
        if world > 1:
            # rank-local solve -> one all-gather of headers + snapshots -> finalize (copula_var.distributed)
            from copula_var.distributed import device_sharded_var
            with torch.cuda.stream(s_):
                shardeds.append(device_sharded_var(p, args, T_total, dev))
    plan = plans[0]

    def step_fn(i):
        k = i % nf
        with torch.cuda.stream(streams[k]):
            # pi = outer product of the per-asset forecasts (compute_forecast_combinations), so the
            # fast path is asserted (a violating date would fail the solve status check below)
            plans[k].set_dates_device(per, d_a.data_ptr(), b_ptr, fast=fast_ok)   # forces tables recompute
            if world == 1:
                plans[k].solve_device(args, vars_[k].data_ptr())
            else:
                shardeds[k].solve(check=False)

    for i in range(a.warmup):
        step_fn(i)
    torch.cuda.synchronize()
    dom = "mass" if a.strategy == "prefix" else "solve"                       # dominant kernel
    for p in plans:
        p.enable_timing(True if a.time_all else (dom,))
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        step_fn(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    kt = {}
    for k in ("tables", "mass", "solve", "finalize"):
        ms_n = [p.kernel_time(k) for p in plans]
        kt[k] = (sum(m for m, _ in ms_n), sum(n_ for _, n_ in ms_n))
    for p in plans:                      # convergence within the bisection budget (outside the timed region)
        p.solve_status()
    vals = (vars_[0] if world == 1 else shardeds[0].var).cpu().numpy()
    ms_step = elapsed / a.steps * 1e3
    value = T_total * a.steps / elapsed

    # dominant kernel: k_mass (PREFIX) or the per-date solve k_direct (DIRECT)
    dom_ms, dom_n = kt[dom]
    dom_avg_s = dom_ms / max(dom_n, 1) / 1e3
    alg_bytes = 8.0 * plan.reach_nodes * per          # one f64 joint-mass word per reachable node
    achieved = alg_bytes / dom_avg_s / 1e9 if dom_avg_s > 0 else 0.0
    # with batches in flight a launch's duration includes time its workgroups wait for
    # the previous batch's CUs; the per-step figure is the delivered rate
    achieved_step = alg_bytes / (elapsed / a.steps) / 1e9
    # FP64 basis: per reachable node ~14 FLOP + 1 pow (counted as 1) for Student
    flop_node = {"student": 15.0, "gaussian": 14.0, "plackett": 16.0}[c.copula] + (9.0 if c.dim == 3 else 0.0)
    fp64_tflops = flop_node * plan.reach_nodes * per / dom_avg_s / 1e12 if dom_avg_s > 0 else 0.0
    traffic = None
    pmc_path = os.path.join(REPO, "profiles", f"pmc_traffic_cfg{a.config}.json")
    if os.path.exists(pmc_path):
        try:
            pm = json.load(open(pmc_path))
            if pm.get("dates_per_launch") == per and pm.get("strategy", "prefix") == a.strategy:
                traffic = pm.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    kernels = {k: {"avg_us": (v[0] / max(v[1], 1)) * 1e3, "launches": v[1]} for k, v in kt.items() if v[1]}

    e2e = None
    if a.e2e and world == 1:
        e2e = end_to_end(a, c, block, per, plans, streams, vars_, args, vals, dev)

    cpu = None
    if rank == 0 and world == 1 and a.cpu_baseline:
        cpu = cpu_baseline(c, ipt, uvs, ggp, ptf_mean, vals, a)

    if rank == 0:
        out = {
            "metric": METRICS.get(a.config, f"VaR dates solved/sec, {c.name}"),
            "value": value,
            "unit": "VaR-dates/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": f"synthetic ({c.model} returns, seed {c.seed}; injected in-sample params; fixed copula)",
            "config": {"workload": f"cfg{a.config}: {c.name}", "model": c.model, "copula": c.copula,
                       "dim": c.dim, "grid": f"{c.num_points}^{c.dim}", "dates_per_gpu": per,
                       "global_dates": T_total, "n_in": c.n_in, "parallelism": f"dates/dp{world}",
                       "strategy": a.strategy, "inflight": nf},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": {"prefix": "k_mass (joint-mass row prefix)",
                                    "direct": "k_direct (per-date slab-on-the-fly solve)",
                                    "compact": "k_compact (per-date solve, one-wave tail)",
                                    "sorted": "k_sorted (per-date solve over the v*-sorted node list)",
                                    "sweep": "k_sorted<SWEEP> (per-date solve, one pass per bisection cell)"}[a.strategy],
                         "alg_bytes_per_launch": alg_bytes, "avg_launch_us": dom_avg_s * 1e6,
                         "achieved_per_step": achieved_step,
                         "reach_nodes_per_date": plan.reach_nodes,
                         "fp64": {"achieved_tflops": fp64_tflops, "peak_tflops": FP64_PEAK_TFLOPS,
                                  "frac": fp64_tflops / FP64_PEAK_TFLOPS, "flop_per_node": flop_node}},
            "kernels": kernels,
            "forecast_stage_s": t_fc,
            "e2e": e2e,
            "var_checksum": float(np.nansum(vals)),
            "var_nan": int(np.isnan(vals).sum()),
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    for p in plans:
        p.close()
    if world > 1:
        dist.destroy_process_group()


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
            plans[k].set_dates_device(per, *ptrs(mts[k]), fast=c.model == "msm")   # cvq_msm_tables: rank-1 pi
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


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except Exception:
        pass
    return None


if __name__ == "__main__":
    main()
