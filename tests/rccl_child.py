"""Child process of tests/test_rccl_gpu.py: one NCCL (= RCCL on ROCm) rank on cuda:0.

Initialises the process group exactly as bench.py does for N > 1 ranks
(init_process_group("nccl", device_id=...)), then runs the sharded solve of the full cfg 2
batch (tests/golden/fullbatch_cfg2.npz) through copula_var.distributed.device_sharded_var:
local solve -> all_gather_into_tensor (distributed._gather's NCCL branch) -> packed finalize.
Prints one JSON line with the outcome; exits non-zero on any mismatch."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path[:0] = [os.path.join(REPO, "copula-msm-and-copula-garch-var_amd"), REPO]


def main():
    import numpy as np
    import torch
    import torch.distributed as dist
    from copula_var import engine
    from copula_var.distributed import _gather, device_sharded_var
    from copula_var.engine import QuadraturePlan

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    out = {"backend": dist.get_backend()}
    try:
        # the collective itself
        t = torch.arange(12, dtype=torch.float64, device=dev).view(1, -1)
        g = _gather(t, 1)
        out["gather_ok"] = bool(torch.equal(g, t))
        z = dict(np.load(os.path.join(HERE, "golden", "fullbatch_cfg2.npz"), allow_pickle=False))
        T = int(z["T"])
        p = QuadraturePlan(str(z["model"]), str(z["copula"]), int(z["dim"]), z["x_values"], z["step"],
                           z["densities"], z["combos"], z["weights"], z["copula_params"],
                           vol_states=z["unique_vol_states"], device=0)
        try:
            p.set_dates((z["forecasts_by_states"], z["forecasts"]))
            args = engine.solve_args(float(z["ptf_mean"]))
            sv = device_sharded_var(p, args, T, dev)
            var = sv.solve(check=True).cpu().numpy()
            out["iterations"] = p.solve_status()
        finally:
            p.close()
        out["var_equal"] = bool(np.array_equal(var, z["var"]))
        out["iterations_equal"] = out["iterations"] == int(z["iterations"])
        out["mismatch"] = int((var != z["var"]).sum())
    finally:
        dist.destroy_process_group()
    print(json.dumps(out), flush=True)
    ok = out["backend"] == "nccl" and out["gather_ok"] and out["var_equal"] and out["iterations_equal"]
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
