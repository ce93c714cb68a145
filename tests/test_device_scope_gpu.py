"""The library's device discipline.

Every C entry point restores the caller's current HIP device on return (cvq::DeviceScope) and
switches to its plan's or argument's device for its own work -- torch shares the process's
current device, so a plan on device 1 must not move torch's.  The plan entries that only
synchronise and copy (node counts, stamps, kernel times) set the plan's device too, so a plan
on the NULL stream of another device syncs that device.  And the engine's node counts follow
the plan that actually ran a routed solve (strategy "auto" sends levels above v_cap to an
unrestricted sibling plan)."""
import numpy as np
import pytest
import torch

from conftest import load_golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu(gpu_available):
    if not gpu_available:
        pytest.fail("GPU tests were selected but no HIP device / libcvq.so is available")


def _plan(z, device=0, strategy="auto"):
    from copula_var.engine import QuadraturePlan
    p = QuadraturePlan(str(z["model"]), str(z["copula"]), int(z["dim"]), z["x_values"], z["step"], z["densities"],
                       z["combos"], z["weights"], z["copula_params"], vol_states=z.get("unique_vol_states"),
                       device=device, strategy=strategy)
    if str(z["model"]) == "msm":
        p.set_dates((z["forecasts_by_states"], z["forecasts"]))
    else:
        p.set_dates([z["sigma_forecasts"]])
    return p


def test_out_of_range_device_is_rejected_and_current_device_kept():
    import ctypes as C
    from copula_var import _native as N
    from copula_var.engine import QuadraturePlan
    torch.cuda.set_device(0)
    bad = torch.cuda.device_count() + 7
    x = np.linspace(0.1, 0.9, 9)
    out = np.empty_like(x)
    rc = N.lib().cvq_special(bad, 0, 6.0, N.ptr(x), x.size, N.ptr(out), N.MEM_HOST)
    assert rc != 0
    assert torch.cuda.current_device() == 0
    z = load_golden("cfg1")
    with pytest.raises((ValueError, N.NativeError)):
        QuadraturePlan(str(z["model"]), str(z["copula"]), 2, z["x_values"], z["step"], z["densities"], z["combos"],
                       z["weights"], z["copula_params"], device=bad)
    assert torch.cuda.current_device() == 0
    n = C.c_int32(0)
    assert N.lib().cvq_device_count(C.byref(n)) == 0 and n.value == torch.cuda.device_count()


def test_plan_on_another_device_keeps_torch_device():
    if torch.cuda.device_count() < 2:
        pytest.skip("needs 2 GPUs")
    z = load_golden("cfg2_n64")
    torch.cuda.set_device(0)
    p = _plan(z, device=1, strategy="compact")
    try:
        p.count_nodes(True)
        var, it = p.calc_var(float(z["ptf_mean"]))
        assert torch.cuda.current_device() == 0
        assert p.nodes_evaluated() > 0
        assert torch.cuda.current_device() == 0
    finally:
        p.close()
    assert np.array_equal(var, z["var"])


def test_node_counts_follow_a_routed_local_solve():
    """An auto SORTED plan (cfg 1: GARCH Gaussian) holds the nodes with v* <= v_cap = 0 only; a
    solve whose second guess reaches above 0 runs on the COMPACT sibling, and its node count
    is read from there (solve_local and compute_integral record the routed plan too)."""
    from copula_var import engine
    from copula_var.engine import QuadraturePlan
    z = load_golden("cfg1")
    p = _plan(z)
    try:
        assert p.strategy == "sorted"
        args = engine.solve_args(float(z["ptf_mean"]), second_guess=(-3.5, 0.5))
        T = p.T
        ln, off = QuadraturePlan.packed_block_len(args, T)
        blk = torch.zeros(ln, dtype=torch.float64, device="cuda")
        p.count_nodes(True)
        p.solve_local(args, blk[off:].data_ptr(), blk.data_ptr())
        torch.cuda.synchronize()
        assert p._wide is not None and p._wide.strategy == "compact"
        n_routed = p.nodes_evaluated()
        assert n_routed > 0 and n_routed == p._wide.nodes_evaluated()
        var, it = p.calc_var(float(z["ptf_mean"]))            # back on the SORTED plan itself
        assert np.array_equal(var, z["var"])
        n_own = p.nodes_evaluated()
        assert n_own > 0
    finally:
        p.close()
