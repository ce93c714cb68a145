"""Date-sharded calc_var: one process per GPU, RCCL over xGMI.

The reference parallelises calc_var over dates with joblib
(utils/calc_integral/calc_integral.py:211-223), but its bisection is coupled
across the whole batch: the iteration count is the max over all dates (Q2,
utils/calc_var_class.py:278) and an all-zero iteration stops every date (Q4,
:293).  Sharding dates across ranks keeps those semantics with ONE exchange:

1. every rank solves its contiguous date block with a fixed bisection budget
   and records per-date snapshots + a 16-byte header (``cvq_solve_local``);
2. one all-gather of the headers and one of the snapshots;
3. every rank finalises the full VaR vector from them (``cvq_solve_finalize``).

Per step that is 16 B x world + 8 B x (K+1) x T_total over the fabric (<= 2 MB
at T = 5000) -- latency-bound, so it is issued as two collectives, not per
iteration.  The solve itself has no data-path collective.

``ShardedVaR`` takes the local and finalize steps as callables on tensors so
the same sharding / collective code runs on GPUs (RCCL, the plan's device
entry points) and in CPU tests (gloo, the oracle's restatement).
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple

import torch
import torch.distributed as dist


def shard(T_total: int, rank: int, world: int) -> Tuple[int, int, int]:
    """Contiguous block of rank `rank`: (first date, end date, block rows per rank)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("rank must be in [0, world)")
    per = -(-int(T_total) // world)
    lo = min(rank * per, T_total)
    return lo, min(lo + per, T_total), per


def _gather(t: torch.Tensor, world: int, group=None) -> torch.Tensor:
    out = torch.empty((world * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out, t.contiguous(), group=group)
    else:
        dist.all_gather(list(out.chunk(world)), t.contiguous(), group=group)
    return out


class ShardedVaR:
    """calc_var over T_total dates split across the ranks of `group`.

    local(hdr, snaps): solve this rank's block; hdr is int64[2] (the 16-byte
        cvq Header), snaps float64[per, stride] (rows past the block stay NaN).
    finalize(hdr_all, snaps_all, var): full VaR vector from the gathered data.
    check(): optional convergence check after the finalize (raises on failure).
    """

    def __init__(self, T_total: int, stride: int, local: Callable, finalize: Callable,
                 device: torch.device, group=None, check: Optional[Callable] = None):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.T_total = int(T_total)
        self.lo, self.hi, self.per = shard(self.T_total, self.rank, self.world)
        self.stride = int(stride)
        self._local, self._finalize, self._check = local, finalize, check
        self.hdr = torch.zeros(2, dtype=torch.int64, device=device)
        self.snaps = torch.full((self.per, self.stride), float("nan"), dtype=torch.float64, device=device)
        self.var = torch.empty(self.T_total, dtype=torch.float64, device=device)

    def solve(self, check: bool = True) -> torch.Tensor:
        """Full VaR vector on every rank.  check: verify convergence within the
        bisection budget after the finalize (synchronises; the status is global, from
        the gathered headers, so every rank raises together)."""
        self._local(self.hdr, self.snaps)
        if self.world == 1:
            self._finalize(self.hdr, self.snaps, self.var)
        else:
            hdr_all = _gather(self.hdr, self.world, self.group)
            snaps_all = _gather(self.snaps, self.world, self.group)
            self._finalize(hdr_all, snaps_all, self.var)
        if check and self._check is not None:
            self._check()
        return self.var


def device_sharded_var(plan, args, T_total: int, device: torch.device, group=None) -> ShardedVaR:
    """ShardedVaR wired to a QuadraturePlan's device entry points (plan holds this rank's block).

    The plan is bound to torch's current stream at every solve, so its kernels, the
    snapshot buffers' initialisation and the collectives are ordered on one stream."""
    stride = plan.snap_stride(args)
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    holder: dict = {}

    def local(hdr, snaps):
        plan.set_stream(torch.cuda.current_stream(device).cuda_stream)
        plan.solve_local(args, hdr.data_ptr(), snaps.data_ptr())

    def finalize(hdr_all, snaps_all, var):
        plan.solve_finalize(args, hdr_all.data_ptr(), world, snaps_all.data_ptr(), holder["per"], T_total,
                            var.data_ptr())

    s = ShardedVaR(T_total, stride, local, finalize, device, group, check=plan.solve_status)
    holder["per"] = s.per
    return s
