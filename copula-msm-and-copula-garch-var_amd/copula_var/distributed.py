"""Date-sharded calc_var: one process per GPU, RCCL over xGMI.

The reference parallelises calc_var over dates with joblib
(utils/calc_integral/calc_integral.py:211-223), but its bisection is coupled
across the whole batch: the iteration count is the max over all dates (Q2,
utils/calc_var_class.py:278) and an all-zero iteration stops every date (Q4,
:293).  Sharding dates across ranks keeps those semantics with ONE exchange:

1. every rank solves its contiguous date block with a fixed bisection budget
   and records per-date snapshots + a 16-byte header (``cvq_solve_local``),
   both into ONE per-rank block (snapshots, then the header);
2. one all-gather of the blocks;
3. every rank finalises the full VaR vector from them (``cvq_solve_finalize_packed``).

Per step that is 8 B x (K+1) x T_total + 16 B x world over the fabric (<= 1 MB
at T = 5000) -- latency-bound, so it is ONE collective, not one per iteration
or per array.  The solve itself has no data-path collective.

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

    Each rank owns one float64 block of `block_len` values: its snapshots
    [per, stride] (rows past its dates stay NaN) and, at `hdr_off`, the 16-byte cvq
    Header viewed as int64[2].
    local(hdr, snaps): solve this rank's block into those two views.
    finalize(blocks, var): full VaR vector from the gathered blocks [world, block_len].
    check(): optional convergence check after the finalize (raises on failure).
    """

    def __init__(self, T_total: int, stride: int, local: Callable, finalize: Callable,
                 device: torch.device, group=None, check: Optional[Callable] = None,
                 block_len: Optional[int] = None, hdr_off: Optional[int] = None):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.T_total = int(T_total)
        self.lo, self.hi, self.per = shard(self.T_total, self.rank, self.world)
        self.stride = int(stride)
        self._local, self._finalize, self._check = local, finalize, check
        if hdr_off is None:                                   # snapshots, padded to 16 B, then the header
            hdr_off = (self.per * self.stride + 1) & ~1
        self.hdr_off = int(hdr_off)
        self.block_len = int(block_len if block_len is not None else self.hdr_off + 2)
        self.block = torch.full((self.block_len,), float("nan"), dtype=torch.float64, device=device)
        self.snaps = self.block[: self.per * self.stride].view(self.per, self.stride)
        self.hdr = self.block[self.hdr_off: self.hdr_off + 2].view(torch.int64)
        self.hdr.zero_()
        self.var = torch.empty(self.T_total, dtype=torch.float64, device=device)

    def solve_local(self) -> None:
        """This rank's part of solve() alone: its block's local solve, no exchange (timing)."""
        self._local(self.hdr, self.snaps)

    def solve(self, check: bool = True) -> torch.Tensor:
        """Full VaR vector on every rank.  check: verify convergence within the
        bisection budget after the finalize (synchronises; the status is global, from
        the gathered headers, so every rank raises together)."""
        self._local(self.hdr, self.snaps)
        # a process group of one still takes the collective (the path every N > 1 run takes)
        blocks = (self.block.view(1, -1) if not dist.is_initialized()
                  else _gather(self.block.view(1, -1), self.world, self.group))
        self._finalize(blocks, self.var)
        if check and self._check is not None:
            self._check()
        return self.var


def device_sharded_var(plan, args, T_total: int, device: torch.device, group=None) -> ShardedVaR:
    """ShardedVaR wired to a QuadraturePlan's device entry points (plan holds this rank's block).

    The plan is bound to torch's current stream at every solve, so its kernels, the
    snapshot buffers' initialisation and the collectives are ordered on one stream."""
    stride = plan.snap_stride(args)
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    per = shard(T_total, 0, world)[2]
    block_len, hdr_off = plan.packed_block_len(args, per)     # the library's packed layout

    def local(hdr, snaps):
        plan.set_stream(torch.cuda.current_stream(device).cuda_stream)
        plan.solve_local(args, hdr.data_ptr(), snaps.data_ptr())

    def finalize(blocks, var):
        plan.solve_finalize_packed(args, blocks.data_ptr(), world, per, T_total, var.data_ptr())

    return ShardedVaR(T_total, stride, local, finalize, device, group, check=plan.solve_status,
                      block_len=block_len, hdr_off=hdr_off)
