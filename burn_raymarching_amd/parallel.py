"""View-sharded data parallelism for the training step.

One process per GPU. Rays are independent and every ray does identical work, so whole views
shard across ranks with perfect balance. The only data-path collective is one sum all-reduce
of the packed activated-space gradient [centers 3M | colors 3M | radius M | light 3 |
ambient 1] (7M+4 floats, 28 KB at M=256), plus the 1-float loss: latency-bound messages, so
RCCL's ring over xGMI is used as is. The loss is normalised by the GLOBAL ray count inside the
kernel (inv_count = 1/(3 N_global)), so the summed gradient equals the single-process
gradient of the mean loss. The compute_loss penalties and Adam run replicated AFTER the
all-reduce (identical on every rank), so they are not multiplied by the world size.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Sequence

import torch


@dataclass
class Shard:
    """Which views a rank renders at a step.

    Weak scaling (global_views == 0): every rank renders `views_per_rank` views per step, so the
    step covers views_per_rank * world views. Strong scaling (global_views = V > 0): a step covers
    V views in all, split into contiguous parts over the ranks (V // world each, the first
    V % world ranks one more), so the work per step is fixed as the world grows."""
    rank: int
    world: int
    views_per_rank: int
    ring: int  # number of cameras in the rotation
    global_views: int = 0

    def count(self, rank: int | None = None) -> int:
        """Views per step of `rank` (default: this rank)."""
        r = self.rank if rank is None else rank
        if self.global_views <= 0:
            return self.views_per_rank
        base, extra = divmod(self.global_views, self.world)
        return base + (1 if r < extra else 0)

    @property
    def views_total(self) -> int:
        """Views per step over all ranks."""
        return self.global_views if self.global_views > 0 else self.views_per_rank * self.world

    def views(self, step: int) -> list[int]:
        """Views of this rank at `step`: a contiguous block of the ring, rotating every step."""
        if self.global_views <= 0:
            first = ((step * self.world + self.rank) * self.views_per_rank) % self.ring
            n = self.views_per_rank
        else:
            start = sum(self.count(r) for r in range(self.rank))
            first = (step * self.global_views + start) % self.ring
            n = self.count()
        return [(first + j) % self.ring for j in range(n)]


class ViewShardedStep:
    """One data-parallel training step.

    step_fn(views, inv_count, grads_out, loss_out) computes this rank's contribution (the
    fused forward + loss seed + backward over its views) into the packed gradient buffer and
    the loss-sum scalar; the default for training is rm_train_step_camera (see bench.py /
    train). optim_fn(grads) applies the replicated optimizer step.
    """

    def __init__(self, shard: Shard, rays_per_view: int, num_params: int, device,
                 step_fn: Callable[[Sequence[int], float, torch.Tensor, torch.Tensor], None],
                 optim_fn: Callable[[torch.Tensor], None] | None = None, group=None, collective: bool = True):
        self.shard = shard
        # collective=False: one process runs one rank's share of a world-size-N step alone (its
        # views and the global ray count, no all-reduce: bench.py --as-rank)
        self.collective = collective
        self.rays_global = rays_per_view * shard.views_total
        self.inv_count = 1.0 / (3.0 * self.rays_global)
        # one buffer, one collective: [packed gradient | loss sum]
        self.buf = torch.zeros(num_params + 1, device=device)
        self.grads = self.buf[:num_params]
        self.loss = self.buf[num_params:]
        self.step_fn = step_fn
        self.optim_fn = optim_fn
        self.group = group
        # time_allreduce: hipEvents on the compute stream around the all-reduce of the next steps
        # (the collective plus the wait for the slowest rank), read by collect_allreduce_ms()
        self.time_allreduce = False
        self._ar_events = []

    def __call__(self, step: int) -> None:
        views = self.shard.views(step)
        self.step_fn(views, self.inv_count, self.grads, self.loss)
        if self.shard.world > 1 and self.collective:
            import torch.distributed as dist
            if self.time_allreduce:
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ev[0].record()
            dist.all_reduce(self.buf, group=self.group)
            if self.time_allreduce:
                ev[1].record()
                self._ar_events.append(ev)
        if self.optim_fn is not None:
            self.optim_fn(self.grads)

    def collect_allreduce_ms(self, reset: bool = True):
        """Mean ms per timed all-reduce since the last reset (None if none was timed)."""
        if not self._ar_events:
            return None
        torch.cuda.synchronize()
        ms = [a.elapsed_time(b) for a, b in self._ar_events]
        if reset:
            self._ar_events = []
        return sum(ms) / len(ms)

    def mean_loss(self) -> float:
        """Reconstruction loss (training.rs:34 mean) of the last step, over all ranks."""
        return float(self.loss.item()) * self.inv_count
