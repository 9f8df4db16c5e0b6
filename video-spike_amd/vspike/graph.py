"""One train step replayed as a hipGraph: `Trainer.step` (src/trainer/base.py:144-159) with its
~330 launches captured once and re-issued by a single `hipGraphLaunch` per step.

Why: the eager step enqueues ~330 kernels from Python (autograd, ctypes, the optimizer's per-step
rows); on a slower host or under a tracer the GPU idles between the backward's last kernel, the
optimizer and the next forward (profiles/r03_v2_timeline.txt: 0.5-1.0 ms per 6.4-ms step under
rocprofv3).  A replay keeps the GPU's queue full with ~20 us of host work per step.

What changes versus the eager step: nothing in the arithmetic — the same kernels with the same
operands run in the same stream order (the weight-gradient side stream is forked and joined by
events, which capture as graph edges).  Host-side state moves per replay exactly as `step` moves
it: FusedAdamW.stage counts the step and sends the scheduler's lr + bias-correction step into the
captured hyper-parameter block before the replay; the scheduler steps after it.

Contract (as torch.cuda.graphs' whole-network capture):
  * the model, optimizer state, activation arenas and bf16 shadows exist before capture (run at
    least one eager `Trainer.step` first — the bench's warm-up does);
  * inputs/targets are copied into the captured tensors when a different tensor is passed;
  * the loss returned by `step` is a fresh device scalar per step, like the eager step's;
  * single process (no data-parallel exchange inside the graph; `Trainer` with `exchange=None`).
"""
from __future__ import annotations

import torch

from .optim import FusedAdamW


class GraphedStep:
    def __init__(self, trainer, inputs: torch.Tensor, target: torch.Tensor):
        if trainer.exchange is not None:
            raise ValueError("GraphedStep: the data-parallel exchange is not captured; run the eager step")
        if not isinstance(trainer.optimizer, FusedAdamW):
            raise TypeError("GraphedStep needs vspike.optim.FusedAdamW (its update reads a captured hyper block)")
        if not inputs.is_cuda:
            raise ValueError("GraphedStep runs on the GPU only")
        self.trainer = trainer
        self.inputs, self.target = inputs, target
        opt, model = trainer.optimizer, trainer.model
        # EVERY trainable parameter needs its Adam moments before capture: state created lazily inside
        # the capture would live in the graph pool and be re-zeroed by every replay
        missing = [p for grp in opt.param_groups for p in grp["params"]
                   if p.requires_grad and not opt.state.get(p)]
        if missing:
            raise RuntimeError(f"GraphedStep: {len(missing)} trainable parameter(s) have no optimizer state; run one "
                               "eager Trainer.step first (optimizer state, arenas, shadows)")
        # allocated outside the capture: a tensor made inside it would be re-zeroed by every replay
        self.hyper = opt.static_hyper()
        torch.cuda.synchronize()
        opt.zero_grad(set_to_none=True)     # the captured backward installs the graph's own .grad
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):  # captured on torch's internal side stream
            out = model(self.inputs)
            loss = trainer.criterion(out, self.target)
            loss.backward()
            opt.launch_static(self.hyper)
            self.loss = loss.detach()
        self.out = out.detach()

    def step(self, inputs: torch.Tensor = None, target: torch.Tensor = None) -> torch.Tensor:
        if inputs is not None and inputs is not self.inputs:
            self.inputs.copy_(inputs)
        if target is not None and target is not self.target:
            self.target.copy_(target)
        tr = self.trainer
        tr.optimizer.stage(self.hyper)
        self.graph.replay()
        if tr.lr_scheduler is not None:
            tr.lr_scheduler.step()
        return self.loss.clone()
