"""The training step of `src/trainer/base.py:144-159`, re-stated for the HIP path.

    outputs = model(inputs); loss = criterion(outputs, ap); loss.backward()
    [all-reduce of gradients]; optimizer.step(); lr_scheduler.step(); optimizer.zero_grad()

Differences by design: the loss stays on the device (the reference's per-step `loss.item()`,
base.py:154, is a host sync — `train_epoch` here collects device scalars and syncs once per
epoch), and the data-parallel exchange is vspike.dp.GradExchange instead of DDP hooks.
"""
from __future__ import annotations

from typing import Iterable, List, Optional

import torch

from .dp import GradExchange
from .loss import make_criterion
from .metrics import eval_session
from .optim import FusedAdamW


def input_modalities(config) -> List[str]:
    """`src/trainer/base.py:8-14`."""
    mods = config["data"]["modalities"]
    return [m for m in mods if mods[m]["input"]]


def model_inputs(config, batch):
    """`src/trainer/base.py:61-70`: Linear -> cat of flattened input modalities, else video."""
    if config["model"]["model_class"] == "Linear":
        return torch.cat([batch[m].flatten(1) for m in input_modalities(config)], dim=-1)
    return batch["video"]


def build_optimizer(model, config, total_steps: int, world: int = 1):
    """`src/train.py:44-57`: AdamW(lr, wd, eps) + OneCycleLR(max_lr=lr, pct_start, div_factor)."""
    o = config["optimizer"]
    opt = FusedAdamW([p for p in model.parameters() if p.requires_grad], lr=float(o["lr"]),
                     weight_decay=float(o["wd"]), eps=float(o["eps"]), grad_scale=1.0 / world)
    sched = torch.optim.lr_scheduler.OneCycleLR(optimizer=opt, total_steps=max(1, total_steps), max_lr=float(o["lr"]),
                                                pct_start=float(o["warmup_pct"]),
                                                div_factor=float(o["div_factor"]))
    return opt, sched


class Trainer:
    def __init__(self, model, optimizer, lr_scheduler=None, config=None, criterion=None,
                 exchange: Optional[GradExchange] = None):
        """criterion: default = the config's `training.loss` (make_criterion: "poisson", the
        reference's PoissonNLL of src/train.py:59, or "mse")."""
        self.model, self.optimizer, self.lr_scheduler = model, optimizer, lr_scheduler
        self.config, self.exchange = config, exchange
        self.criterion = criterion if criterion is not None else make_criterion(config)

    def step(self, inputs, target) -> torch.Tensor:
        outputs = self.model(inputs)
        loss = self.criterion(outputs, target)
        loss.backward()
        if self.exchange is not None:
            self.exchange.finish()
        self.optimizer.step()
        if self.lr_scheduler is not None:
            self.lr_scheduler.step()
        self.optimizer.zero_grad(set_to_none=True)
        return loss.detach()

    def train_epoch(self, batches: Iterable) -> float:
        self.model.train()
        losses = [self.step(model_inputs(self.config, b) if self.config else b["video"], b["ap"]) for b in batches]
        return float(torch.stack(losses).mean().item()) if losses else float("nan")

    @torch.no_grad()
    def eval_epoch(self, batches: Iterable, metrics=("bps", "rsquared")) -> dict:
        """`src/trainer/base.py:161-206`: per batch the loss; per session (`batch['eid'][0]`) the
        concatenated gt / log-rate outputs go through `metrics_list` (exp fused, on the device).
        Returns the reference's `eval_res` dict: eval_loss and eval_<metric>, each rounded to 5
        places as base.py:198,203 does."""
        import numpy as np
        self.model.eval()
        losses, sessions = [], {}
        for b in batches:
            out = self.model(model_inputs(self.config, b) if self.config else b["video"])
            losses.append(self.criterion(out, b["ap"]))
            eid = b["eid"][0] if "eid" in b else "session"
            s = sessions.setdefault(eid, {"gt": [], "preds": []})
            s["gt"].append(b["ap"])
            s["preds"].append(out)
        res = {k: [] for k in metrics}
        for s in sessions.values():
            r = eval_session(torch.cat(s["gt"], 0), torch.cat(s["preds"], 0), metrics)
            for k, v in r.items():
                res[k].append(v)
        out = {"eval_loss": round(float(np.mean([float(x) for x in losses])), 5) if losses else float("nan")}
        out.update({f"eval_{k}": round(float(np.mean(v)), 5) for k, v in res.items()})
        return out
