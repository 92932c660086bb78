"""Fused flat-arena optimizers (Adam, SGD+momentum).

The reference builds ``torch.optim.Adam(model.parameters(), lr=utils.LR)``
(``/root/reference/main.py:125``) and steps it after the gradient average
(``main.py:155``).  Here the whole update is ONE streaming HIP kernel over the flat
fp32 master / gradient / moment buffers of :class:`~mpi_pytorch_amd.parallel.ParamArena`:
it applies the DP ``1/N`` gradient scale, weight decay, the Adam (or SGD-momentum)
update, and writes the bf16 weight shadow that the MFMA kernels read - one HBM pass
instead of per-tensor launches plus a cast pass.

``state_dict()`` / ``load_state_dict()`` speak ``torch.optim.Adam`` / ``torch.optim.SGD``
format exactly (per-parameter ``exp_avg``/``exp_avg_sq``/``step`` or ``momentum_buffer``
in the torchvision layout, ``param_groups`` with ``params`` = indices into
``model.parameters()``), so checkpoints round-trip with the reference's
``helpers.load_checkpoint`` (``helpers.py:10-15``).
"""
from __future__ import annotations

from typing import Dict, List

import torch
import torch.nn as nn

from .ops import functional as Fn
from .parallel.arena import ParamArena


def _export(p, t):
    f = getattr(p, "_mpa_export", None)
    return f(t) if f is not None else t


def _import(p, t):
    f = getattr(p, "_mpa_import", None)
    return f(t) if f is not None else t


class _FlatOptimizer:
    kind = "base"

    def __init__(self, params: List[nn.Parameter], arena: ParamArena):
        self.params = list(params)
        self.arena = arena
        dev = arena.device
        self.step_t = torch.zeros(1, dtype=torch.float32, device=dev)
        self.grad_scale = 1.0
        self.param_groups = [self._group_defaults()]
        self.param_groups[0]["params"] = self.params

    # torch.optim-like surface ------------------------------------------------------
    def zero_grad(self, set_to_none: bool = False) -> None:
        self.arena.zero_grad()

    @property
    def lr(self) -> float:
        return self.param_groups[0]["lr"]

    @lr.setter
    def lr(self, v: float) -> None:
        self.param_groups[0]["lr"] = v

    def _group_defaults(self) -> Dict:
        raise NotImplementedError

    def _update(self, lo: int, hi: int) -> None:
        raise NotImplementedError

    def _kernel(self):
        return Fn.K(self.arena.master)

    def _shadow(self):
        s = self.arena.train_shadow()
        return s if s is not None else torch.empty(0, device=self.arena.device)

    def state_dict(self) -> Dict:
        state = {}
        torch_step = float(self.step_t.item())
        for i, p in enumerate(self.params):
            if not p.requires_grad or torch_step == 0:
                continue
            o, e = self.arena.slice_of(p)
            state[i] = self._param_state(p, o, e, torch_step)
        g = {k: v for k, v in self.param_groups[0].items() if k != "params"}
        g["params"] = list(range(len(self.params)))
        return {"state": state, "param_groups": [g]}

    def load_state_dict(self, sd: Dict) -> None:
        g = sd["param_groups"][0]
        for k, v in g.items():
            if k != "params":
                self.param_groups[0][k] = v
        steps = []
        for i, st in sd["state"].items():
            p = self.params[int(i)]
            if not p.requires_grad:
                continue
            o, e = self.arena.slice_of(p)
            steps.append(self._load_param_state(p, o, e, st))
        if steps:
            self.step_t.fill_(max(steps))


class FusedAdam(_FlatOptimizer):
    kind = "adam"

    def __init__(self, params, arena: ParamArena, lr=1e-3, betas=(0.9, 0.999), eps=1e-8,
                 weight_decay=0.0):
        self._init = dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay)
        super().__init__(params, arena)
        n = max(arena.n_train, 1)
        self.exp_avg = torch.zeros(n, dtype=torch.float32, device=arena.device)
        self.exp_avg_sq = torch.zeros(n, dtype=torch.float32, device=arena.device)

    def _group_defaults(self):
        d = dict(self._init)
        d.update(amsgrad=False, maximize=False, foreach=None, capturable=False,
                 differentiable=False, fused=None)
        return d

    def _update(self, lo: int, hi: int) -> None:
        g = self.param_groups[0]
        b1, b2 = g["betas"]
        sh = self._shadow()
        self._kernel().adam_step(self.arena.master[lo:hi], self.arena.grad[lo:hi],
                                 self.exp_avg[lo:hi], self.exp_avg_sq[lo:hi],
                                 sh[lo:hi] if sh.numel() else sh, self.step_t,
                                 float(g["lr"]), float(b1), float(b2), float(g["eps"]),
                                 float(g["weight_decay"]), float(self.grad_scale))

    def step(self) -> None:
        if self.arena.n_train == 0:
            return
        self._update(0, self.arena.n_train)
        self.arena.refresh_transposed(step_inc=self.step_t)

    def _param_state(self, p, o, e, step):
        return {"step": torch.tensor(step),
                "exp_avg": _export(p, self.exp_avg[o:e].view(p.shape)).detach().cpu().clone(),
                "exp_avg_sq": _export(p, self.exp_avg_sq[o:e].view(p.shape)).detach().cpu().clone()}

    def _load_param_state(self, p, o, e, st):
        self.exp_avg[o:e].copy_(_import(p, st["exp_avg"].to(self.exp_avg.device)).reshape(-1))
        self.exp_avg_sq[o:e].copy_(_import(p, st["exp_avg_sq"].to(self.exp_avg.device)).reshape(-1))
        s = st.get("step", 0)
        return float(s.item() if torch.is_tensor(s) else s)


class FusedSGD(_FlatOptimizer):
    kind = "sgd"

    def __init__(self, params, arena: ParamArena, lr=0.1, momentum=0.9, dampening=0.0,
                 weight_decay=0.0, nesterov=False):
        self._init = dict(lr=lr, momentum=momentum, dampening=dampening,
                          weight_decay=weight_decay, nesterov=nesterov)
        super().__init__(params, arena)
        self.momentum_buffer = torch.zeros(max(arena.n_train, 1), dtype=torch.float32,
                                           device=arena.device)

    def _group_defaults(self):
        d = dict(self._init)
        d.update(maximize=False, foreach=None, differentiable=False, fused=None)
        return d

    def _update(self, lo: int, hi: int) -> None:
        g = self.param_groups[0]
        sh = self._shadow()
        self._kernel().sgd_step(self.arena.master[lo:hi], self.arena.grad[lo:hi],
                                self.momentum_buffer[lo:hi], sh[lo:hi] if sh.numel() else sh,
                                self.step_t, float(g["lr"]), float(g["momentum"]),
                                float(g["dampening"]), float(g["weight_decay"]),
                                bool(g["nesterov"]), float(self.grad_scale))

    def step(self) -> None:
        if self.arena.n_train == 0:
            return
        self._update(0, self.arena.n_train)
        self.arena.refresh_transposed(step_inc=self.step_t)

    def _param_state(self, p, o, e, step):
        return {"momentum_buffer":
                _export(p, self.momentum_buffer[o:e].view(p.shape)).detach().cpu().clone()}

    def _load_param_state(self, p, o, e, st):
        mb = st.get("momentum_buffer")
        if mb is not None:
            self.momentum_buffer[o:e].copy_(_import(p, mb.to(self.momentum_buffer.device)).reshape(-1))
        return 1.0


def build_optimizer(name: str, model: nn.Module, lr: float, momentum: float = 0.9,
                    weight_decay: float = 0.0):
    arena = model._mpa_arena
    params = list(model.parameters())
    if name == "adam":
        return FusedAdam(params, arena, lr=lr, weight_decay=weight_decay)
    if name == "sgd":
        return FusedSGD(params, arena, lr=lr, momentum=momentum, weight_decay=weight_decay)
    raise ValueError(name)
