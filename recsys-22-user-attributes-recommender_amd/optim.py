"""FusedAdam: torch.optim.Adam semantics on the gfx950 multi-tensor Adam kernel.

Matches the optimizers the reference modules build (core/modules/*_training_module.py:
configure_optimizers -> torch.optim.Adam(lr, betas, weight_decay) with L2-coupled decay):
one launch updates every dense parameter; the item table, when its gradient arrives as a
row-sparse `SparseTablePlan`, gets the exact dense update from the compact rows
(asme_adam_rows_step) without ever materialising a dense (V, d) gradient.
"""
from __future__ import annotations

import ctypes

import torch

from ._lib import call, ptr, stream
from . import ops
from .ops import LazyTableState


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0,
                 lazy_table: bool = True, fused_apply: bool = True, rest_rows: bool = True):
        """lazy_table: the item table's exact lazy Adam (False: every row's update from the compact rows each step);
        fused_apply: its table gradient reduced and applied in one pass; rest_rows: a fresh table without weight
        decay starts with its rows at rest.  The last three are bit-identical A/B forms of the same update."""
        if lr < 0.0 or eps < 0.0 or weight_decay < 0.0:
            raise ValueError("invalid Adam hyper-parameter")
        super().__init__(params, dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay))
        self.lazy_table = lazy_table
        self.fused_apply = fused_apply
        self.rest_rows = rest_rows

    def flush(self):
        """Bring lazily-updated item tables fully up to date (exact dense-Adam state)."""
        for group in self.param_groups:
            for p in group["params"]:
                tg = getattr(p, "_asme_table_grad", None)
                if tg is not None and tg.lazy is not None:
                    tg.lazy.flush()

    def zero_grad(self, set_to_none: bool = True):
        """as torch's, and for a row-sparse item table: drops the applied plan (the kept ".grad" a step without a new
        backward would reuse) and a pending plan whose backward ran but whose optimizer step was skipped (GradScaler's
        inf/NaN skip, a trainer skipping the step) -- the one signal that a table gradient is to be discarded.  A
        plan that has no gradient yet (zero_grad between training_step and backward, Lightning's closure order)
        is kept."""
        super().zero_grad(set_to_none=set_to_none)
        for group in self.param_groups:
            for p in group["params"]:
                tg = getattr(p, "_asme_table_grad", None)
                if tg is not None:
                    tg.drop_applied()
                    if tg.plan is not None and not tg.plan.consumed and tg.plan.has_gradient():
                        tg.plan.release()
                        tg.plan = None

    def state_dict(self):
        """flush first: lazily-deferred table rows must be current in the saved moments"""
        self.flush()
        return super().state_dict()

    def load_state_dict(self, state_dict):
        """flush, then drop every lazy table state: it holds references to the old moment tensors and the
        old step; it is rebuilt from the loaded state at the next sparse step"""
        self.flush()
        for group in self.param_groups:
            for p in group["params"]:
                tg = getattr(p, "_asme_table_grad", None)
                if tg is not None:
                    tg.lazy = None
                    if tg.plan is not None:  # rows staged from the old state: the loaded state is current
                        tg.plan.staged = None
        super().load_state_dict(state_dict)
        for st in self.state.values():  # torch may restore `step` as a tensor; the kernels take an int
            if "step" in st and torch.is_tensor(st["step"]):
                st["step"] = int(st["step"].item())

    def _state(self, p):
        st = self.state[p]
        if not st:
            st["step"] = 0
            st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
        return st

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        ops.note_param_write()  # (the kernels below write the parameters behind torch's version counter)
        for group in self.param_groups:
            b1, b2 = group["betas"]
            lr, eps, wd = float(group["lr"]), float(group["eps"]), float(group["weight_decay"])
            by_step = {}
            for p in group["params"]:
                tg = getattr(p, "_asme_table_grad", None)
                plan = tg.plan if tg is not None else None
                reapply = plan is None and tg is not None and tg.applied is not None and p.grad is None
                if reapply:  # a step without a new backward: the last gradient again, like a kept .grad
                    plan = tg.applied
                if plan is not None:
                    if p.grad is not None:
                        raise RuntimeError("item table got a dense gradient while its sparse plan is active "
                                           "(tied / full-catalogue heads need table_grad='dense')")
                    fresh = not self.state[p]  # moments created now: all +0
                    st = self._state(p)
                    st["step"] += 1
                    V, D = p.shape
                    if self.lazy_table:
                        if tg.lazy is None:
                            tg.lazy = LazyTableState(p, st["exp_avg"], st["exp_avg_sq"])
                            tg.lazy.start(st["step"] - 1, fresh, wd, self.rest_rows)  # every row current up to now
                        elif reapply:  # no forward caught these rows up this time
                            tg.lazy.catch_up(plan.unique, plan.count, plan.capacity)
                        tg.lazy.record(st["step"], lr, b1, b2, eps, wd)
                        tg.lazy.apply(plan, st["step"], self.fused_apply)
                    else:
                        call("asme_adam_rows_step", ptr(p), ptr(st["exp_avg"]), ptr(st["exp_avg_sq"]), V, D,
                             ptr(plan.row_slot_map()), ptr(plan.grad_rows), lr, b1, b2, eps, wd, st["step"], stream())
                    tg.applied = plan
                    tg.plan = None
                    continue
                if p.grad is None:
                    continue
                if tg is not None and tg.lazy is not None:  # switching back to dense gradients
                    tg.lazy.flush()
                    tg.lazy = None
                if p.grad.is_sparse:
                    raise RuntimeError("FusedAdam does not support torch sparse gradients")
                st = self._state(p)
                st["step"] += 1
                by_step.setdefault(st["step"], []).append(p)
            for step, ps in by_step.items():
                n = len(ps)
                arr = ctypes.c_void_p * n
                P = arr(*[ptr(p) for p in ps])
                for p in ps:
                    if not p.grad.is_contiguous():
                        p.grad = p.grad.contiguous()
                G = arr(*[ptr(p.grad) for p in ps])
                M = arr(*[ptr(self.state[p]["exp_avg"]) for p in ps])
                Vv = arr(*[ptr(self.state[p]["exp_avg_sq"]) for p in ps])
                N = (ctypes.c_int64 * n)(*[p.numel() for p in ps])
                call("asme_adam_step", n, P, G, M, Vv, N, lr, b1, b2, eps, wd, step, stream())
        return loss
