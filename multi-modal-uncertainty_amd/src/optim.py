"""BertAdam with the pytorch_pretrained_bert 0.6.x interface (train.py:16,142-147).

``BertAdam(params, lr, warmup=-1, t_total=-1, schedule='warmup_linear', b1=0.9,
b2=0.999, e=1e-6, weight_decay=0.01, max_grad_norm=1.0)``; per-param state keys
``step`` / ``next_m`` / ``next_v``; ``ReduceLROnPlateau`` drives ``group['lr']``.

When every parameter lives in one MMBT ParamStore on the GPU (the hot path) the
step is ONE fused multi-tensor HIP launch sequence (mmu_bertadam_step) over the
flat f32 buffers, which also refreshes the bf16 GEMM weight copies.  Other
parameter sets (e.g. small CPU models driven by the framework tests) take the
per-tensor torch loop below, which restates the same update.
"""
import torch

from . import kernels as K
from .params import STORES

CHUNK = 65536


def warmup_linear(x, warmup=0.002):
    if x < warmup:
        return x / warmup
    return max((x - 1.0) / (warmup - 1.0), 0.0)


SCHEDULES = {"warmup_linear": warmup_linear}


def _sched(step, group):
    t_total = group["t_total"]
    if t_total is None or t_total < 0:
        return 1.0
    return SCHEDULES[group["schedule"]](float(step) / t_total, group["warmup"])


class BertAdam(torch.optim.Optimizer):
    def __init__(self, params, lr, warmup=-1, t_total=-1, schedule="warmup_linear", b1=0.9, b2=0.999, e=1e-6,
                 weight_decay=0.01, max_grad_norm=1.0):
        if lr < 0.0:
            raise ValueError(f"Invalid learning rate: {lr}")
        if schedule not in SCHEDULES:
            raise ValueError(f"Invalid schedule parameter: {schedule}")
        if not 0.0 <= warmup < 1.0 and warmup != -1:
            raise ValueError(f"Invalid warmup: {warmup}")
        defaults = dict(lr=lr, schedule=schedule, warmup=warmup, t_total=t_total, b1=b1, b2=b2, e=e,
                        weight_decay=weight_decay, max_grad_norm=max_grad_norm)
        super().__init__(params, defaults)
        self._fused = None
        self._fused_key = None
        self._host_steps_valid = True
        # factor on the gradients of the NEXT step only (then back to 1): data parallelism's
        # 1/world, set by dp.GradBucketer.finish() instead of scaling the summed gradients in a
        # separate pass (the fused kernel folds it into the clip coefficient)
        self.grad_scale = 1.0

    # ------------------------------------------------------------------ fused path setup
    def _find_store(self):
        ps = [p for g in self.param_groups for p in g["params"]]
        if not ps or not all(p.is_cuda for p in ps):
            return None
        for st in list(STORES):
            if st.flat is None or st.flat.device != ps[0].device:
                continue
            base, end = st.flat.data_ptr(), st.flat.data_ptr() + 4 * st.numel()
            if all(base <= p.data_ptr() < end for p in ps):
                return st
        return None

    def _layout_key(self):
        p = self.param_groups[0]["params"][0]
        return (p.device, p.data_ptr())

    def _ensure_fused(self):
        """(Re)build the fused state when the parameters moved (Module.to rebuilds the store)."""
        key = self._layout_key()
        if key != self._fused_key:
            if self._fused is not None:  # keep moments across a move: hand them back as per-param state
                self._sync_steps()
                for p in list(self.state):
                    s = self.state[p]
                    if "next_m" in s:
                        s["next_m"], s["next_v"] = s["next_m"].clone(), s["next_v"].clone()
            self._fused = None
            self._build_fused()
            self._fused_key = key

    def _build_fused(self):
        st = self._find_store()
        if st is None:
            return
        decay = [g for g in self.param_groups if g["weight_decay"] > 0]
        nodecay = [g for g in self.param_groups if g["weight_decay"] <= 0]
        if len(decay) > 1 or len(nodecay) > 1:
            return
        g0 = self.param_groups[0]
        for g in self.param_groups:
            for k in ("schedule", "warmup", "t_total", "b1", "b2", "e", "max_grad_norm"):
                if g[k] != g0[k]:
                    return
        group_of = {}
        for g in self.param_groups:
            for p in g["params"]:
                group_of[id(p)] = 0 if g["weight_decay"] > 0 else 1
        names = [n for n in st.names if id(st.params[n]) in group_of]
        dev = st.device
        m = torch.zeros_like(st.flat)
        v = torch.zeros_like(st.flat)
        host_steps = [0] * len(names)
        for i, n in enumerate(names):  # carry over state loaded via load_state_dict / earlier generic steps
            p = st.params[n]
            s = self.state.get(p, {})
            o, k = st.offsets[n], p.numel()
            if "next_m" in s:
                st._shaped(m, o, p).copy_(s["next_m"])
                st._shaped(v, o, p).copy_(s["next_v"])
                host_steps[i] = int(s["step"])
        steps = torch.tensor(host_steps, dtype=torch.int32).to(dev)
        self._fused = dict(store=st, names=names, m=m, v=v, steps=steps, group_of=group_of, active=None,
                           table=None, n_chunks=0, ws=None, flat_grad_owned=len(names) == len(st.names))
        for i, n in enumerate(names):
            p = st.params[n]
            o, k = st.offsets[n], p.numel()
            # same element layout as the parameter view (conv weights are channels-last in the flat buffer)
            self.state[p] = {"step": host_steps[i], "next_m": st._shaped(m, o, p), "next_v": st._shaped(v, o, p)}
        self._host_steps_valid = True

    def _table(self):
        f = self._fused
        st = f["store"]
        active = tuple(bool(st.params[n].requires_grad) for n in f["names"])
        if active == f["active"]:
            return
        rows, chunks = [], []
        for t, n in enumerate(f["names"]):
            p = st.params[n]
            k = p.numel()
            first = len(chunks)
            for s in range(0, k, CHUNK):
                chunks.append((t, s, min(CHUNK, k - s)))
            bo = st.coffsets.get(n, -1)
            rows.append((st.offsets[n], k, f["group_of"][id(p)], bo, int(active[t]), first, len(chunks) - first))
        flat = [x for r in rows for x in r] + [x for c in chunks for x in c]
        f["table"] = torch.tensor(flat, dtype=torch.int64).to(st.device)
        f["n_chunks"] = len(chunks)
        f["ws"] = torch.empty(len(chunks) + 2 * len(rows), dtype=torch.float32, device=st.device)
        f["active"] = active

    # ------------------------------------------------------------------ API
    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        self._ensure_fused()
        if self._fused is not None:
            self._step_fused()
        else:
            self._step_generic()
        return loss

    def _step_fused(self):
        f = self._fused
        st = f["store"]
        self._table()
        lr_decay = lr_nodecay = 0.0
        wd = 0.0
        for g in self.param_groups:
            if g["weight_decay"] > 0:
                lr_decay, wd = g["lr"], g["weight_decay"]
            else:
                lr_nodecay = g["lr"]
        g0 = self.param_groups[0]
        t_total = g0["t_total"] if g0["t_total"] is not None else -1
        K.bertadam_step(st.flat, st.grad, f["m"], f["v"], st.compute, f["table"], f["steps"], len(f["names"]),
                        f["n_chunks"], lr_decay, lr_nodecay, wd, g0["warmup"], t_total, g0["b1"], g0["b2"], g0["e"],
                        g0["max_grad_norm"], f["ws"], grad_scale=self.grad_scale)
        self.grad_scale = 1.0
        st.sync_transposed()  # the K-major bf16 weight copies the data-gradient GEMMs read
        self._host_steps_valid = False

    def _step_generic(self):
        for group in self.param_groups:
            for p in group["params"]:
                if p.grad is None:
                    continue
                grad = p.grad if self.grad_scale == 1.0 else p.grad * self.grad_scale
                state = self.state[p]
                if len(state) == 0:
                    state["step"] = 0
                    state["next_m"] = torch.zeros_like(p)
                    state["next_v"] = torch.zeros_like(p)
                m, v = state["next_m"], state["next_v"]
                if group["max_grad_norm"] > 0:
                    n = grad.norm()
                    coef = group["max_grad_norm"] / (n + 1e-6)
                    if coef < 1:
                        grad = grad * coef
                m.mul_(group["b1"]).add_(grad, alpha=1 - group["b1"])
                v.mul_(group["b2"]).addcmul_(grad, grad, value=1 - group["b2"])
                update = m / (v.sqrt() + group["e"])
                if group["weight_decay"] > 0.0:
                    update = update + group["weight_decay"] * p
                p.add_(update, alpha=-group["lr"] * _sched(state["step"], group))
                state["step"] += 1
        self.grad_scale = 1.0

    def zero_grad(self, set_to_none=False):
        self._ensure_fused()
        f = self._fused
        if f is not None and f["flat_grad_owned"]:
            f["store"].zero_grad()
            return
        for g in self.param_groups:
            for p in g["params"]:
                if p.grad is not None:
                    if set_to_none and f is None:
                        p.grad = None
                    else:
                        p.grad.zero_()

    def _sync_steps(self):
        f = self._fused
        if f is None or self._host_steps_valid:
            return
        st = f["store"]
        host = f["steps"].cpu().tolist()
        for n, s in zip(f["names"], host):
            self.state[st.params[n]]["step"] = int(s)
        self._host_steps_valid = True

    def state_dict(self):
        self._sync_steps()
        return super().state_dict()

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self._fused, self._fused_key = None, None  # rebuilt from the loaded state at the next step

    def get_lr(self):
        """Scheduled lr of every parameter (pytorch_pretrained_bert BertAdam.get_lr)."""
        self._sync_steps()
        lr = []
        for group in self.param_groups:
            for p in group["params"]:
                state = self.state[p]
                lr.append(0 if len(state) == 0 else group["lr"] * _sched(state["step"], group))
        return lr
