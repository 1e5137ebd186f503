"""BertAdam restatement (test infrastructure only).

The reference constructs ``pytorch_pretrained_bert.BertAdam(groups, lr, warmup, t_total)``
at train.py:142-147 with the default schedule 'warmup_linear', b1 0.9, b2 0.999,
e 1e-6, max_grad_norm 1.0, and weight-decay groups 0.01 / 0.0 split by name
(train.py:137-141).  pytorch_pretrained_bert (0.6.x) is not vendored or installed;
this follows its published algorithm:

    for each param p with grad g:                        (per tensor, not global)
        g <- g * min(1, max_grad_norm / (||g||_2 + 1e-6))  # clip_grad_norm_(p, 1.0)
        m <- b1*m + (1-b1)*g ;  v <- b2*v + (1-b2)*g*g
        u <- m / (sqrt(v) + e)  + wd * p                   # no bias correction
        p <- p - lr * sched(step / t_total) * u            # step BEFORE increment
        step += 1
    sched = warmup_linear(x, w): x/w if x < w else max((x-1)/(w-1), 0)

Parity: "unpinned" beyond that formula (no executable BertAdam exists offline).
"""
import torch


def warmup_linear(x, warmup):
    if x < warmup:
        return x / warmup
    return max((x - 1.0) / (warmup - 1.0), 0.0)


def schedule_factor(step, warmup, t_total):
    if t_total is None or t_total < 0:
        return 1.0
    return warmup_linear(float(step) / t_total, warmup)


def bertadam_step(params, grads, ms, vs, steps, lr, wds, warmup, t_total,
                  b1=0.9, b2=0.999, eps=1e-6, max_grad_norm=1.0):
    """In-place fp32 update of lists of tensors; ``steps`` is a list of ints (returned +1)."""
    new_steps = []
    for p, g, m, v, st, wd in zip(params, grads, ms, vs, steps, wds):
        g = g.clone()
        if max_grad_norm > 0:
            n = g.double().norm().item()
            coef = max_grad_norm / (n + 1e-6)
            if coef < 1.0:
                g.mul_(coef)
        m.mul_(b1).add_(g, alpha=1 - b1)
        v.mul_(b2).addcmul_(g, g, value=1 - b2)
        upd = m / (v.sqrt() + eps)
        if wd > 0.0:
            upd = upd + wd * p
        p.add_(-(lr * schedule_factor(st, warmup, t_total)) * upd)
        new_steps.append(st + 1)
    return new_steps
