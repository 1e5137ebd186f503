"""Ensemble / MC-dropout uncertainty metrics (test infrastructure only).

North-star metrics; the reference has none of them in code.
Conventions follow the reference's analysis code: per-member softmax, then mean
over members (notebooks/food101_robustness.py:25-36, notebooks/utils.py:22-23).

* probs_mean(logits[S..., C])  mean over every leading "member/pass" axis of softmax
* nll(p_bar, y)      -mean_i log p_bar[i, y_i]     (at K=T=1 equals the reference
                                                   CrossEntropyLoss, src/mmbt.py:243)
* ece(p_bar, y, 15)  equal-width confidence bins on max p_bar (build-defined; "parity unpinned")
"""
import numpy as np


def softmax(z, axis=-1):
    z = np.asarray(z, dtype=np.float64)
    z = z - z.max(axis=axis, keepdims=True)
    e = np.exp(z)
    return e / e.sum(axis=axis, keepdims=True)


def probs_mean(logits, member_axes=(0,)):
    return softmax(logits).mean(axis=tuple(member_axes))


def nll(p_bar, y, floor=1e-12):
    p = p_bar[np.arange(len(y)), np.asarray(y)]
    return float(-np.log(np.maximum(p, floor)).mean())


def ece(p_bar, y, n_bins=15):
    conf = p_bar.max(axis=1)
    pred = p_bar.argmax(axis=1)
    correct = (pred == np.asarray(y)).astype(np.float64)
    # bin b holds conf in (b/n, (b+1)/n]; conf == 0 falls in bin 0
    b = np.clip(np.ceil(conf * n_bins).astype(np.int64) - 1, 0, n_bins - 1)
    tot = 0.0
    N = len(conf)
    for k in range(n_bins):
        sel = b == k
        if sel.any():
            tot += sel.sum() / N * abs(correct[sel].mean() - conf[sel].mean())
    return float(tot)


def accuracy(p_bar, y):
    return float((p_bar.argmax(1) == np.asarray(y)).mean())
