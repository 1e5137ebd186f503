"""Statistics of the attention-dropout pair draws (csrc/attention.hip pair_draw): per-key drop
rate, pairwise correlation of the 16 decisions drawn from one block hash, and the joint drop
count against Binomial(16, p).  CPU / numpy restatement of the kernel's integer arithmetic.

  python tools/dropout_draws.py [--n 22] [--p 0.1]
"""
import argparse
from math import comb

import numpy as np

MUL24 = [0x9E3779, 0x85EBCB, 0xC2B2AF, 0xA7D4EB, 0x965667, 0xD3A265, 0xFD7047, 0xB55A4F]


def pair_draw(hb, i):
    r = 4 * i
    src = ((hb >> r) | (hb << (32 - r))) & 0xFFFFFFFF if r else hb  # v_alignbit rotr
    x = ((src & 0xFFFFFF) * MUL24[i]) & 0xFFFFFFFF                   # v_mul_u32_u24
    return x ^ (x >> 16)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=22)
    ap.add_argument("--p", type=float, default=0.1)
    a = ap.parse_args()
    N = 1 << a.n
    thr = int(a.p * 65536 + 0.5)
    hb = np.random.default_rng(0).integers(0, 2 ** 32, N, dtype=np.uint64)
    dec = []
    for i in range(8):
        h = pair_draw(hb, i)
        dec += [(h & 0xFFFF) < thr, ((h >> 16) & 0xFFFF) < thr]
    D = np.stack(dec, 1).astype(np.float64)
    C = np.corrcoef(D.T)
    np.fill_diagonal(C, 0)
    cnt = np.bincount(D.sum(1).astype(int), minlength=17)[:8] / N
    exp = np.array([comb(16, k) * a.p ** k * (1 - a.p) ** (16 - k) for k in range(8)])
    print(f"drop rate per key: {D.mean(0).min():.5f} .. {D.mean(0).max():.5f} (p = {a.p})")
    print(f"max |pairwise corr| {np.abs(C).max():.2e} (noise 1/sqrt(N) = {N ** -0.5:.2e})")
    print("joint drop count obs/exp, k = 0..7:", np.round(cnt / exp, 3))


if __name__ == "__main__":
    main()
