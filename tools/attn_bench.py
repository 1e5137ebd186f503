"""Attention kernel throughput at the bench workload (B=256, L=513, 12 heads x 64):
forward / backward with and without attention-probs dropout; the backward also emits the
Q/K/V bias-gradient column sums as the encoder's does.  MMU_LIB_PATH selects another build.

  python tools/attn_bench.py [--batch 256] [--len 513]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "multi-modal-uncertainty_amd"))
from src import kernels as K  # noqa: E402
from gemm_bench import timed  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--len", type=int, default=513)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    B, L, H, dev = a.batch, a.len, 12, "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    qkv = (torch.randn(B * L, 3 * 768, generator=g, device=dev)).to(torch.bfloat16)
    km = torch.zeros(B, L, device=dev)
    km[: B // 2, L - L // 4:] = -10000.0
    O = torch.empty(B * L, 768, dtype=torch.bfloat16, device=dev)
    lse = torch.empty(B * H, L, device=dev)
    dO = torch.randn(B * L, 768, generator=g, device=dev).to(torch.bfloat16)
    dqkv = torch.empty(B * L, 3 * 768, dtype=torch.bfloat16, device=dev)
    delta = torch.empty(B * H, L, device=dev)
    dm = K.dropmask_empty(B, L, H, dev)
    dbp = K.attention_dbias_parts(B, L, H, dev)
    fl_f = 4.0 * B * H * L * L * 64  # QK^T + PV
    fl_b = 2.5 * fl_f                # S, dP, dV, dK, dQ recompute + products
    for p in (0.0, 0.1):
        tf = timed(lambda: K.attention_fwd(qkv, km, O, lse, B, L, H, p, 7, dm if p > 0 else None), a.iters)
        tb = timed(lambda: K.attention_bwd(qkv, km, O, dO, lse, delta, dqkv, B, L, H, p, 7,
                                           dm if p > 0 else None, dbp), a.iters)
        print(f"p={p:.1f}  fwd {tf:.3f} ms ({fl_f / tf / 1e9:6.1f} TF/s)   bwd {tb:.3f} ms "
              f"({fl_b / tb / 1e9:6.1f} TF/s)", flush=True)


if __name__ == "__main__":
    main()
