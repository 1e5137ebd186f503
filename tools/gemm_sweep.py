"""K-sweep of one mmu_gemm shape: separates the per-tile fixed cost (prologue + epilogue,
the intercept) from the main-loop rate (the slope).  Random bf16 operands.

  python tools/gemm_sweep.py [--m 131328] [--n 768] [--epi store|drop_res|gelu]
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
    ap.add_argument("--m", type=int, default=256 * 513)
    ap.add_argument("--n", type=int, default=768)
    ap.add_argument("--epi", default="store")
    ap.add_argument("--ks", default="64,128,256,512,768,1536,3072")
    ap.add_argument("--bk", type=int, default=1, help="B K-major (1) or N-major (0)")
    a = ap.parse_args()
    dev, bf = "cuda", torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)
    M, N = a.m, a.n
    out = torch.empty(M, N, dtype=bf, device=dev)
    R = (torch.rand(M, N, generator=g, device=dev) - 0.5).to(bf)
    aux = torch.empty(M, N, dtype=bf, device=dev)
    bias = torch.randn(N, device=dev)
    for k in [int(x) for x in a.ks.split(",")]:
        A = (torch.rand(M, k, generator=g, device=dev) * 2 - 1).to(bf)
        B = (torch.rand(N, k, generator=g, device=dev) * 2 - 1).to(bf)
        if not a.bk:
            B = B.t().contiguous()
        if a.epi == "drop_res":
            e = K.epilogue(K.EPI_BIAS_DROP_RES, bias=bias, residual=R, drop_p=0.1, seed=3)
        elif a.epi == "gelu":
            e = K.epilogue(K.EPI_BIAS_GELU, bias=bias, aux=aux)
        else:
            e = None
        fn = lambda: K.gemm(A, k, True, B, k if a.bk else N, bool(a.bk), out, N, M, N, k, epi=e)  # noqa: E731
        t = timed(fn, 10)
        fl = 2.0 * M * N * k
        print(f"K={k:5d}  {t:.4f} ms ({fl / t / 1e9:7.1f} TF/s)", flush=True)


if __name__ == "__main__":
    main()
