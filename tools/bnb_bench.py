"""The trunk's 1x1 data-gradient products with the BatchNorm backward reduction in the epilogue
(mmu_gemm STORE_BNB / ADD_RES_BNB, src/resnet.py _Conv1x1.backward) at the batch-256 shapes of
every ResNet-152 stage: conv1 of an identity block (K = width, N = 4 width, gated skip residual)
and conv3 (K = 4 width, N = width).  Random operands.

  python tools/bnb_bench.py [--batch 256] [--iters 10]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "multi-modal-uncertainty_amd"))
from src import kernels as K  # noqa: E402


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        best = min(best, a.elapsed_time(b))
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    dev, bf = "cuda", torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)
    print(f"{'product':34s} {'M':>7s} {'K':>5s} {'N':>5s} {'ms':>8s} {'GB/s':>7s}")
    for width, hw in ((64, 56), (128, 28), (256, 14), (512, 7)):
        M = a.batch * hw * hw
        for name, Kd, N, skip in (("conv1 dX + skip + bn reduce", width, 4 * width, True),
                                  ("conv3 dX + bn reduce", 4 * width, width, False)):
            if N % 128:  # (layer1's conv3 data gradient stays on MIOpen)
                continue
            dy = (torch.rand(M, Kd, generator=g, device=dev) - 0.5).to(bf)
            w = (torch.rand(Kd, N, generator=g, device=dev) - 0.5).to(bf)
            x = (torch.rand(a.batch, N, hw, hw, generator=g, device=dev) - 0.5).to(bf).contiguous(
                memory_format=torch.channels_last)
            mask = torch.randint(0, 256, (M * N // 8,), dtype=torch.uint8, device=dev, generator=g)
            mean = torch.rand(N, device=dev, generator=g) - 0.5
            res = (torch.rand(M, N, generator=g, device=dev) - 0.5).to(bf) if skip else None
            rmask = torch.randint(0, 256, (M * N // 8,), dtype=torch.uint8, device=dev, generator=g) if skip else None
            out = torch.empty(M, N, dtype=bf, device=dev)
            table = K.bn_stats_table(M, N, dev)[0]
            epi = K.epilogue(K.EPI_ADD_RES_BNB if skip else K.EPI_STORE_BNB, residual=res, colsum=table,
                             bn=(x, mask, mean), res_mask=rmask)
            t = min(timed(lambda: K.gemm(dy, Kd, 1, w, N, 0, out, N, M, N, Kd, epi=epi), a.iters) for _ in range(2))
            byts = M * Kd * 2 + M * N * (2 + 2 + 0.125 + (2.125 if skip else 0))
            print(f"{name:34s} {M:7d} {Kd:5d} {N:5d} {t:8.3f} {byts / t / 1e6:7.0f}", flush=True)


if __name__ == "__main__":
    main()
