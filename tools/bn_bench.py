"""BatchNorm kernels (mmu_batchnorm_fwd/bwd) at ResNet-152 shapes, B=256, against the
bytes they must move (fwd: 3 passes of X [+ skip], bwd: 6 reads + 1-2 writes).

  python tools/bn_bench.py [--batch N]   (MMU_BN_TARGET / MMU_BN_MIN: grid A/B)
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
    N = ap.parse_args().batch
    dev, cl = "cuda", torch.channels_last
    for (C, H, W, skip) in [(64, 112, 112, False), (64, 56, 56, False), (256, 56, 56, True), (128, 28, 28, False),
                            (512, 28, 28, True), (256, 14, 14, False), (1024, 14, 14, True), (512, 7, 7, False),
                            (2048, 7, 7, True)]:
        x = torch.randn(N, C, H, W, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
        s = torch.randn_like(x) if skip else None
        Y, dX = torch.empty_like(x), torch.empty_like(x)
        dS = torch.empty_like(x) if skip else None
        w, b = torch.ones(C, device=dev), torch.zeros(C, device=dev)
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        sm, si = torch.empty(C, device=dev), torch.empty(C, device=dev)
        dw, db = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
        tf = timed(lambda: K.batchnorm_fwd(x, Y, w, b, rm, rv, True, 0.1, 1e-5, relu=True, skip=s,
                                           save_mean=sm, save_invstd=si), 10)
        tb = timed(lambda: K.batchnorm_bwd(x, Y, x, w, sm, si, True, dX, dS, dw, db), 10)
        mk = torch.empty(x.numel() // 8, dtype=torch.uint8, device=dev)
        tfm = timed(lambda: K.batchnorm_fwd(x, Y, w, b, rm, rv, True, 0.1, 1e-5, relu=True, skip=s,
                                            save_mean=sm, save_invstd=si, relu_mask=mk), 10)
        tbm = timed(lambda: K.batchnorm_bwd(x, None, x, w, sm, si, True, dX, dS, dw, db, relu_mask=mk), 10)
        nb = x.numel() * 2
        bf = (3 + (1 if skip else 0)) * nb
        bb = (6 + 1 + (1 if skip else 0)) * nb
        print(f"N{N} C{C:5d} {H:3d}x{W:<3d} skip={int(skip)}  fwd {tf * 1e3:7.1f} us ({bf / tf / 1e9:6.2f} TB/s)"
              f"   bwd {tb * 1e3:7.1f} us ({bb / tb / 1e9:6.2f} TB/s)"
              f"   | relu mask: fwd {tfm * 1e3:7.1f} us  bwd {tbm * 1e3:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
