"""Time the ResNet-152 trunk's BatchNorm launches (forward + backward) at one batch size, shape
by shape, with the library that is loaded (MMU_LIB_PATH selects another build of the same
ABI for a same-box A/B).  Per shape: the BatchNorm2d flavour src/resnet.py runs there (bn1 /
bn2: ReLU + mask; bn3: residual + ReLU + mask, dSkip in the backward; downsample: plain) and
how many times a train step runs it.

  python tools/bn_bench.py [--batch 32] [--iters 20]
"""
import argparse
import os
import sys
from collections import Counter

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "multi-modal-uncertainty_amd"))
from src import kernels as K  # noqa: E402


def trunk_bns():
    """(C, H, kind) -> count per train step; kind in relu / skip / plain"""
    c = Counter()
    c[(64, 112, "relu")] += 1
    cin, H = 64, 56
    for i, (width, n) in enumerate(zip((64, 128, 256, 512), (3, 8, 36, 3))):
        for b in range(n):
            s = 2 if (b == 0 and i > 0) else 1
            c[(width, H, "relu")] += 1
            Ho = H // s
            c[(width, Ho, "relu")] += 1
            c[(4 * width, Ho, "skip")] += 1
            if b == 0:
                c[(4 * width, Ho, "plain")] += 1
            cin, H = 4 * width, Ho
    return c


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev, cl, bf = "cuda", torch.channels_last, torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)
    tot_f = tot_b = 0.0
    print(f"batch {a.batch}, library {os.environ.get('MMU_LIB_PATH', 'in-tree')}")
    for (C, H, kind), n in sorted(trunk_bns().items()):
        x = torch.randn(a.batch, C, H, H, generator=g, device=dev).to(bf).contiguous(memory_format=cl)
        sk = torch.randn_like(x).contiguous(memory_format=cl) if kind == "skip" else None
        y = torch.empty_like(x)
        w, b = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        nbt = torch.zeros((), dtype=torch.int64, device=dev)
        sm, si = torch.empty(C, device=dev), torch.empty(C, device=dev)
        relu = kind != "plain"
        mask = torch.empty(x.numel() // 8, dtype=torch.uint8, device=dev) if relu else None
        dy = torch.randn_like(x).contiguous(memory_format=cl)
        dx = torch.empty_like(x)
        ds = torch.empty_like(x) if kind == "skip" else None
        dw, db = torch.zeros(C, device=dev), torch.zeros(C, device=dev)

        def fwd():
            K.batchnorm_fwd(x, y, w, b, rm, rv, True, 0.1, 1e-5, relu=relu, skip=sk, num_batches_tracked=nbt,
                            save_mean=sm, save_invstd=si, relu_mask=mask)

        def bwd():
            K.batchnorm_bwd(dy, None, x, w, sm, si, relu, dx, ds, dw, db, relu_mask=mask)

        res = []
        for fn in (fwd, bwd):
            for _ in range(3):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            res.append(e0.elapsed_time(e1) * 1e3 / a.iters)
        tot_f += res[0] * n
        tot_b += res[1] * n
        mb = x.numel() * 2 / 1e6
        print(f"{n:3d} x C {C:4d} {H:3d}x{H:<3d} {kind:5s} {mb:8.1f} MB: fwd {res[0]:7.1f} us  bwd {res[1]:7.1f} us",
              flush=True)
    print(f"per step: fwd {tot_f / 1e3:.2f} ms, bwd {tot_b / 1e3:.2f} ms, total {(tot_f + tot_b) / 1e3:.2f} ms")


if __name__ == "__main__":
    main()
