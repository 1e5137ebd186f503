"""The strided convs of ResNet-152 (first block of layer2..4: conv2 3x3 / stride 2 and the 1x1 /
stride 2 downsample) at a train batch: mmu_conv_implicit / mmu_conv_wgrad vs MIOpen (torch conv
on the same channels-last bf16 tensors), us per call, and the mmu error vs torch fp32.

  python tools/conv_strided_bench.py [--batch 256]
"""
import argparse
import os
import sys

import torch

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "multi-modal-uncertainty_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("MIOPEN_USER_DB_PATH", os.path.join(REPO, "multi-modal-uncertainty_amd", "miopen_db"))
from src import kernels as K  # noqa: E402
from gemm_bench import timed  # noqa: E402

SHAPES = [(128, 128, 3, 56), (256, 256, 3, 28), (512, 512, 3, 14),  # conv2 (Cin, Cout, k, H in)
          (256, 512, 1, 56), (512, 1024, 1, 28), (1024, 2048, 1, 14)]  # downsample


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    n = a.batch
    torch.backends.cudnn.benchmark = True
    cl, dev, bf = torch.channels_last, "cuda", torch.bfloat16
    conv, cbw = torch.ops.aten.convolution, torch.ops.aten.convolution_backward
    tot = {"miopen": 0.0, "mmu": 0.0}
    print(f"batch {n}: strided convs, us per call (MIOpen | mmu), mmu rel err vs fp32")
    for cin, cout, k, h in SHAPES:
        s, pad = 2, k // 2
        x = torch.randn(n, cin, h, h, device=dev).to(bf).contiguous(memory_format=cl)
        wt = (torch.randn(cout, cin, k, k, device=dev) * 0.05).to(bf).contiguous(memory_format=cl)
        y = conv(x, wt, None, (s, s), (pad, pad), (1, 1), False, (0, 0), 1).contiguous(memory_format=cl)
        dy = torch.randn_like(y).contiguous(memory_format=cl)
        yk = torch.empty_like(y)
        dw = torch.zeros(cout, cin, k, k, device=dev).contiguous(memory_format=cl)
        fl = 2.0 * n * y.shape[2] * y.shape[3] * cout * cin * k * k
        row = []
        t0 = timed(lambda: conv(x, wt, None, (s, s), (pad, pad), (1, 1), False, (0, 0), 1), a.iters)
        t1 = timed(lambda: K.conv_implicit(x, wt, yk, k, s), a.iters)
        ref = torch.nn.functional.conv2d(x.float(), wt.float(), stride=s, padding=pad)
        ef = (yk.float() - ref).norm().item() / ref.norm().item()
        row.append(f"fwd {t0 * 1e3:6.1f} | {t1 * 1e3:6.1f} ({fl / t1 / 1e9:4.0f} TF/s, err {ef:.1e})")
        tot["miopen"] += t0
        tot["mmu"] += min(t0, t1)
        if cin % 256 == 0 and cout % 128 == 0:
            t2 = timed(lambda: cbw(dy, x, wt, None, (s, s), (pad, pad), (1, 1), False, (0, 0), 1,
                                   (False, True, False)), a.iters)
            t3 = timed(lambda: K.conv_wgrad(dy, x, dw, k, s, accumulate=False), a.iters)
            rdw = torch.nn.grad.conv2d_weight(x.float(), wt.shape, dy.float(), stride=s, padding=pad)
            ew = (dw - rdw).norm().item() / rdw.norm().item()
            row.append(f"dW {t2 * 1e3:6.1f} | {t3 * 1e3:6.1f} ({fl / t3 / 1e9:4.0f} TF/s, err {ew:.1e})")
            tot["miopen"] += t2
            tot["mmu"] += min(t2, t3)
        print(f"  Cin {cin:4d} Cout {cout:4d} k{k} s2 {h:3d}x{h:<3d}: " + " | ".join(row), flush=True)
    print(f"sum: MIOpen {tot['miopen']:.3f} ms, best-of-both {tot['mmu']:.3f} ms")


if __name__ == "__main__":
    main()
