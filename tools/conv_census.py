"""Which ResNet-152 convolution products still run on MIOpen in the train step, and what each
costs: every StoreConv2d of the trunk is traced once at the given batch (forward hook: input
shape, stride, and whether src/resnet.py routes its forward / dX / dW to mmu kernels), then
each MIOpen product is timed standalone (torch.ops.aten.convolution /
convolution_backward, bf16 channels-last, the shipped find-db) and multiplied by its count.

  python tools/conv_census.py [--batch 256]
"""
import argparse
import os
import sys
from collections import Counter

import torch

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "multi-modal-uncertainty_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("MIOPEN_USER_DB_PATH", os.path.join(REPO, "multi-modal-uncertainty_amd", "miopen_db"))
from src import resnet as R  # noqa: E402
from gemm_bench import timed  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = True
    dev, cl, bf = "cuda", torch.channels_last, torch.bfloat16
    shapes = Counter()

    def add(C, Co, k, s, H):
        M = a.batch * H * H  # the routing rules of src/resnet.py at the train batch
        if k == 1 and s == 1:
            f, d, w = R._mmu_1x1(C, Co, M, H)
        elif k in (1, 3):
            f, d, w = R._mmu_conv((k, s), (a.batch, C, H, H), Co)
        else:
            f = d = w = False
        shapes[(C, Co, k, s, H, H, f, d, w)] += 1

    # ResNet-152 v1.5 (src/resnet.py resnet152_trunk): stem, then Bottlenecks with the stride on
    # the 3x3 conv and a strided 1x1 downsample on the first block of layers 2-4
    add(3, 64, 7, 2, 224)
    cin, H = 64, 56
    for i, (width, n) in enumerate(zip((64, 128, 256, 512), (3, 8, 36, 3))):
        for b in range(n):
            s = 2 if (b == 0 and i > 0) else 1
            add(cin, width, 1, 1, H)
            add(width, width, 3, s, H)
            Ho = H // s
            add(width, 4 * width, 1, 1, Ho)
            if b == 0:
                add(cin, 4 * width, 1, s, H)
            cin, H = 4 * width, Ho
    print(f"batch {a.batch}: MIOpen products per train step (forward, dX, dW), standalone ms")
    tot = {"fwd": 0.0, "dx": 0.0, "dw": 0.0}
    for (C, Co, k, s, H, W, f, d, w), n in sorted(shapes.items()):
        N = a.batch
        x = torch.randn(N, C, H, W, device=dev).to(bf).contiguous(memory_format=cl)
        wt = (torch.randn(Co, C, k, k, device=dev) * 0.05).to(bf).contiguous(memory_format=cl)
        pad = k // 2
        y = torch.ops.aten.convolution(x, wt, None, (s, s), (pad, pad), (1, 1), False, (0, 0), 1)
        dy = torch.randn_like(y).contiguous(memory_format=cl)
        first = k == 7  # the stem: no input gradient
        row = []
        for name, on_mmu, fn in (
                ("fwd", f, lambda: torch.ops.aten.convolution(x, wt, None, (s, s), (pad, pad), (1, 1), False, (0, 0), 1)),
                ("dx", d or first, lambda: torch.ops.aten.convolution_backward(
                    dy, x, wt, None, (s, s), (pad, pad), (1, 1), False, (0, 0), 1, (True, False, False))),
                ("dw", w, lambda: torch.ops.aten.convolution_backward(
                    dy, x, wt, None, (s, s), (pad, pad), (1, 1), False, (0, 0), 1, (False, True, False)))):
            if on_mmu:
                row.append(f"{name} mmu")
                continue
            t = timed(fn, a.iters)
            tot[name] += t * n
            gf = 2.0 * N * y.shape[2] * y.shape[3] * Co * C * k * k / 1e9
            row.append(f"{name} {t * 1e3:7.1f} us ({gf / t:6.0f} TF/s)")
        if k == 3 and s == 1 and C % 64 == 0 and Co % 64 == 0:  # the implicit-GEMM kernels on the same shapes
            from src import kernels as K
            yk = torch.empty_like(y)
            dxk = torch.empty_like(x)
            wf = wt.flip(2, 3).permute(1, 2, 3, 0).contiguous()
            tf = timed(lambda: K.conv3x3_implicit(x, wt, yk), a.iters)
            td = timed(lambda: K.conv3x3_implicit(dy, wf, dxk), a.iters)
            err = (yk.float() - y.float()).abs().max().item() / max(y.float().abs().max().item(), 1e-6)
            row.append(f"mmu fwd {tf * 1e3:7.1f} us dX {td * 1e3:7.1f} us (rel err {err:.1e})")
        print(f"{n:3d} x Cin {C:4d} Cout {Co:4d} k{k} s{s} {H:3d}x{W:<3d}: " + " | ".join(row), flush=True)
    print("MIOpen ms per step: " + ", ".join(f"{k} {v:.2f}" for k, v in tot.items()) + f", total {sum(tot.values()):.2f}")


if __name__ == "__main__":
    main()
