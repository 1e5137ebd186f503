"""Short-K filter gradients of the 1x1 convs at batch 32 (K = N*H*W = 1.5-25 K pixels over 4-16
output tiles): mmu_gemm (split-K into f32 slabs + reduce) vs MIOpen, us per call; run under
rocprofv3 --kernel-trace to split the mmu time into the GEMM and the slab reduce.

  python tools/wgrad_small.py [--batch 32]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    n = a.batch
    torch.backends.cudnn.benchmark = True
    dev, cl, bf = "cuda", torch.channels_last, torch.bfloat16
    cbw = torch.ops.aten.convolution_backward
    for cin, cout, h in [(1024, 256, 14), (256, 1024, 14), (512, 128, 28), (128, 512, 28), (2048, 512, 7),
                         (512, 2048, 7), (256, 128, 56)]:
        x = torch.randn(n, cin, h, h, device=dev).to(bf).contiguous(memory_format=cl)
        dy = torch.randn(n, cout, h, h, device=dev).to(bf).contiguous(memory_format=cl)
        w = torch.randn(cout, cin, 1, 1, device=dev).to(bf).contiguous(memory_format=cl)
        g = torch.zeros(cout, cin, device=dev)
        M = n * h * h
        xr, dyr = x.permute(0, 2, 3, 1).reshape(M, cin), dy.permute(0, 2, 3, 1).reshape(M, cout)
        mm = lambda: K.gemm(dyr, cout, 0, xr, cin, 0, g, cin, cout, cin, M,
                            epi=K.epilogue(K.EPI_STORE, accumulate=True))
        mi = lambda: cbw(dy, x, w, None, (1, 1), (0, 0), (1, 1), False, (0, 0), 1, (False, True, False))
        t0, t1 = timed(mi, a.iters), timed(mm, a.iters)
        fl = 2.0 * M * cin * cout
        print(f"  {cin:4d}->{cout:4d} {h:2d}x{h:<2d} K={M:6d}: MIOpen {t0 * 1e3:6.1f} us | mmu {t1 * 1e3:6.1f} us "
              f"({fl / t1 / 1e9:5.0f} TF/s)", flush=True)


if __name__ == "__main__":
    main()
