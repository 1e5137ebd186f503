"""ResNet stem conv (7x7 / 2, 3 -> 64) at the bench batch: mmu_stem_conv_fwd / _wgrad vs MIOpen
(torch conv on the same channels-last bf16 tensors), us per call.

  python tools/stem_bench.py [--batch 256]
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
    ap.add_argument("--batch", type=int, default=256)
    n = ap.parse_args().batch
    torch.backends.cudnn.benchmark = True
    cl, dev = torch.channels_last, "cuda"
    x = torch.randn(n, 3, 224, 224, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
    w = (torch.randn(64, 3, 7, 7, device=dev) * 0.1).to(torch.bfloat16).contiguous(memory_format=cl)
    y = torch.empty(n, 64, 112, 112, dtype=torch.bfloat16, device=dev).contiguous(memory_format=cl)
    dy = torch.randn(n, 64, 112, 112, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
    dw = torch.zeros(64, 3, 7, 7, device=dev).contiguous(memory_format=cl)
    conv = torch.ops.aten.convolution
    cbw = torch.ops.aten.convolution_backward
    fl = 2.0 * n * 112 * 112 * 64 * 147
    rows = [("MIOpen fwd", lambda: conv(x, w, None, (2, 2), (3, 3), (1, 1), False, (0, 0), 1)),
            ("mmu fwd", lambda: K.stem_conv_fwd(x, w, y)),
            ("MIOpen dW", lambda: cbw(dy, x, w, None, (2, 2), (3, 3), (1, 1), False, (0, 0), 1, (False, True, False))),
            ("mmu dW", lambda: K.stem_conv_wgrad(dy, x, dw, accumulate=True))]
    print(f"batch {n}")
    for name, fn in rows:
        t = timed(fn, 10)
        print(f"  {name:11s} {t * 1e3:8.1f} us  ({fl / t / 1e9:6.1f} TF/s)", flush=True)


if __name__ == "__main__":
    main()
