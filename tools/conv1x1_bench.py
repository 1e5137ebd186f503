"""1x1 stride-1 convolutions of the ResNet-152 trunk: MIOpen (what torch's conv runs) vs the
same products as mmu_gemm calls on the channels-last image ([N*H*W, C] row-major).

  fwd:  Y[m, o]  = sum_i X[m, i] W[o, i]      (A = X K-major, B = W K-major)
  dX:   dX[m, i] = sum_o dY[m, o] W[o, i]     (A = dY K-major, B = W N-major)
  dW:   dW[o, i] = sum_m dY[m, o] X[m, i]     (A = dY M-major, B = X N-major; f32, split-K)

  python tools/conv1x1_bench.py [--batch N]
"""
import argparse
import os
import sys

import torch

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "multi-modal-uncertainty_amd"))
os.environ.setdefault("MIOPEN_USER_DB_PATH", os.path.join(REPO, "multi-modal-uncertainty_amd", "miopen_db"))
from src import kernels as K  # noqa: E402
from gemm_bench import timed  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    N = ap.parse_args().batch
    torch.backends.cudnn.benchmark = True
    dev, cl = "cuda", torch.channels_last
    # (Cin, Cout, H): layer2..4 conv1 / conv3 (every stride-1 1x1 with both widths % 128 == 0)
    shapes = [(256, 64, 56), (64, 256, 56), (512, 128, 28), (128, 512, 28), (1024, 256, 14), (256, 1024, 14),
              (2048, 512, 7), (512, 2048, 7), (64, 64, 56), (256, 128, 56), (512, 256, 28), (1024, 512, 14)]
    print(f"batch {N}; us per call (best of 10); TF/s in brackets")
    for cin, cout, H in shapes:
        x = (torch.randn(N, cin, H, H, device=dev) * 0.5).to(torch.bfloat16).contiguous(memory_format=cl)
        w = (torch.randn(cout, cin, 1, 1, device=dev) * cin ** -0.5).to(torch.bfloat16).contiguous(memory_format=cl)
        dy = (torch.randn(N, cout, H, H, device=dev) * 0.5).to(torch.bfloat16).contiguous(memory_format=cl)
        M = N * H * H
        fl = 2.0 * M * cin * cout
        conv = torch.ops.aten.convolution
        cbw = torch.ops.aten.convolution_backward
        t_mf = timed(lambda: conv(x, w, None, (1, 1), (0, 0), (1, 1), False, (0, 0), 1), 10)
        t_md = timed(lambda: cbw(dy, x, w, None, (1, 1), (0, 0), (1, 1), False, (0, 0), 1, (True, False, False)), 10)
        t_mw = timed(lambda: cbw(dy, x, w, None, (1, 1), (0, 0), (1, 1), False, (0, 0), 1, (False, True, False)), 10)
        X2, W2, dY2 = x.permute(0, 2, 3, 1).reshape(M, cin), w.reshape(cout, cin), dy.permute(0, 2, 3, 1).reshape(M, cout)
        Y = torch.empty(M, cout, dtype=torch.bfloat16, device=dev)
        dX = torch.empty(M, cin, dtype=torch.bfloat16, device=dev)
        dW = torch.zeros(cout, cin, dtype=torch.float32, device=dev)
        acc = K.epilogue(K.EPI_STORE, accumulate=True)
        skip = (torch.randn(M, cin, device=dev) * 0.5).to(torch.bfloat16)
        ok_f, ok_d, ok_w = cout % 128 == 0, cin % 128 == 0, cout % 128 == 0 and cin % 128 == 0
        nan = float("nan")
        t_gf = timed(lambda: K.gemm(X2, cin, 1, W2, cin, 1, Y, cout, M, cout, cin), 10) if ok_f else nan
        t_gd = timed(lambda: K.gemm(dY2, cout, 1, W2, cin, 0, dX, cin, M, cin, cout), 10) if ok_d else nan
        t_gw = timed(lambda: K.gemm(dY2, cout, 0, X2, cin, 0, dW, cin, cout, cin, M, epi=acc), 10) if ok_w else nan
        # the Bottleneck's identity-skip join: MIOpen dX + autograd's add vs one GEMM with ADD_RES
        res = K.epilogue(K.EPI_ADD_RES, residual=skip)
        t_ma = timed(lambda: cbw(dy, x, w, None, (1, 1), (0, 0), (1, 1), False, (0, 0), 1,
                                 (True, False, False))[0].permute(0, 2, 3, 1).reshape(M, cin) + skip, 10)
        t_ga = timed(lambda: K.gemm(dY2, cout, 1, W2, cin, 0, dX, cin, M, cin, cout, epi=res), 10) if ok_d else nan
        # parity of the three products against MIOpen (bf16 outputs; dW in f32)
        ref_y = conv(x, w, None, (1, 1), (0, 0), (1, 1), False, (0, 0), 1).permute(0, 2, 3, 1).reshape(M, cout)
        rdx, rdw, _ = cbw(dy, x, w, None, (1, 1), (0, 0), (1, 1), False, (0, 0), 1, (True, True, False))
        dW.zero_()
        e = [nan, nan, nan]
        rel = lambda a, b: float((a.float() - b.float()).abs().max() / b.float().abs().max())  # noqa: E731
        if ok_w:
            K.gemm(dY2, cout, 0, X2, cin, 0, dW, cin, cout, cin, M, epi=acc)
            e[2] = rel(dW, rdw.reshape(cout, cin))
        if ok_f:
            K.gemm(X2, cin, 1, W2, cin, 1, Y, cout, M, cout, cin)
            e[0] = rel(Y, ref_y)
        if ok_d:
            K.gemm(dY2, cout, 1, W2, cin, 0, dX, cin, M, cin, cout, epi=res)
            e[1] = rel(dX, rdx.permute(0, 2, 3, 1).reshape(M, cin) + skip)
        f = lambda t: f"{t * 1e3:7.1f} ({fl / t / 1e9:5.0f})"  # noqa: E731
        print(f"{cin:4d}->{cout:4d} {H:2d}x{H:<2d} M={M:7d} | MIOpen fwd {f(t_mf)} dX {f(t_md)} dW {f(t_mw)} "
              f"dX+add {t_ma * 1e3:7.1f} | mmu fwd {f(t_gf)} dX {f(t_gd)} dW {f(t_gw)} dX+add {t_ga * 1e3:7.1f} | "
              f"rel err {e[0]:.1e} {e[1]:.1e} {e[2]:.1e}", flush=True)


if __name__ == "__main__":
    main()
