"""Run ONE hot kernel of the bench workload a few times, for rocprofv3 PMC passes
(counters per dispatch; no timing of its own).

  python tools/kprof.py attn_fwd|attn_bwd|gemm_w1|gemm_qkv|gemm_dz|gemm_wgrad|ln_fwd|ln_bwd|bn_fwd|bn_bwd|stem_fwd|stem_wgrad
                        [--reps 3]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "multi-modal-uncertainty_amd"))
from src import kernels as K  # noqa: E402

HID, FFN = 768, 3072


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("which")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    B, L, H, dev, bf = a.batch, 513, 12, "cuda", torch.bfloat16
    M = B * L
    g = torch.Generator(device=dev).manual_seed(0)

    def rnd(*s):
        return (torch.rand(*s, generator=g, device=dev) * 2 - 1).to(bf)

    if a.which.startswith("attn"):
        qkv = torch.randn(M, 3 * HID, generator=g, device=dev).to(bf)
        km = torch.zeros(B, L, device=dev)
        O = torch.empty(M, HID, dtype=bf, device=dev)
        lse = torch.empty(B * H, L, device=dev)
        dO = torch.randn(M, HID, generator=g, device=dev).to(bf)
        dqkv = torch.empty(M, 3 * HID, dtype=bf, device=dev)
        delta = torch.empty(B * H, L, device=dev)
        dm = K.dropmask_empty(B, L, H, dev)
        K.attention_fwd(qkv, km, O, lse, B, L, H, 0.1, 7, dm)
        if a.which == "attn_fwd":
            fn = lambda: K.attention_fwd(qkv, km, O, lse, B, L, H, 0.1, 7, dm)  # noqa: E731
        else:
            fn = lambda: K.attention_bwd(qkv, km, O, dO, lse, delta, dqkv, B, L, H, 0.1, 7, dm)  # noqa: E731
    elif a.which.startswith("ln_"):  # the encoder's output LayerNorm, forward / backward (f32 input)
        S = torch.randn(M, HID, generator=g, device=dev)
        w, b = torch.randn(HID, device=dev), torch.randn(HID, device=dev)
        Y = torch.empty(M, HID, dtype=bf, device=dev)
        mean, rstd = torch.empty(M, device=dev), torch.empty(M, device=dev)
        K.layernorm_fwd_f32(S, w, b, Y, None, mean, rstd)
        dY = rnd(M, HID)
        dX, dXd = torch.empty(M, HID, dtype=bf, device=dev), torch.empty(M, HID, dtype=bf, device=dev)
        P = K.ln_parts(M)
        pw, pb, pbias = (torch.empty(P, HID, device=dev) for _ in range(3))
        fn = (lambda: K.layernorm_fwd_f32(S, w, b, Y, None, mean, rstd)) if a.which == "ln_fwd" else \
            (lambda: K.layernorm_bwd(dY, S, mean, rstd, w, dX, dXd, 0.1, 5, pw, pb, pbias))  # noqa: E731
    elif a.which.startswith("stem_"):  # the ResNet stem conv (7x7 / 2, 3 -> 64) on 224 x 224 images
        cl = torch.channels_last
        x = torch.randn(B, 3, 224, 224, generator=g, device=dev).to(bf).contiguous(memory_format=cl)
        wt = (torch.randn(64, 3, 7, 7, generator=g, device=dev) * 0.1).to(bf).contiguous(memory_format=cl)
        y = torch.empty(B, 64, 112, 112, dtype=bf, device=dev).contiguous(memory_format=cl)
        dy = torch.randn(B, 64, 112, 112, generator=g, device=dev).to(bf).contiguous(memory_format=cl)
        dw = torch.zeros(64, 3, 7, 7, device=dev).contiguous(memory_format=cl)
        fn = (lambda: K.stem_conv_fwd(x, wt, y)) if a.which == "stem_fwd" else \
            (lambda: K.stem_conv_wgrad(dy, x, dw, accumulate=True))  # noqa: E731
    elif a.which.startswith("bn_"):  # layer3 bn3 (+ skip, ReLU): [B*14*14, 1024] channels-last
        Nb, C, H = B, 1024, 14
        cl = torch.channels_last
        x = torch.randn(Nb, C, H, H, generator=g, device=dev).to(bf).contiguous(memory_format=cl)
        skip = torch.randn(Nb, C, H, H, generator=g, device=dev).to(bf).contiguous(memory_format=cl)
        y = torch.empty_like(x)
        w, b = torch.ones(C, device=dev), torch.zeros(C, device=dev)
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        nbt = torch.zeros((), dtype=torch.int64, device=dev)
        sm, si = torch.empty(C, device=dev), torch.empty(C, device=dev)
        mask = torch.empty(x.numel() // 8, dtype=torch.uint8, device=dev)
        K.batchnorm_fwd(x, y, w, b, rm, rv, True, 0.1, 1e-5, relu=True, skip=skip, num_batches_tracked=nbt,
                        save_mean=sm, save_invstd=si, relu_mask=mask)
        dy = torch.randn(Nb, C, H, H, generator=g, device=dev).to(bf).contiguous(memory_format=cl)
        dx, ds = torch.empty_like(x), torch.empty_like(x)
        dw, db = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
        fn = (lambda: K.batchnorm_fwd(x, y, w, b, rm, rv, True, 0.1, 1e-5, relu=True, skip=skip,  # noqa: E731
                                      num_batches_tracked=nbt, save_mean=sm, save_invstd=si, relu_mask=mask)) \
            if a.which == "bn_fwd" else \
            (lambda: K.batchnorm_bwd(dy, None, x, w, sm, si, True, dx, ds, dw, db, relu_mask=mask))  # noqa: E731
    else:
        X, A = rnd(M, HID), rnd(M, HID)
        W1, W2, Wqkv = rnd(FFN, HID), rnd(HID, FFN), rnd(3 * HID, HID)
        b1, bqkv = torch.randn(FFN, device=dev), torch.randn(3 * HID, device=dev)
        out = torch.empty(M, FFN, dtype=bf, device=dev)
        Zs = rnd(M, FFN)
        cs = torch.zeros(FFN, device=dev)
        dY, dZ = rnd(M, HID), rnd(M, FFN)
        gW = torch.zeros(FFN, HID, device=dev)
        fns = {
            "gemm_w1": lambda: K.gemm(A, HID, True, W1, HID, True, out, FFN, M, FFN, HID,
                                      epi=K.epilogue(K.EPI_BIAS_GELU, bias=b1, aux=Zs)),
            "gemm_qkv": lambda: K.gemm(X, HID, True, Wqkv, HID, True, out, 3 * HID, M, 3 * HID, HID,
                                       epi=K.epilogue(K.EPI_STORE, bias=bqkv)),
            "gemm_dz": lambda: K.gemm(dY, HID, True, W2, FFN, False, out, FFN, M, FFN, HID,
                                      epi=K.epilogue(K.EPI_DGELU, aux=Zs, colsum=cs)),
            "gemm_wgrad": lambda: K.gemm(dZ, FFN, False, A, HID, False, gW, HID, FFN, HID, M,
                                         epi=K.epilogue(K.EPI_STORE, accumulate=True)),
        }
        fn = fns[a.which]
    for _ in range(a.reps):
        fn()
    torch.cuda.synchronize()
    print("ok", a.which, flush=True)


if __name__ == "__main__":
    main()
