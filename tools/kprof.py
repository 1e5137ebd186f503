"""Run ONE hot kernel of the bench workload a few times, for rocprofv3 PMC passes
(counters per dispatch; no timing of its own).

  python tools/kprof.py attn_fwd|attn_bwd|gemm_w1|gemm_qkv|gemm_dz|gemm_wgrad [--reps 3]
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
