"""Per-shape throughput of the BERT-layer GEMMs (mmu_gemm) at the bench workload
(M = 256 x 513 token rows), with hipBLASLt (torch.matmul) on the same shapes as a
yardstick.  Random operands (zero-filled data inflates MFMA clocks).

  python tools/gemm_bench.py [--rows 131328] [--iters 10]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "multi-modal-uncertainty_amd"))
from src import kernels as K  # noqa: E402

HID, FFN = 768, 3072


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
    ap.add_argument("--rows", type=int, default=256 * 513)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--cases", default="", help="comma-separated substrings: run only the matching cases")
    ap.add_argument("--no-ref", action="store_true", help="skip the hipBLASLt yardstick")
    a = ap.parse_args()
    M, dev, bf = a.rows, "cuda", torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)

    def rnd(*s):
        return (torch.rand(*s, generator=g, device=dev) * 2 - 1).to(bf)

    X, A, O = rnd(M, HID), rnd(M, HID), rnd(M, HID)
    Hh = rnd(M, FFN)
    dY, dqkv, dZ = rnd(M, HID), rnd(M, 3 * HID), rnd(M, FFN)
    Wqkv, Wo, W1, W2 = rnd(3 * HID, HID), rnd(HID, HID), rnd(FFN, HID), rnd(HID, FFN)
    Wqkvt, Wot, W1t, W2t = (w.t().contiguous() for w in (Wqkv, Wo, W1, W2))
    bqkv, bo, b1 = (torch.randn(n, device=dev) for n in (3 * HID, HID, FFN))
    out768, out2304, out3072 = (torch.empty(M, n, dtype=bf, device=dev) for n in (HID, 3 * HID, FFN))
    Zs = rnd(M, FFN)
    gW = torch.zeros(FFN, HID, device=dev)
    gW2, gWq, gWo = torch.zeros(HID, FFN, device=dev), torch.zeros(3 * HID, HID, device=dev), torch.zeros(HID, HID, device=dev)
    cs = torch.zeros(FFN, device=dev)
    cases = [
        ("fwd qkv  X.Wqkv^T+b", M, 3 * HID, HID,
         lambda: K.gemm(X, HID, True, Wqkv, HID, True, out2304, 3 * HID, M, 3 * HID, HID,
                        epi=K.epilogue(K.EPI_STORE, bias=bqkv)),
         lambda: torch.matmul(X, Wqkv.t())),
        ("fwd o    drop_res", M, HID, HID,
         lambda: K.gemm(O, HID, True, Wo, HID, True, out768, HID, M, HID, HID,
                        epi=K.epilogue(K.EPI_BIAS_DROP_RES, bias=bo, residual=X, drop_p=0.1, seed=1)),
         lambda: torch.matmul(O, Wo.t())),
        ("fwd ffn1 gelu", M, FFN, HID,
         lambda: K.gemm(A, HID, True, W1, HID, True, out3072, FFN, M, FFN, HID,
                        epi=K.epilogue(K.EPI_BIAS_GELU, bias=b1, aux=Zs)),
         lambda: torch.matmul(A, W1.t())),
        ("fwd ffn1 gelu, no aux", M, FFN, HID,
         lambda: K.gemm(A, HID, True, W1, HID, True, out3072, FFN, M, FFN, HID,
                        epi=K.epilogue(K.EPI_BIAS_GELU, bias=b1)),
         lambda: torch.matmul(A, W1.t())),
        ("fwd ffn1 bias only", M, FFN, HID,
         lambda: K.gemm(A, HID, True, W1, HID, True, out3072, FFN, M, FFN, HID,
                        epi=K.epilogue(K.EPI_STORE, bias=b1)),
         lambda: torch.matmul(A, W1.t())),
        ("fwd o    bias only", M, HID, HID,
         lambda: K.gemm(O, HID, True, Wo, HID, True, out768, HID, M, HID, HID,
                        epi=K.epilogue(K.EPI_STORE, bias=bo)),
         lambda: torch.matmul(O, Wo.t())),
        ("fwd o    res, no dropout", M, HID, HID,
         lambda: K.gemm(O, HID, True, Wo, HID, True, out768, HID, M, HID, HID,
                        epi=K.epilogue(K.EPI_BIAS_DROP_RES, bias=bo, residual=X, drop_p=0.0, seed=1)),
         lambda: torch.matmul(O, Wo.t())),
        ("fwd ffn2 drop_res", M, HID, FFN,
         lambda: K.gemm(Hh, FFN, True, W2, FFN, True, out768, HID, M, HID, FFN,
                        epi=K.epilogue(K.EPI_BIAS_DROP_RES, bias=bo, residual=A, drop_p=0.1, seed=2)),
         lambda: torch.matmul(Hh, W2.t())),
        ("bwd dZ   dgelu+colsum", M, FFN, HID,
         lambda: K.gemm(dY, HID, True, W2, FFN, False, out3072, FFN, M, FFN, HID,
                        epi=K.epilogue(K.EPI_DGELU, aux=Zs, colsum=cs)),
         lambda: torch.matmul(dY, W2)),
        ("bwd dA   add_res", M, HID, FFN,
         lambda: K.gemm(dZ, FFN, True, W1, HID, False, out768, HID, M, HID, FFN,
                        epi=K.epilogue(K.EPI_ADD_RES, residual=dY)),
         lambda: torch.matmul(dZ, W1)),
        ("bwd dX   qkv add_res", M, HID, 3 * HID,
         lambda: K.gemm(dqkv, 3 * HID, True, Wqkv, HID, False, out768, HID, M, HID, 3 * HID,
                        epi=K.epilogue(K.EPI_ADD_RES, residual=dY)),
         lambda: torch.matmul(dqkv, Wqkv)),
        ("bwd dO   store", M, HID, HID,
         lambda: K.gemm(dY, HID, True, Wo, HID, False, out768, HID, M, HID, HID),
         lambda: torch.matmul(dY, Wo)),
        # the same data-grad products with a K-major (transposed) copy of the weight as B
        ("bwd dZ   B=W2^T kmaj", M, FFN, HID,
         lambda: K.gemm(dY, HID, True, W2t, HID, True, out3072, FFN, M, FFN, HID,
                        epi=K.epilogue(K.EPI_DGELU, aux=Zs, colsum=cs)),
         lambda: torch.matmul(dY, W2)),
        ("bwd dZ   B=W2^T kmaj, no colsum", M, FFN, HID,
         lambda: K.gemm(dY, HID, True, W2t, HID, True, out3072, FFN, M, FFN, HID,
                        epi=K.epilogue(K.EPI_DGELU, aux=Zs)),
         lambda: torch.matmul(dY, W2)),
        ("bwd dA   B=W1^T kmaj", M, HID, FFN,
         lambda: K.gemm(dZ, FFN, True, W1t, FFN, True, out768, HID, M, HID, FFN,
                        epi=K.epilogue(K.EPI_ADD_RES, residual=dY)),
         lambda: torch.matmul(dZ, W1)),
        ("bwd dX   B=Wqkv^T kmaj", M, HID, 3 * HID,
         lambda: K.gemm(dqkv, 3 * HID, True, Wqkvt, 3 * HID, True, out768, HID, M, HID, 3 * HID,
                        epi=K.epilogue(K.EPI_ADD_RES, residual=dY)),
         lambda: torch.matmul(dqkv, Wqkv)),
        ("bwd dO   B=Wo^T kmaj", M, HID, HID,
         lambda: K.gemm(dY, HID, True, Wot, HID, True, out768, HID, M, HID, HID),
         lambda: torch.matmul(dY, Wo)),
        ("wgrad W1 dZ^T.A f32acc", FFN, HID, M,
         lambda: K.gemm(dZ, FFN, False, A, HID, False, gW, HID, FFN, HID, M,
                        epi=K.epilogue(K.EPI_STORE, accumulate=True)),
         lambda: torch.matmul(dZ.t(), A)),
        ("wgrad W2 dY^T.H f32acc", HID, FFN, M,
         lambda: K.gemm(dY, HID, False, Hh, FFN, False, gW2, FFN, HID, FFN, M,
                        epi=K.epilogue(K.EPI_STORE, accumulate=True)),
         lambda: torch.matmul(dY.t(), Hh)),
        ("wgrad Wqkv dQKV^T.X f32acc", 3 * HID, HID, M,
         lambda: K.gemm(dqkv, 3 * HID, False, X, HID, False, gWq, HID, 3 * HID, HID, M,
                        epi=K.epilogue(K.EPI_STORE, accumulate=True)),
         lambda: torch.matmul(dqkv.t(), X)),
        ("wgrad Wo dS1^T.O f32acc", HID, HID, M,
         lambda: K.gemm(dY, HID, False, O, HID, False, gWo, HID, HID, HID, M,
                        epi=K.epilogue(K.EPI_STORE, accumulate=True)),
         lambda: torch.matmul(dY.t(), O)),
    ]
    print(f"{'gemm':26s} {'M':>7s} {'N':>5s} {'K':>7s} {'mmu_gemm':>18s} {'hipBLASLt':>18s}")
    want = [c for c in a.cases.split(",") if c]
    for name, m, n, k, f_mmu, f_ref in cases:
        if want and not any(w in name for w in want):
            continue
        fl = 2.0 * m * n * k
        t1 = min(timed(f_mmu, a.iters) for _ in range(3))
        t2 = float("nan") if a.no_ref else timed(f_ref, a.iters)
        print(f"{name:26s} {m:7d} {n:5d} {k:7d} {t1:8.3f}ms {fl / t1 / 1e9:6.0f}T {t2:8.3f}ms {fl / t2 / 1e9:6.0f}T",
              flush=True)


if __name__ == "__main__":
    main()
