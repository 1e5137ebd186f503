"""Where a big-kernel GEMM launch spends its time, from in-kernel s_memtime stamps (diagnostic
build: make -C multi-modal-uncertainty_amd/csrc EXTRA=-DMMU_GEMM_STAMPS OUT=../../ab/stamps.so
OBJDIR=../../ab/stamps_obj, then MMU_LIB_PATH=ab/stamps.so python tools/gemm_stamps.py).

Per workgroup (wave 0): t0 start, t1 first K-tile in LDS, t2 K loop done, t3 epilogue done
(stores drained).  Reports per-block averages of prologue / K loop / epilogue, the launch
span, and how the blocks fall into rounds (start-time clusters).
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "multi-modal-uncertainty_amd"))
from src import _native, kernels as K  # noqa: E402

HID, FFN = 768, 3072


def main():
    M, dev, bf = 256 * 513, "cuda", torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)

    def rnd(*s):
        return (torch.rand(*s, generator=g, device=dev) * 2 - 1).to(bf)

    X, O, Hh = rnd(M, HID), rnd(M, HID), rnd(M, FFN)
    dY, dZ, R = rnd(M, HID), rnd(M, FFN), rnd(M, HID)
    Wqkv, Wo, W1, W2 = rnd(3 * HID, HID), rnd(HID, HID), rnd(FFN, HID), rnd(HID, FFN)
    bqkv, bo, b1 = (torch.randn(n, device=dev) for n in (3 * HID, HID, FFN))
    out768, out2304, out3072, aux = (torch.empty(M, n, dtype=bf, device=dev) for n in (HID, 3 * HID, FFN, FFN))
    gW = torch.zeros(FFN, HID, device=dev)
    cs = torch.zeros(FFN, device=dev)
    cases = {
        "qkv": (M, 3 * HID, HID, lambda: K.gemm(X, HID, True, Wqkv, HID, True, out2304, 3 * HID, M, 3 * HID, HID,
                                                 epi=K.epilogue(K.EPI_STORE, bias=bqkv))),
        "wo": (M, HID, HID, lambda: K.gemm(O, HID, True, Wo, HID, True, out768, HID, M, HID, HID,
                                            epi=K.epilogue(K.EPI_BIAS_DROP_RES, bias=bo, residual=R, drop_p=0.1,
                                                           seed=3))),
        "w1": (M, FFN, HID, lambda: K.gemm(X, HID, True, W1, HID, True, out3072, FFN, M, FFN, HID,
                                            epi=K.epilogue(K.EPI_BIAS_GELU, bias=b1, aux=aux))),
        "dz": (M, FFN, HID, lambda: K.gemm(dY, HID, True, W2, FFN, False, out3072, FFN, M, FFN, HID,
                                            epi=K.epilogue(K.EPI_DGELU, aux=aux, colsum=cs))),
        "da": (M, HID, FFN, lambda: K.gemm(dZ, FFN, True, W1, HID, False, out768, HID, M, HID, FFN,
                                            epi=K.epilogue(K.EPI_ADD_RES, residual=R))),
        "do": (M, HID, HID, lambda: K.gemm(dY, HID, True, Wo, HID, False, out768, HID, M, HID, HID)),
        "wgrad": (FFN, HID, M, lambda: K.gemm(dZ, FFN, False, X, HID, False, gW, HID, FFN, HID, M,
                                              epi=K.epilogue(K.EPI_STORE, accumulate=True))),
    }
    lib = _native.load()
    fn = lib.mmu_debug_gemm_stamps
    fn.restype, fn.argtypes = ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]
    names = sys.argv[1:] or list(cases)
    for name in names:
        Mm, N, Kd, f = cases[name]
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        f()
        e1.record()
        e1.synchronize()
        ms = e0.elapsed_time(e1)
        nblk = ((Mm + 255) // 256) * ((N + 255) // 256)
        if name == "wgrad":
            nblk *= 8  # split-K slices (upper bound; unused slots stay zero)
        buf = np.zeros((nblk, 4), dtype=np.uint64)
        assert fn(buf.ctypes.data, nblk) == 0
        st = buf[buf[:, 3] > 0].astype(np.int64)
        t0 = st[:, 0] - st[:, 0].min()
        span = st[:, 3].max() - st[:, 0].min()
        ghz = span / (ms * 1e6)
        pro, loop, epi = st[:, 1] - st[:, 0], st[:, 2] - st[:, 1], st[:, 3] - st[:, 2]
        tot = st[:, 3] - st[:, 0]
        busy = tot.sum() / (span * 256)  # fraction of CU-time inside a block (1 block / CU)
        kst = (Kd + 63) // 64 if name != "wgrad" else None
        print(f"{name:6s} {ms:.3f} ms  blocks {len(st)}  span {span / 1e3:.0f} kcyc ({ghz:.2f} GHz equiv)  "
              f"per block: prologue {pro.mean() / 1e3:.1f}k  loop {loop.mean() / 1e3:.1f}k"
              + (f" ({loop.mean() / kst:.0f}/K-step)" if kst else "")
              + f"  epilogue {epi.mean() / 1e3:.1f}k  total {tot.mean() / 1e3:.1f}k  CU occupancy {busy:.2f}  "
              f"start spread p50/p90 {np.percentile(t0, 50) / 1e3:.0f}k/{np.percentile(t0, 90) / 1e3:.0f}k",
              flush=True)
        # rounds: blocks sorted by start; gap between the first 256 and the next
        s0 = np.sort(t0)
        for r in range(0, min(len(s0), 256 * 3), 256):
            seg = tot[np.argsort(t0)][r:r + 256]
            print(f"        round {r // 256}: start {s0[r] / 1e3:.0f}k..{s0[min(r + 255, len(s0) - 1)] / 1e3:.0f}k"
                  f"  block time mean {seg.mean() / 1e3:.1f}k", flush=True)


if __name__ == "__main__":
    main()
