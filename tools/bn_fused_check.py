"""BatchNorm small-map fused passes (stats / reduce + finalize in one kernel) against the two-kernel
path: run once per library (MMU_LIB_PATH selects the other build) on the trunk's batch-32 map
shapes, save every output, then compare the two files bitwise.

  python tools/bn_fused_check.py --out a.pt ; MMU_LIB_PATH=ab/base.so python tools/bn_fused_check.py --out b.pt
  python tools/bn_fused_check.py --compare a.pt b.pt
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "multi-modal-uncertainty_amd"))

# (rows, C): batch-32 layer2 / layer3 / layer4 maps (fused) and a layer1 map (two-kernel path)
SHAPES = [(25088, 128), (6272, 256), (6272, 1024), (1568, 512), (1568, 2048), (100352, 64), (17, 64)]


def run(out):
    from src import kernels as K
    dev = torch.device("cuda", 0)
    res = {}
    for rows, C in SHAPES:
        g = torch.Generator(device=dev).manual_seed(rows + C)
        X = (torch.randn(rows, C, generator=g, device=dev) * 2 + 0.5).to(torch.bfloat16)
        S = torch.randn(rows, C, generator=g, device=dev).to(torch.bfloat16)
        w = torch.rand(C, generator=g, device=dev) + 0.5
        b = torch.randn(C, generator=g, device=dev)
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        nbt = torch.zeros((), dtype=torch.int64, device=dev)
        Y = torch.empty_like(X)
        sm, si = torch.empty(C, device=dev), torch.empty(C, device=dev)
        mask = torch.empty(rows * C // 8, dtype=torch.uint8, device=dev)
        K.batchnorm_fwd(X, Y, w, b, rm, rv, True, 0.1, 1e-5, relu=True, skip=S, num_batches_tracked=nbt,
                        save_mean=sm, save_invstd=si, relu_mask=mask)
        dY = torch.randn(rows, C, generator=g, device=dev).to(torch.bfloat16)
        dX, dS = torch.empty_like(X), torch.empty_like(X)
        dw, db = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
        K.batchnorm_bwd(dY, None, X, w, sm, si, True, dX, dS, dw, db, relu_mask=mask)
        torch.cuda.synchronize()
        res[(rows, C)] = {k: v.cpu() for k, v in dict(Y=Y, sm=sm, si=si, rm=rm, rv=rv, nbt=nbt, mask=mask, dX=dX,
                                                        dS=dS, dw=dw, db=db).items()}
    torch.save(res, out)
    print("saved", out)


def compare(a, b):
    A, B = torch.load(a, weights_only=True), torch.load(b, weights_only=True)
    bad = 0
    for key in A:
        for k in A[key]:
            same = torch.equal(A[key][k], B[key][k])
            if not same:
                bad += 1
                d = (A[key][k].float() - B[key][k].float()).abs().max().item()
                print(f"{key} {k}: differs (max abs {d:.3e})")
    print("all outputs bitwise equal" if not bad else f"{bad} outputs differ")
    return bad


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--out")
    ap.add_argument("--compare", nargs=2)
    a = ap.parse_args()
    if a.compare:
        sys.exit(1 if compare(*a.compare) else 0)
    run(a.out)
