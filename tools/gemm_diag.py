"""Where a big-tile GEMM result is wrong: per tile-local 16x16 block (rows x cols mod 256) error
counts of mmu_gemm (both operands K-major) against torch, for a given shape; it located the
last-K-tile wait of round 5's ping-pong variant (profiles/r5_gemm_pingpong_ab.txt).
  python tools/gemm_diag.py M N K [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "multi-modal-uncertainty_amd"))
from src import kernels as K  # noqa: E402

M, N, Kd = (int(v) for v in sys.argv[1:4])
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 3
g = torch.Generator(device="cuda").manual_seed(0)
A = (torch.rand(M, Kd, generator=g, device="cuda") * 2 - 1).bfloat16()
B = (torch.rand(N, Kd, generator=g, device="cuda") * 2 - 1).bfloat16()
ref = A.float() @ B.float().t()
for r in range(reps):
    out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    K.gemm(A, Kd, True, B, Kd, True, out, N, M, N, Kd)
    torch.cuda.synchronize()
    bad = (out.float() - ref).abs() > 0.02 * ref.abs().max()
    n = int(bad.sum())
    print(f"rep {r}: {n} bad of {M * N}")
    if n:
        idx = bad.nonzero()
        rows, cols = idx[:, 0], idx[:, 1]
        tiles = torch.unique(rows // 256 * 1000 + cols // 256)
        print("  tiles (tm*1000+tn) with errors:", tiles[:20].tolist(), "count", tiles.numel())
        blk = torch.zeros(16, 16, dtype=torch.int64, device="cuda")
        blk.index_put_(((rows % 256) // 16, (cols % 256) // 16), torch.ones_like(rows), accumulate=True)
        print("  tile-local 16x16 blocks (row-block x col-block) with errors:")
        for i in range(16):
            print("   ", " ".join(f"{int(v):4d}" for v in blk[i].tolist()))
