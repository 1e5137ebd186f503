"""LayerNorm forward / backward kernels at the bench workload (M = 256 x 513 rows, H = 768)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "multi-modal-uncertainty_amd"))
from src import kernels as K  # noqa: E402
from gemm_bench import timed  # noqa: E402


def main():
    M, H, dev = 256 * 513, 768, "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.randn(M, H, generator=g, device=dev).to(torch.bfloat16)
    dY = torch.randn(M, H, generator=g, device=dev).to(torch.bfloat16)
    w, b = torch.rand(H, device=dev) + 0.5, torch.randn(H, device=dev)
    Y = torch.empty_like(X)
    mean, rstd = torch.empty(M, device=dev), torch.empty(M, device=dev)
    dX, dXd = torch.empty_like(X), torch.empty_like(X)
    P = K.ln_parts(M)
    pw, pb, pbias = (torch.empty(P, H, device=dev) for _ in range(3))
    os.environ["MMU_LN_V2"] = "0"
    tf0 = timed(lambda: K.layernorm_fwd(X, w, b, Y, mean, rstd), 10)
    Y0 = Y.clone()
    os.environ["MMU_LN_V2"] = "1"
    tf = timed(lambda: K.layernorm_fwd(X, w, b, Y, mean, rstd), 10)
    print(f"LN fwd row-per-wave 8-B {tf0 * 1e3:7.1f} us ({2 * M * H * 2 / tf0 / 1e9:5.2f} TB/s)  identical: "
          f"{bool(torch.equal(Y0, Y))}", flush=True)
    tb = timed(lambda: K.layernorm_bwd(dY, X, mean, rstd, w, dX, dXd, 0.1, 3, pw, pb, pbias), 10)
    nb = M * H * 2
    print(f"LN fwd {tf * 1e3:7.1f} us ({2 * nb / tf / 1e9:5.2f} TB/s)   bwd {tb * 1e3:7.1f} us "
          f"({4 * nb / tb / 1e9:5.2f} TB/s)", flush=True)


if __name__ == "__main__":
    main()
