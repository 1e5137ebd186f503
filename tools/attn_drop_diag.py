import os, sys, torch
sys.path[:0] = ["multi-modal-uncertainty_amd", "tests"]
from src import kernels as k
from test_kernels_gpu import make_attn_inputs, attn_ref, rnd
dev = "cuda"
for (B, L, p) in ((2, 60, 0.2), (2, 130, 0.1), (2, 60, 0.0)):
    qkv, km = make_attn_inputs(dev, B, L, pad=False, seed=5, scale=1.0)
    O = torch.empty(B * L, 768, dtype=torch.bfloat16, device=dev)
    lse = torch.empty(B * 12, L, device=dev)
    dm = k.dropmask_empty(B, L, 12, dev)
    k.attention_fwd(qkv, km, O, lse, B, L, drop_p=p, seed=99, dropmask=dm if p > 0 else None)
    mask = k.dropmask_dense(dm, L).view(B, 12, L, L) if p > 0 else None
    dO = rnd(B * L, 768, dev=dev, seed=7)
    dqkv = torch.zeros(B * L, 2304, dtype=torch.bfloat16, device=dev)
    delta = torch.empty(B * 12, L, device=dev)
    k.attention_bwd(qkv, km, O, dO, lse, delta, dqkv, B, L, drop_p=p, seed=99, dropmask=dm if p > 0 else None)
    x = qkv.float().requires_grad_(True)
    o2, _ = attn_ref(x, km, B, L, dropmask=mask, p=p)
    (g,) = torch.autograd.grad(o2, x, dO.float())
    for part, nm in enumerate("QKV"):
        a = dqkv[:, 768 * part:768 * (part + 1)].float(); r = g[:, 768 * part:768 * (part + 1)]
        ratio = (a * r).sum() / (r * r).sum()
        print(f"L={L} p={p} d{nm}: rel err {((a - r).norm() / r.norm()).item():.3e} best-fit scale {ratio.item():.4f}")
