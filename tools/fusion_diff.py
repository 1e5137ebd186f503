"""Localise a difference between the BatchNorm-fusion paths (resnet.BN_STATS_FUSION /
BN_BWD_FUSION on vs off): the small MMBT of tests/test_dp_gpu.py's sync-BN worker (B = 8),
one training step each way from the same weights; per-BatchNorm output, saved statistics and
the flat gradient compared, plus the same batch reordered as the summation-order yardstick."""
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "multi-modal-uncertainty_amd"), os.path.join(HERE, "..")]
from src import resnet as R  # noqa: E402
from src.mmbt import MultimodalBertClf  # noqa: E402
from src.testing import small_args, synthetic_batch  # noqa: E402
from oracle.weights import SMALL  # noqa: E402


def step(x, y, fwd, bwd, perm=None, B=8):
    R.BN_STATS_FUSION, R.BN_BWD_FUSION = fwd, bwd
    torch.manual_seed(0)
    m = MultimodalBertClf(small_args(bert_hidden_dropout=0.0, bert_attn_dropout=0.0, dropout=0.0,
                                     img_precision="bf16")).to("cuda").train()
    outs = {}
    for name, mod in m.named_modules():
        if isinstance(mod, R.BatchNorm2d):
            def hook(mod_, inp, out, name=name):
                o = out.detach().float()
                outs[name] = o[perm.argsort()] if perm is not None else o
            mod.register_forward_hook(hook)
    if perm is not None:
        x, y = tuple(t[perm] for t in x), y[perm]
    m.compute_loss(m(*x), y).backward()
    torch.cuda.synchronize()
    return outs, m.store.grad.clone(), {n: b.detach().clone() for n, b in m.named_buffers() if "running" in n}


def main():
    torch.backends.cudnn.deterministic = True
    B = int(os.environ.get("B", "8"))
    x, y = synthetic_batch(B, 16, lens=[16, 9, 12, 16, 5, 16, 11, 14][:B] * (B // 8 or 1), vocab=SMALL.vocab, seed=31)
    x, y = tuple(t.cuda() for t in x), y.cuda()
    perm = torch.cat([torch.arange(B // 2, B), torch.arange(0, B // 2)]).cuda()
    base = step(x, y, False, False)
    rel = lambda a, b: ((a - b).norm() / b.norm().clamp_min(1e-30)).item()
    for tag, args in (("reordered", (False, False, perm)), ("fwd fusion", (True, False)),
                      ("bwd fusion", (False, True)), ("both", (True, True))):
        outs, g, bufs = step(x, y, *args)
        worst = sorted(((rel(outs[n], base[0][n]), n) for n in base[0]), reverse=True)[:4]
        bw = sorted(((rel(bufs[n], base[2][n]), n) for n in base[2]), reverse=True)[:3]
        print(f"{tag:12s} grad {rel(g, base[1]):.3e}  BN outputs worst {[(f'{e:.1e}', n) for e, n in worst]}")
        print(f"{'':12s} running stats worst {[(f'{e:.1e}', n) for e, n in bw]}", flush=True)
        if tag == "fwd fusion":
            for n in base[0]:  # module order: where the difference starts
                print(f"    {n:45s} out {rel(outs[n], base[0][n]):.2e}  running_mean "
                      f"{rel(bufs[n + '.running_mean'], base[2][n + '.running_mean']):.2e}  running_var "
                      f"{rel(bufs[n + '.running_var'], base[2][n + '.running_var']):.2e}")


if __name__ == "__main__":
    main()
