"""One tiny MMBT train step on cuda:0 through the HIP path, checked against the CPU oracle
(used by __graft_entry__.smoke(); the oracle is test infrastructure, never the product path)."""
import torch


def run_smoke():
    if not torch.cuda.is_available():
        raise RuntimeError("smoke: no HIP device")
    from oracle import mmbt_ref as R
    from oracle.weights import SMALL, make_state_dict
    from . import _native
    from .mmbt import MultimodalBertClf
    from .optim import BertAdam
    from .testing import small_args, synthetic_batch

    _native.load()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    args = small_args(bert_hidden_dropout=0.0, bert_attn_dropout=0.0)
    model = MultimodalBertClf(args)
    sd = make_state_dict(0, SMALL)
    model.load_state_dict(sd, strict=True)
    model.to(dev)
    x, y = synthetic_batch(2, 16, lens=[16, 9], vocab=SMALL.vocab, seed=0)
    with torch.no_grad():
        ref = R.forward(sd, x[0], x[1], x[2], x[3], SMALL)  # model(*x) order (src/framework.py:175)
    model.eval()
    with torch.no_grad():
        out = model(*(t.to(dev) for t in x)).float().cpu()
    err = (out - ref).abs().max().item()
    scale = ref.abs().max().item()
    if not err <= 2e-2 * scale + 2e-3:
        raise AssertionError(f"smoke: logits differ from oracle: max err {err:.3e} (scale {scale:.3e})")
    model.train()
    opt = BertAdam(model.parameters(), lr=1e-4, warmup=0.1, t_total=10)
    opt.zero_grad()
    loss = model.compute_loss(model(*(t.to(dev) for t in x)), y.to(dev))
    loss.backward()
    opt.step()
    opt.zero_grad()
    torch.cuda.synchronize()
    if opt._fused is None:
        raise AssertionError("smoke: fused BertAdam path not taken")
    if not torch.isfinite(loss).item():
        raise AssertionError("smoke: non-finite loss")
    print(f"smoke ok: logits max err {err:.2e} (scale {scale:.2e}), train loss {loss.item():.4f}")
