"""A11: the batched 43-variant robustness pass (src/robustness.py) against the
reference's own per-batch loop (eval_mmbt_robustness.py:77-93), recorded by
oracle/gen_golden.py --what robustness from the reference MultimodalBertClf:
[B, 3 + 2n, C] logits in the reference's stacking order (full, image-only, text-only,
n image controls, n text controls), with the control index sets drawn from the global
torch RNG in the reference's order (all image draws, then all text draws).

Tolerance (north star, bf16): max |error| <= 1e-2 * max |reference logit| over the stack.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("tag,cfgname", [("small_t16", "small"), ("full_t508", "full")])
def test_robustness_stack_matches_reference_golden(dev, tag, cfgname):
    from oracle.weights import SMALL, FULL, make_state_dict, checksum
    from src.mmbt import MultimodalBertClf
    from src.robustness import robustness_logits
    from src.testing import small_args, make_args, synthetic_batch
    g = np.load(os.path.join(GOLD, f"robustness_{tag}.npz"))
    cfg = SMALL if cfgname == "small" else FULL
    args = (small_args if cfgname == "small" else make_args)(img_precision="fp32")
    torch.manual_seed(0)
    model = MultimodalBertClf(args)
    sd = make_state_dict(int(g["wseed"]), cfg)
    assert abs(checksum(sd) - float(g["weight_checksum"])) < 1e-6 * float(g["weight_checksum"])
    model.load_state_dict(sd, strict=True)
    model = model.to(dev).eval()
    B, T = g["text"].shape
    x, _ = synthetic_batch(B, T, vocab=cfg.vocab, lens=g["mask"].sum(1).tolist(), seed=int(g["seed"]))
    assert np.array_equal(x[0].numpy(), g["text"])
    assert abs(float(x[3].double().sum()) - float(g["img_sum"])) < 1e-3
    x = tuple(t.to(dev) for t in x)
    n = int(g["n_repeats"])
    torch.manual_seed(int(g["rng_seed"]))
    got = robustness_logits(model, *x, n_repeats=n).cpu().double().numpy()
    ref = g["preds"].astype(np.float64)
    assert got.shape == ref.shape == (B, 3 + 2 * n, cfg.n_classes)
    err = np.abs(got - ref).max(axis=(0, 2))
    scale = np.abs(ref).max()
    assert (err <= 1e-2 * scale).all(), f"per-variant max err {err} vs scale {scale:.3e}"
    # the RNG draw order: the same seed gives the reference's index sets
    from src.mmbt import control_indices
    torch.manual_seed(int(g["rng_seed"]))
    S = T + cfg.num_image_embeds + 2
    img_idx = np.stack([control_indices(S, cfg.num_image_embeds + 1).numpy() for _ in range(n)])
    txt_idx = np.stack([control_indices(S, T).numpy() for _ in range(n)])
    assert np.array_equal(img_idx, g["indices_image"]) and np.array_equal(txt_idx, g["indices_text"])


def test_robustness_equals_per_variant_forwards(dev):
    """The batched pass equals the model's own single-variant forwards called in the
    reference loop's order (same seed): batching by length changes nothing."""
    from oracle.weights import SMALL, make_state_dict
    from src.mmbt import MultimodalBertClf
    from src.robustness import robustness_logits
    from src.testing import small_args, synthetic_batch
    torch.manual_seed(0)
    model = MultimodalBertClf(small_args(img_precision="fp32"))
    model.load_state_dict(make_state_dict(3, SMALL), strict=True)
    model = model.to(dev).eval()
    x, _ = synthetic_batch(3, 20, vocab=SMALL.vocab, lens=[20, 7, 13], seed=8)
    x = tuple(t.to(dev) for t in x)
    n = 4
    torch.manual_seed(99)
    got = robustness_logits(model, *x, n_repeats=n)
    torch.manual_seed(99)
    with torch.no_grad():
        outs = [model(*x), model.forward_img_only(*x), model.forward_txt_only(*x)]
        for modal in ("image", "text"):
            outs += [model.forward_control(*x, modal) for _ in range(n)]
    want = torch.stack(outs, dim=1)
    assert got.shape == want.shape == (3, 3 + 2 * n, 101)
    scale = want.abs().max().item()
    assert (got - want).abs().max().item() <= 2e-3 * scale
