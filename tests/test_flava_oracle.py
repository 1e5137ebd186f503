"""CPU: the FLAVA fusion-transformer restatement (oracle/flava_ref.py) is pinned against the
reference's own src/model.py outputs (tests/golden/flava_*.npz, oracle/gen_golden.py)."""
import json
import os

import numpy as np
import pytest
import torch

GOLD = os.path.join(os.path.dirname(__file__), "golden")
CASES = {"vanilla": dict(out_dim=1), "multihead_avgpool": dict(out_dim=2, avg_pool=True),
         "cls_multihead": dict(out_dim=2, clstoken=True), "full_b32": dict(out_dim=2)}


def load_case(tag):
    from oracle import flava_ref as FR
    g = np.load(os.path.join(GOLD, f"flava_{tag}.npz"))
    cfg = FR.FlavaConfig(**CASES[tag])
    sd = FR.make_state_dict(int(g["seed"]), cfg)
    img, txt, y = FR.make_inputs(int(g["B"]), int(g["L_img"]), int(g["L_txt"]), cfg.n_classes, cfg.out_dim,
                                 int(g["seed"]) + 1)
    assert abs(float(img.double().sum()) - float(g["img_sum"])) < 1e-6 * abs(float(g["img_sum"])) + 1e-6
    assert np.array_equal(y.numpy(), g["y"])
    return g, cfg, sd, img, txt, y


@pytest.mark.parametrize("tag", list(CASES))
def test_flava_oracle_matches_reference(tag):
    from oracle import flava_ref as FR
    g, cfg, sd, img, txt, y = load_case(tag)
    keys = json.load(open(os.path.join(GOLD, f"flava_{tag}_keys.json")))["state_dict_keys"]
    assert keys == [k for k, *_ in FR.key_shapes(cfg)]
    with torch.no_grad():
        lo = FR.forward(sd, img, txt, cfg)
    np.testing.assert_allclose(lo.numpy(), g["logits"], rtol=1e-4, atol=1e-5)
    assert abs(float(FR.compute_loss(lo, y, eval=True)) - float(g["loss_eval"])) < 1e-5
    # train mode (dropout 0): loss and every parameter's gradient norm
    params = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
    img2, txt2, y2 = FR.data_forming(img, txt, y, "train", "Vanilla" if cfg.out_dim == 1 else "MultiHead")
    lo = FR.forward(params, img2, txt2, cfg, train=True)
    loss = FR.compute_loss(lo, y2)
    loss.backward()
    assert abs(float(loss) - float(g["loss_train"])) < 1e-5
    names = json.load(open(os.path.join(GOLD, f"flava_{tag}_keys.json")))["named_parameters"]
    norms = np.array([float(params[n].grad.double().norm()) for n in names])
    np.testing.assert_allclose(norms, g["grad_norms"], rtol=2e-4, atol=1e-7)


def test_flava_mimo_forming_follows_reference_rng():
    from oracle import flava_ref as FR
    g, cfg, sd, img, txt, y = load_case("vanilla")
    torch.manual_seed(99)
    pi, pt, py = FR.data_forming(img, txt, y, "train", "MIMO-shuffle-instance")
    assert np.array_equal(py.numpy(), g["mimo_y"])
    np.testing.assert_allclose(pi.double().sum((1, 2)).numpy(), g["mimo_img_rowsum"], rtol=1e-12)
    np.testing.assert_allclose(pt.double().sum((1, 2)).numpy(), g["mimo_txt_rowsum"], rtol=1e-12)
