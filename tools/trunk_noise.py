"""Where the bf16 trunk's gradient noise comes from: one train step of the golden MMBT batch
(tests/golden/mmbt_*.npz, B = 2) with the product trunk and with single components swapped
for PyTorch's own bf16 ops; per-tensor grad-norm relative error against the fp32 reference's
norms (the golden), summarised over the trunk tensors (median / 90th percentile / max)."""
import json
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "multi-modal-uncertainty_amd"), os.path.join(HERE, "..")]
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
from test_mmbt_gpu import GOLD, _train_step, fixture  # noqa: E402
from src import resnet as R  # noqa: E402


def torch_bn(x, w, b, skip, bn, relu, sink=None, *_):
    # (MIOpen's NHWC batch-norm crashes in host code below batch 8: resnet.BatchNorm2d's guard)
    with torch.backends.cudnn.flags(enabled=x.shape[0] >= R.BatchNorm2d.MIOPEN_MIN_BATCH):
        y = F.batch_norm(x, bn.running_mean, bn.running_var, w, b, True, bn.momentum, bn.eps)
    if skip is not None:
        y = y + skip
    return torch.relu(y) if relu else y


VARIANTS = {
    "hip": {},
    "hip, bf16 stream (no residue)": {"STREAM_RESIDUE": False},
    "hip, convs on MIOpen": {"_mmu_conv": lambda *a: (False, False, False), "_mmu_1x1": lambda *a: (False, False, False)},
    "hip, BN on torch": {"bn": True},
    "hip, stem on MIOpen": {"_is_stem": lambda *a: False},
    "hip, no BN-bwd fusion": {"BN_BWD_FUSION": False},
    "hip, no BN fusion": {"BN_BWD_FUSION": False, "BN_STATS_FUSION": False},
}


def run(tag, cfgname, dev="cuda"):
    g, cfg = fixture(tag)
    names = json.load(open(os.path.join(GOLD, f"mmbt_{tag}_keys.json")))["named_parameters"]
    ref = dict(zip(names, (float(v) for v in g["grad_norms"])))
    floor = 1e-4 * float(np.max(g["grad_norms"]))
    trunk = [n for n in names if "img_encoder" in n and ref[n] > floor]

    def summ(norms):
        e = np.array([abs(norms[n] - ref[n]) / ref[n] for n in trunk])
        return f"median {np.median(e):.2e}  p90 {np.quantile(e, 0.9):.2e}  max {e.max():.2e}  (>1e-2: {(e > 1e-2).sum()}/{len(e)})"
    _, tn, _, _ = _train_step(cfgname, g, dev, "torch_bf16", cfg)
    print(f"[{tag}] torch bf16            {summ(tn)}", flush=True)
    for name, patch in VARIANTS.items():
        saved = {}
        for k, v in patch.items():
            if k == "bn":
                saved["bn"] = R._BatchNormAct.apply
                R._BatchNormAct.apply = torch_bn
            else:
                saved[k] = getattr(R, k)
                setattr(R, k, v)
        try:
            _, hn, _, _ = _train_step(cfgname, g, dev, "bf16", cfg)
        finally:
            for k, v in saved.items():
                if k == "bn":
                    R._BatchNormAct.apply = v
                else:
                    setattr(R, k, v)
        print(f"[{tag}] {name:22s} {summ(hn)}", flush=True)


if __name__ == "__main__":
    for tag, cfgname in (("small_t16", "small"), ("small_b8", "small"), ("full_t508c", "full")):
        run(tag, cfgname)
