"""CPU emulation of the bf16 trunk's storage precision (which stored tensors, if kept in f32,
bring the product trunk within the north star's 1e-2 of the fp32 reference).

The oracle's functional ResNet-152 (oracle/mmbt_ref.resnet_trunk) is re-run with bf16
rounding inserted where the HIP trunk stores a bf16 tensor: conv operands / filters, conv
outputs, BatchNorm outputs, the block output (residual stream); in the backward the same
points round the gradient (the HIP trunk's activation gradients are bf16 too).  BERT, the
embeddings and the head stay fp32, so what moves is the trunk's contribution alone.  For each
storage variant it prints what tests/test_mmbt_gpu.py measures on the GPU: the train-step
trunk grad-norm relative errors (median / p90 / max over tensors above the floor) against the
golden, and the BN-fitted eval logits of the 5 forward variants.

    python tools/trunk_precision.py [full_t508|small_t16|small_b8] [variant ...]
"""
import json
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..")]
from oracle import mmbt_ref as R  # noqa: E402
from oracle.weights import FULL, SMALL, make_state_dict  # noqa: E402
import dataclasses  # noqa: E402

GOLD = os.path.join(HERE, "..", "tests", "golden")
RES = R.RES


def _rb(t):
    return t.to(torch.bfloat16).to(t.dtype)


class _Q(torch.autograd.Function):
    """round the value (fwd) and / or the gradient (bwd) to bf16"""

    @staticmethod
    def forward(ctx, x, v, g):
        ctx.g = g
        return _rb(x) if v else x.clone()

    @staticmethod
    def backward(ctx, dy):
        return (_rb(dy) if ctx.g else dy), None, None


def _res8(t):
    """bf16 hi + the 8-bit stream residue of csrc/batchnorm.hip (res = rint((v - hi) * 2^15 / 2^e(hi)),
    clamped to +-127): the value the next block's skip reads"""
    hi = _rb(t)
    e = torch.floor(torch.log2(hi.abs().clamp_min(1e-30)))
    s = torch.exp2(e)
    r = torch.clamp(torch.round((t - hi) / s * 32768.0), -127, 127)
    return torch.where(hi == 0, hi, hi + r * s / 32768.0)


class _R8(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return _res8(x)

    @staticmethod
    def backward(ctx, dy):
        return _rb(dy)


def Q(x, v=True, g=True):
    if not (v or g):
        return x
    return _Q.apply(x, v, g)


# storage variants: which tensors are f32 instead of bf16
VARIANTS = {
    "fp32": None,
    "bf16 (round-4 HIP trunk)": dict(),
    "f32 stream fwd": dict(stream_v=False),
    "f32 stream fwd+bwd": dict(stream_v=False, stream_g=False),
    "f32 stream + f32 bn3 in": dict(stream_v=False, stream_g=False, c3=False),
    "bf16 + 8-bit stream residue": dict(res8=True),
    "f32 stream layer4": dict(stream_v=False, stages=(3,)),
    "f32 stream layer3+4": dict(stream_v=False, stages=(2, 3)),
    "bf16 grads only": dict(stream_v=False, conv_v=False, bn_v=False, w=False, c3=False, img=False),
    "bf16 values only": dict(stream_g=False, conv_g=False, bn_g=False),
    "res8, f32 image": dict(res8=True, img=False),
    "res8, f32 image + stem filter": dict(res8=True, img=False, stem_w=False),
    "res8, f32 stem out": dict(res8=True, stem_out=False),
    "res8, f32 image + stem filter + out": dict(res8=True, img=False, stem_w=False, stem_out=False),
}


def trunk(sd, img, cfg, train, o, momentum=0.1):
    """the oracle's resnet_trunk with bf16 storage points (o = variant dict, None = fp32)"""
    if o is None:
        return R.resnet_trunk(sd, img, cfg, train) if momentum == 0.1 else _trunk_m(sd, img, cfg, train, momentum)
    sv, sg = o.get("stream_v", True), o.get("stream_g", True)
    cv, cg = o.get("conv_v", True), o.get("conv_g", True)
    bv, bg = o.get("bn_v", True), o.get("bn_g", True)
    wq = o.get("w", True)
    c3q = o.get("c3", True)
    stages = o.get("stages", (0, 1, 2, 3))

    def W(k):
        return Q(sd[k], wq, False)

    def bn(p, x):
        return F.batch_norm(x, sd[p + "running_mean"], sd[p + "running_var"], sd[p + "weight"], sd[p + "bias"],
                            training=train, momentum=momentum, eps=1e-5)

    x = Q(img, o.get("img", True), False)
    x = Q(F.conv2d(x, Q(sd[RES + "0.weight"], o.get("stem_w", wq), False), stride=2, padding=3),
          cv and o.get("stem_out", True), cg)
    x = Q(F.relu(bn(RES + "1.", x)), bv, bg)
    x = F.max_pool2d(x, 3, 2, 1)
    for li, nblk in enumerate(cfg.resnet_blocks):
        for b in range(nblk):
            p = f"{RES}{4 + li}.{b}."
            stride = 2 if (b == 0 and li > 0) else 1
            sv = o.get("stream_v", True) or li not in stages
            xin = Q(x, True, False) if (not sv or o.get("res8")) else x  # the conv operand is always bf16
            y = Q(F.conv2d(xin, W(p + "conv1.weight")), cv, cg)
            y = Q(F.relu(bn(p + "bn1.", y)), bv, bg)
            y = Q(F.conv2d(y, W(p + "conv2.weight"), stride=stride, padding=1), cv, cg)
            y = Q(F.relu(bn(p + "bn2.", y)), bv, bg)
            y = Q(F.conv2d(y, W(p + "conv3.weight")), c3q and cv, c3q and cg)
            y = bn(p + "bn3.", y)
            if b == 0:
                s = Q(F.conv2d(xin, W(p + "downsample.0.weight"), stride=stride), cv, cg)
                x = bn(p + "downsample.1.", s)
                x = _R8.apply(x) if o.get("res8") else Q(x, sv, sg)  # the downsample BN's output: the skip
            x = F.relu(y + x)
            x = _R8.apply(x) if o.get("res8") else Q(x, sv, sg)
    return x


def _trunk_m(sd, img, cfg, train, momentum):
    x = F.conv2d(img, sd[RES + "0.weight"], stride=2, padding=3)

    def bn(p, x):
        return F.batch_norm(x, sd[p + "running_mean"], sd[p + "running_var"], sd[p + "weight"], sd[p + "bias"],
                            training=train, momentum=momentum, eps=1e-5)
    x = F.max_pool2d(F.relu(bn(RES + "1.", x)), 3, 2, 1)
    for li, nblk in enumerate(cfg.resnet_blocks):
        for b in range(nblk):
            p = f"{RES}{4 + li}.{b}."
            stride = 2 if (b == 0 and li > 0) else 1
            y = F.relu(bn(p + "bn1.", F.conv2d(x, sd[p + "conv1.weight"])))
            y = F.relu(bn(p + "bn2.", F.conv2d(y, sd[p + "conv2.weight"], stride=stride, padding=1)))
            y = bn(p + "bn3.", F.conv2d(y, sd[p + "conv3.weight"]))
            if b == 0:
                x = bn(p + "downsample.1.", F.conv2d(x, sd[p + "downsample.0.weight"], stride=stride))
            x = F.relu(y + x)
    return x


def load(tag):
    g = np.load(os.path.join(GOLD, f"mmbt_{tag}.npz"))
    names = json.load(open(os.path.join(GOLD, f"mmbt_{tag}_keys.json")))["named_parameters"]
    cfg = SMALL if tag.startswith("small") else FULL  # (bn_last_gamma below: the FULL_C fixtures)
    if "bn_last_gamma" in g:
        cfg = dataclasses.replace(cfg, bn_last_gamma=float(g["bn_last_gamma"]))
    sd = make_state_dict(int(g["wseed"]), cfg)
    B, T = g["text"].shape
    gen = torch.Generator().manual_seed(int(g["seed"]))
    torch.randint(1000, cfg.vocab, (B, T), generator=gen)
    img = torch.randn(B, 3, 224, 224, generator=gen)
    assert abs(float(img.double().sum()) - float(g["img_sum"])) < 1e-3
    x = tuple(torch.from_numpy(g[k]) for k in ("text", "segment", "mask")) + (img,)
    return g, names, cfg, sd, x, torch.from_numpy(g["y"])


def train_grads(g, names, cfg, sd, x, y, o):
    sd = {k: (v.clone().requires_grad_(True) if v.is_floating_point() and "running" not in k else v.clone())
          for k, v in sd.items()}
    txt, seg, mask, img = x
    feats = R.row_pool(trunk(sd, img, cfg, True, o), cfg.num_image_embeds)
    # reference argument order: forward(txt, mask, segment, img) receives (text, segment, mask, img)
    logits = R.forward(sd, txt, seg, mask, img, cfg, "full", feats=feats)
    loss = R.cross_entropy(logits, y)
    loss.backward()
    norms = {}
    for n in names:
        k = n.replace("enc.img_embeddings.LayerNorm", "enc.txt_embeddings.LayerNorm")
        t = sd.get(n, sd.get(k))
        norms[n] = float(t.grad.double().norm()) if t is not None and t.grad is not None else 0.0
    return float(loss), norms


def bnfit_logits(g, cfg, sd, x, o):
    sd = {k: v.clone() for k, v in sd.items()}
    txt, seg, mask, img = x
    with torch.no_grad():
        trunk(sd, img, cfg, True, o, momentum=1.0)
        feats = R.row_pool(trunk(sd, img, cfg, False, o), cfg.num_image_embeds)
        out = {"full": R.forward(sd, txt, seg, mask, img, cfg, "full", feats=feats),
               "img_only": R.forward(sd, txt, seg, mask, img, cfg, "img_only", feats=feats),
               "txt_only": R.forward(sd, txt, seg, mask, img, cfg, "txt_only", feats=feats)}
        for modal in ("image", "text"):
            out[f"control_{modal}"] = R.forward(sd, txt, seg, mask, img, cfg, "control",
                                                indices=torch.from_numpy(g[f"indices_control_{modal}"]), feats=feats)
    return {k: v.numpy() for k, v in out.items()}


def main():
    args = sys.argv[1:]
    gl = None
    if args and args[0].startswith("--gamma-last="):
        gl = float(args.pop(0).split("=")[1])
    tag = args[0] if args else "full_t508"
    want = args[1:] or list(VARIANTS)
    torch.set_num_threads(os.cpu_count())
    g, names, cfg, sd, x, y = load(tag)
    ref = dict(zip(names, (float(v) for v in g["grad_norms"])))
    if gl is not None:  # another trunk recipe: the fp32 restatement is the reference
        g = dict(g)
        for k in sd:
            if k.endswith("bn3.weight"):
                sd[k] = sd[k] - 0.3 + gl
        _, n32 = train_grads(g, names, cfg, sd, x, y, None)
        ref = n32
        g["grad_norms"] = np.array([n32[n] for n in names])
        for k, v in bnfit_logits(g, cfg, sd, x, None).items():
            g[f"bnfit_logits_{k}"] = v
        print(f"[{tag}] bn3 gamma recipe N({gl}, 0.02): reference = the fp32 restatement")
    floor = 1e-4 * float(np.max(g["grad_norms"]))
    trunk_names = [n for n in names if "img_encoder" in n and ref[n] > floor]
    for v in want:
        o = VARIANTS[v]
        loss, norms = train_grads(g, names, cfg, sd, x, y, o)
        e = np.array([abs(norms[n] - ref[n]) / ref[n] for n in trunk_names])
        worst = trunk_names[int(e.argmax())]
        lg = bnfit_logits(g, cfg, sd, x, o)
        le = {k: float(np.abs(lg[k] - g[f"bnfit_logits_{k}"]).max() / np.abs(g[f"bnfit_logits_{k}"]).max())
              for k in lg}
        print(f"[{tag}] {v:28s} loss {abs(loss - float(g['loss_train'])) / float(g['loss_train']):.1e} | trunk grads "
              f"median {np.median(e):.2e} p90 {np.quantile(e, 0.9):.2e} max {e.max():.2e} "
              f"(>1e-2: {(e > 1e-2).sum()}/{len(e)}; worst {worst.replace('enc.img_encoder.model.', '')}) | bnfit "
              + " ".join(f"{k} {le[k]:.1e}" for k in lg), flush=True)


if __name__ == "__main__":
    main()
