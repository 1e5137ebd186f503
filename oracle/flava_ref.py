"""fp32 CPU restatement of the FLAVA fusion transformer (test infrastructure only).

SURVEY §8f rank 1 / BASELINE config 5: ``src/model.py:225-374`` on precomputed FLAVA
image / text embeddings (src/dataset.py:196-226).  Functional: every function takes
the state_dict produced by ``make_state_dict`` (reference key names) and plain tensors.

Cited reference lines:
* LayerNorm (fp32 inside)       src/model.py:174-180 (nn.LayerNorm, eps 1e-5)
* QuickGELU                     src/model.py:183-185   x * sigmoid(1.702 x)
* ResidualAttentionBlock        src/model.py:188-212   pre-LN; x + attn(ln_1 x); x + mlp(ln_2 x);
                                mlp = OrderedDict(c_fc, dropout, gelu, c_proj, dropout) (:196-200):
                                the repeated "dropout" key keeps its FIRST position, so the
                                Sequential is c_fc -> Dropout -> QuickGELU -> c_proj (no
                                trailing dropout)
* nn.MultiheadAttention quirk   src/model.py:193,207   batch_first=False while the block receives
                                [B, L, E]: the attention runs over the BATCH axis (sequence = B,
                                "batch" = the L token positions), per head of E / n_head dims
* FlavaFusionTransfomer         src/model.py:225-304   projections, cat, ln_pre, encoder, ln_post,
                                heads (avg_pool: image / text span means; else token i per head)
* ...withCLSToken               src/model.py:306-374   class_embeddings [E, out_dim] prepended
* compute_loss                  src/model.py:290-304   train: CE per member; eval: CE of the mean
* data_forming_func_transformer src/dataset.py:30-54
"""
import math
import zlib
from collections import OrderedDict
from dataclasses import dataclass

import torch
import torch.nn.functional as F


@dataclass(frozen=True)
class FlavaConfig:
    width: int = 768
    heads: int = 3
    layers: int = 3
    n_classes: int = 2
    out_dim: int = 1
    clstoken: bool = False
    avg_pool: bool = False
    drop: float = 0.0
    img_hidden: int = 768
    txt_hidden: int = 768


def key_shapes(cfg):
    """(key, shape, kind) in the reference state_dict order (src/model.py:227-259, 306-330)."""
    E = cfg.width
    # the module's own Parameter precedes its submodules in state_dict order
    out = [("class_embeddings", (E, cfg.out_dim), "cls")] if cfg.clstoken else []
    for i in range(cfg.layers):
        p = f"mm_encoder.resblocks.{i}."
        out += [(p + "attn.in_proj_weight", (3 * E, E), "w"), (p + "attn.in_proj_bias", (3 * E,), "b"),
                (p + "attn.out_proj.weight", (E, E), "w"), (p + "attn.out_proj.bias", (E,), "b"),
                (p + "ln_1.weight", (E,), "ln_w"), (p + "ln_1.bias", (E,), "ln_b"),
                (p + "mlp.c_fc.weight", (4 * E, E), "w"), (p + "mlp.c_fc.bias", (4 * E,), "b"),
                (p + "mlp.c_proj.weight", (E, 4 * E), "w"), (p + "mlp.c_proj.bias", (E,), "b"),
                (p + "ln_2.weight", (E,), "ln_w"), (p + "ln_2.bias", (E,), "ln_b")]
    out += [("ln_pre.weight", (E,), "ln_w"), ("ln_pre.bias", (E,), "ln_b"),
            ("ln_post.weight", (E,), "ln_w"), ("ln_post.bias", (E,), "ln_b"),
            ("image_to_mm_projection.weight", (E, cfg.img_hidden), "w"), ("image_to_mm_projection.bias", (E,), "b"),
            ("text_to_mm_projection.weight", (E, cfg.txt_hidden), "w"), ("text_to_mm_projection.bias", (E,), "b")]
    for i in range(cfg.out_dim):
        out += [(f"output_layers.{i}.weight", (cfg.n_classes, E), "w"), (f"output_layers.{i}.bias", (cfg.n_classes,), "b")]
    return out


def make_state_dict(seed, cfg):
    """Seeded recipe (the build's own; no FLAVA checkpoint exists offline): weights
    N(0, 1/sqrt(fan_in)), biases N(0, 0.02), LayerNorm affine perturbed away from 1 / 0."""
    sd = OrderedDict()
    for name, shape, kind in key_shapes(cfg):
        g = torch.Generator()
        g.manual_seed((int(seed) * 1000003 + zlib.crc32(("flava/" + name).encode())) & 0x7FFFFFFFFFFF)
        if kind == "w":
            t = torch.randn(shape, generator=g) / math.sqrt(shape[1])
        elif kind == "b":
            t = torch.randn(shape, generator=g) * 0.02
        elif kind == "ln_w":
            t = 1.0 + 0.1 * torch.randn(shape, generator=g)
        elif kind == "ln_b":
            t = 0.05 * torch.randn(shape, generator=g)
        else:  # class_embeddings: scale * randn (src/model.py:327-328)
            t = cfg.width ** -0.5 * torch.randn(shape, generator=g)
        sd[name] = t
    return sd


def make_inputs(B, L_img, L_txt, n_classes, out_dim, seed, width=768):
    """Synthetic FLAVA embeddings in collate_fn_flava order (src/dataset.py:216-226)."""
    g = torch.Generator().manual_seed(seed)
    img = torch.randn(B, L_img, width, generator=g)
    txt = torch.randn(B, L_txt, width, generator=g)
    y = torch.randint(0, n_classes, (B,), generator=g)
    return img, txt, y


def _ln(x, sd, p, eps=1e-5):
    return F.layer_norm(x, (x.shape[-1],), sd[p + "weight"], sd[p + "bias"], eps)


def mha_batch_axis(x, sd, p, heads):
    """nn.MultiheadAttention(x, x, x) with batch_first=False on an [B, L, E] tensor
    (src/model.py:205-207): sequence axis = B, batch axis = L."""
    S, N, E = x.shape
    d = E // heads
    qkv = x @ sd[p + "in_proj_weight"].t() + sd[p + "in_proj_bias"]
    q, k, v = qkv.split(E, dim=-1)
    # [S, N, E] -> [N*heads, S, d]
    q, k, v = (t.reshape(S, N * heads, d).transpose(0, 1) for t in (q, k, v))
    a = torch.softmax((q @ k.transpose(1, 2)) / math.sqrt(d), dim=-1)
    o = (a @ v).transpose(0, 1).reshape(S, N, E)
    return o @ sd[p + "out_proj.weight"].t() + sd[p + "out_proj.bias"]


def _dropout(x, p, train, gen):
    if not train or p == 0.0:
        return x
    keep = (torch.rand(x.shape, generator=gen) >= p).to(x.dtype)
    return x * keep / (1.0 - p)


def block(x, sd, i, cfg, train=False, gen=None):
    p = f"mm_encoder.resblocks.{i}."
    x = x + mha_batch_axis(_ln(x, sd, p + "ln_1."), sd, p + "attn.", cfg.heads)
    h = _ln(x, sd, p + "ln_2.") @ sd[p + "mlp.c_fc.weight"].t() + sd[p + "mlp.c_fc.bias"]
    h = _dropout(h, cfg.drop, train, gen)
    h = h * torch.sigmoid(1.702 * h)
    return x + h @ sd[p + "mlp.c_proj.weight"].t() + sd[p + "mlp.c_proj.bias"]


def forward(sd, img, txt, cfg, train=False, gen=None):
    """-> logits [B, out_dim, n_classes] (src/model.py:261-288 / 332-360)."""
    img = img @ sd["image_to_mm_projection.weight"].t() + sd["image_to_mm_projection.bias"]
    txt = txt @ sd["text_to_mm_projection.weight"].t() + sd["text_to_mm_projection.bias"]
    l_img, l_txt = img.shape[1], txt.shape[1]
    x = torch.cat((img, txt), dim=1)
    if cfg.clstoken:
        cls = sd["class_embeddings"].t().unsqueeze(0).expand(x.shape[0], -1, -1)
        x = torch.cat([cls, x], dim=1)
    x = _ln(x, sd, "ln_pre.")
    for i in range(cfg.layers):
        x = block(x, sd, i, cfg, train, gen)
    x = _ln(x, sd, "ln_post.")
    outs = []
    if cfg.avg_pool and not cfg.clstoken:
        outs.append(x[:, :l_img].mean(1) @ sd["output_layers.0.weight"].t() + sd["output_layers.0.bias"])
        outs.append(x[:, l_img:l_img + l_txt].mean(1) @ sd["output_layers.1.weight"].t() + sd["output_layers.1.bias"])
    else:
        for i in range(cfg.out_dim):
            outs.append(x[:, i] @ sd[f"output_layers.{i}.weight"].t() + sd[f"output_layers.{i}.bias"])
    return torch.stack(outs, dim=1)


def compute_loss(y_hat, y, eval=False):
    """src/model.py:290-304: train -> CE over every (sample, member); eval -> CE of the member mean."""
    y = y.reshape(-1)
    y_hat = y_hat.mean(1) if eval else y_hat.reshape(-1, y_hat.shape[2])
    return F.cross_entropy(y_hat, y)


def data_forming(img, txt, y, phase, model_type, gen=None):
    """src/dataset.py:30-54 (MIMO permutations drawn from ``gen`` or the global RNG)."""
    if model_type == "Vanilla" and phase == "train":
        y = y.unsqueeze(1).repeat(1, 1)
    elif model_type == "MultiHead" and phase == "train":
        y = y.unsqueeze(1).repeat(1, 2)
    elif model_type == "MIMO-shuffle-instance" and phase == "train":
        idx = torch.randperm(img.size(0), generator=gen)
        img, y_img = img[idx], y[idx]
        idx = torch.randperm(img.size(0), generator=gen)
        txt, y_txt = txt[idx], y[idx]
        y = torch.stack([y_img, y_txt], dim=1)
    return img, txt, y
