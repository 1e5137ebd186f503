"""fp32 CPU restatement of the MMBT hot path (test infrastructure only).

Functional: every function takes the state_dict produced by oracle/weights.py
(reference key names) and plain tensors.  Cited reference lines:

* image_encoder      src/mmbt.py:40-45 (resnet152 children[:-2] + AdaptiveAvgPool2d((N,1)),
                     flatten, transpose).  ResNet-152 v1.5 (stride on the 3x3) per
                     torchvision (absent here; restated).
* image_embeddings   src/mmbt.py:58-83
* text_embeddings    pytorch_pretrained_bert 0.6.x BertEmbeddings, called src/mmbt.py:121
* bert_layer         pytorch_pretrained_bert 0.6.x BertLayer (BertSelfAttention /
                     BertSelfOutput / BertIntermediate / BertOutput), called src/mmbt.py:124-126
* pooler             BertPooler, src/mmbt.py:128
* forward*           src/mmbt.py:98-234 + clf src/mmbt.py:245-259
* cross_entropy      src/mmbt.py:243,261-262
"""
import math

import torch
import torch.nn.functional as F

from .weights import FULL

EMB = "enc.txt_embeddings."
ENC = "enc.encoder."
RES = "enc.img_encoder.model."


# ----------------------------------------------------------------------------- ResNet-152
def _bn(sd, p, x, train, momentum=0.1, eps=1e-5):
    return F.batch_norm(x, sd[p + "running_mean"], sd[p + "running_var"], sd[p + "weight"],
                        sd[p + "bias"], training=train, momentum=momentum, eps=eps)


def resnet_trunk(sd, x, cfg=FULL, train=False):
    """[B,3,224,224] -> [B,2048,7,7]; v1.5 bottleneck (stride on conv2)."""
    x = F.conv2d(x, sd[RES + "0.weight"], stride=2, padding=3)
    x = F.relu(_bn(sd, RES + "1.", x, train))
    x = F.max_pool2d(x, 3, 2, 1)
    for li, nblk in enumerate(cfg.resnet_blocks):
        for b in range(nblk):
            p = f"{RES}{4 + li}.{b}."
            stride = 2 if (b == 0 and li > 0) else 1
            y = F.relu(_bn(sd, p + "bn1.", F.conv2d(x, sd[p + "conv1.weight"]), train))
            y = F.relu(_bn(sd, p + "bn2.", F.conv2d(y, sd[p + "conv2.weight"], stride=stride, padding=1), train))
            y = _bn(sd, p + "bn3.", F.conv2d(y, sd[p + "conv3.weight"]), train)
            if b == 0:
                x = _bn(sd, p + "downsample.1.", F.conv2d(x, sd[p + "downsample.0.weight"], stride=stride), train)
            x = F.relu(y + x)
    return x


def row_pool(fmap, n):
    """AdaptiveAvgPool2d((n,1)) restated: bin i covers rows floor(i*H/n) .. ceil((i+1)*H/n)-1,
    all columns.  [B,C,H,W] -> [B,n,C] (src/mmbt.py:30,42-44)."""
    Hh = fmap.shape[2]
    bins = []
    for i in range(n):
        s, e = (i * Hh) // n, -((-(i + 1) * Hh) // n)
        bins.append(fmap[:, :, s:e, :].mean(dim=(2, 3)))
    return torch.stack(bins, dim=1)


def image_encoder(sd, img, cfg=FULL, train=False):
    return row_pool(resnet_trunk(sd, img, cfg, train), cfg.num_image_embeds)


# ----------------------------------------------------------------------------- embeddings
def layer_norm(x, w, b, eps):
    mu = x.mean(-1, keepdim=True)
    var = (x - mu).pow(2).mean(-1, keepdim=True)
    return (x - mu) / torch.sqrt(var + eps) * w + b


def image_embeddings(sd, feats, cfg=FULL):
    """[B,N,2048] -> [B,N+2,768]: [CLS] | Linear(img) | [SEP], pos 0..N+1, type 0, LN."""
    B = feats.shape[0]
    word = sd[EMB + "word_embeddings.weight"]
    proj = feats @ sd["enc.img_embeddings.img_embeddings.weight"].t() + sd["enc.img_embeddings.img_embeddings.bias"]
    tok = torch.cat([word[cfg.cls_id].expand(B, 1, -1), proj, word[cfg.sep_id].expand(B, 1, -1)], 1)
    n = tok.shape[1]
    x = tok + sd[EMB + "position_embeddings.weight"][:n] + sd[EMB + "token_type_embeddings.weight"][0]
    return layer_norm(x, sd[EMB + "LayerNorm.weight"], sd[EMB + "LayerNorm.bias"], cfg.ln_eps)


def text_embeddings(sd, ids, seg, cfg=FULL):
    """[B,T] ids, token types -> [B,T,768]; positions restart at 0 for the text."""
    T = ids.shape[1]
    x = (sd[EMB + "word_embeddings.weight"][ids] + sd[EMB + "position_embeddings.weight"][:T]
         + sd[EMB + "token_type_embeddings.weight"][seg])
    return layer_norm(x, sd[EMB + "LayerNorm.weight"], sd[EMB + "LayerNorm.bias"], cfg.ln_eps)


def extended_mask(mask01):
    """(1 - m) * -10000 as [B,1,1,L] fp32 (src/mmbt.py:108-112)."""
    return (1.0 - mask01.float())[:, None, None, :] * -10000.0


# ----------------------------------------------------------------------------- encoder
def gelu(x):
    return x * 0.5 * (1.0 + torch.erf(x / math.sqrt(2.0)))


def _lin(sd, p, x):
    return x @ sd[p + "weight"].t() + sd[p + "bias"]


def _drop(x, p, gen):
    if p <= 0.0:
        return x
    keep = (torch.rand(x.shape, generator=gen) >= p).to(x.dtype)
    return x * keep / (1.0 - p)


def bert_layer(sd, i, x, ext, cfg=FULL, dropout=0.0, gen=None):
    p = f"{ENC}layer.{i}."
    B, L, H = x.shape
    nh, dh = cfg.heads, H // cfg.heads

    def heads(t):
        return t.view(B, L, nh, dh).transpose(1, 2)

    q = heads(_lin(sd, p + "attention.self.query.", x))
    k = heads(_lin(sd, p + "attention.self.key.", x))
    v = heads(_lin(sd, p + "attention.self.value.", x))
    s = q @ k.transpose(-1, -2) / math.sqrt(dh) + ext
    prob = _drop(torch.softmax(s, dim=-1), dropout, gen)
    ctx = (prob @ v).transpose(1, 2).reshape(B, L, H)
    a = layer_norm(_drop(_lin(sd, p + "attention.output.dense.", ctx), dropout, gen) + x,
                   sd[p + "attention.output.LayerNorm.weight"], sd[p + "attention.output.LayerNorm.bias"], cfg.ln_eps)
    h = gelu(_lin(sd, p + "intermediate.dense.", a))
    return layer_norm(_drop(_lin(sd, p + "output.dense.", h), dropout, gen) + a,
                      sd[p + "output.LayerNorm.weight"], sd[p + "output.LayerNorm.bias"], cfg.ln_eps)


def encoder(sd, x, ext, cfg=FULL, dropout=0.0, gen=None):
    for i in range(cfg.n_layers):
        x = bert_layer(sd, i, x, ext, cfg, dropout, gen)
    return x


def pooler(sd, x):
    return torch.tanh(_lin(sd, "enc.pooler.dense.", x[:, 0]))


def classifier(sd, pooled):
    return _lin(sd, "clf.", pooled)


# ----------------------------------------------------------------------------- variants
def encoder_inputs(sd, txt, segment, img, cfg=FULL, train=False, feats=None):
    """(img-token embeddings [B,N+2,H], text embeddings [B,T,H])."""
    if feats is None:
        feats = image_encoder(sd, img, cfg, train)
    return image_embeddings(sd, feats, cfg), text_embeddings(sd, txt, segment, cfg)


def forward(sd, txt, mask, segment, img, cfg=FULL, variant="full", indices=None,
            train=False, dropout=0.0, gen=None, feats=None, return_pooled=False):
    """MultimodalBertClf.forward / forward_img_only / forward_txt_only / forward_control.

    Argument order is the reference's forward(txt, mask, segment, img) (src/mmbt.py:245);
    ``indices`` is the CLS-prefixed sorted index vector forward_control draws
    (src/mmbt.py:198-201), passed explicitly instead of drawn from the global RNG.
    """
    B = txt.shape[0]
    img_e, txt_e = encoder_inputs(sd, txt, segment, img, cfg, train, feats)
    ones = torch.ones(B, cfg.num_image_embeds + 2, dtype=torch.long)
    if variant == "full":
        x, m = torch.cat([img_e, txt_e], 1), torch.cat([ones, mask.long()], 1)
    elif variant == "img_only":
        x, m = img_e, ones
    elif variant == "txt_only":
        x, m = torch.cat([img_e[:, :1], txt_e], 1), torch.cat([ones[:, :1], mask.long()], 1)
    elif variant == "control":
        idx = torch.as_tensor(indices, dtype=torch.long)
        x, m = torch.cat([img_e, txt_e], 1)[:, idx], torch.cat([ones, mask.long()], 1)[:, idx]
    else:
        raise ValueError(variant)
    hid = encoder(sd, x, extended_mask(m), cfg, dropout, gen)
    pooled = pooler(sd, hid)
    logits = classifier(sd, pooled)
    return (logits, pooled) if return_pooled else logits


def control_indices(total_embeds, num_embeds, gen=None):
    """Index draw of forward_control (src/mmbt.py:198-201): CLS(0) + sorted sample of
    ``num_embeds`` positions out of 1..total_embeds-1."""
    perm = torch.randperm(total_embeds - 1, generator=gen)[:num_embeds] + 1
    out = torch.zeros(num_embeds + 1, dtype=torch.long)
    out[1:] = torch.sort(perm).values
    return out


def cross_entropy(logits, y):
    return F.cross_entropy(logits, y)


def robustness(sd, txt, mask, segment, img, cfg=FULL, n_repeats=20, feats=None):
    """Per-batch loop of eval_mmbt_robustness.py:77-93 (eval mode): full, image-only,
    text-only, then ``n_repeats`` image-control and ``n_repeats`` text-control forwards
    (src/mmbt.py:186-234), each control drawing its index set from the global torch RNG
    in that order; stacked along dim 1 -> [B, 3 + 2n, C].  The trunk output is shared
    (it is a pure function of the image in eval mode)."""
    if feats is None:
        feats = image_encoder(sd, img, cfg)
    T = txt.shape[1]
    total = T + cfg.num_image_embeds + 2
    outs = [forward(sd, txt, mask, segment, img, cfg, v, feats=feats) for v in ("full", "img_only", "txt_only")]
    for modal in ("image", "text"):
        n = cfg.num_image_embeds + 1 if modal == "image" else T
        for _ in range(n_repeats):
            outs.append(forward(sd, txt, mask, segment, img, cfg, "control",
                                indices=control_indices(total, n), feats=feats))
    return torch.stack(outs, dim=1)
