"""FLAVA fusion transformer on the HIP kernels -- drop-in for the reference src/model.py:174-374
(BASELINE config 5: precomputed FLAVA embeddings of Hateful Memes).

Same class names, constructor arguments, module tree and state_dict keys as the
reference (``mm_encoder.resblocks.{i}.attn.in_proj_weight`` ...), so reference
checkpoints load strictly.  The parameters live in the reference's own module types
(nn.MultiheadAttention / nn.Linear / nn.LayerNorm); the compute does not go through
them: on a HIP device every block runs as ONE autograd node over bf16 token-major
activations [B*L, E] (row b*L + l):

  h1  = LN1(x)                                   mmu_layernorm_fwd (eps 1e-5)
  qkv = h1 Win^T + bin                           mmu_gemm  STORE+bias      [M, 3E]
  O   = attention over the SAMPLE axis           mmu_seqattn_fwd  (the batch_first=False
                                                 quirk, src/model.py:193,207: sequence = B)
  x1  = x + O Wo^T + bo                          mmu_gemm  BIAS_DROP_RES (p = 0)
  h2  = LN2(x1)                                  mmu_layernorm_fwd
  H   = qgelu(dropout(h2 W1^T + b1))             mmu_gemm  BIAS_DROP_QGELU (saves dH/dz)
  y   = x1 + H W2^T + b2                         mmu_gemm  BIAS_DROP_RES (p = 0)
(the reference's mlp OrderedDict repeats the key "dropout", which keeps its first slot:
c_fc -> Dropout -> QuickGELU -> c_proj, no trailing dropout -- src/model.py:196-200)
Backward: DGELU-epilogue data grads (dH/dz saved by the forward), split-K f32 weight grads,
mmu_layernorm_bwd_res (LN' + the residual's gradient, column sums = the out-proj /
c_proj bias grads), mmu_seqattn_bwd.  Projections (mmu_gemm, batched into the
concatenated sequence) and ln_pre / ln_post (mmu_layernorm) are HIP too; the heads
([B, E] x [E, n_classes] per member) and the loss stay torch f32.

There is no CPU path: CPU tensors raise (DESIGN.md "no fallback").
"""
from collections import OrderedDict
from typing import Any

import torch
import torch.nn as nn

from . import encoder as _enc  # block_timing: bench.py's fused-block roofline
from . import kernels as K

bf16 = torch.bfloat16
LN_EPS = 1e-5


class LayerNorm(nn.LayerNorm):
    """Subclass torch's LayerNorm to handle fp16 (src/model.py:174-180): computes in f32."""

    def forward(self, x):
        return LNFunction.apply(x, self.weight, self.bias, self.eps)


class QuickGELU(nn.Module):
    """x * sigmoid(1.702 x) (src/model.py:183-185); fused into the c_fc GEMM epilogue."""

    def forward(self, x):
        return x * torch.sigmoid(1.702 * x)


# ------------------------------------------------------------------------------ autograd
def _rows(x):
    return x.reshape(-1, x.shape[-1])


class LNFunction(torch.autograd.Function):
    """LayerNorm over the last dim of a bf16 tensor (ln_pre / ln_post / standalone)."""

    @staticmethod
    def forward(ctx, x, w, b, eps):
        X = _rows(x.contiguous()).to(bf16)
        M, E = X.shape
        Y = torch.empty_like(X)
        mean = torch.empty(M, dtype=torch.float32, device=X.device)
        rstd = torch.empty_like(mean)
        K.layernorm_fwd(X, w, b, Y, mean, rstd, eps)
        ctx.save_for_backward(X, w, mean, rstd)
        ctx.shape = x.shape
        return Y.view(x.shape)

    @staticmethod
    def backward(ctx, dy):
        X, w, mean, rstd = ctx.saved_tensors
        dY = _rows(dy.contiguous()).to(bf16)
        M, E = X.shape
        dX = torch.empty_like(X)
        P = K.ln_parts(M)
        pw = torch.empty(P, E, dtype=torch.float32, device=X.device)
        pb = torch.empty_like(pw)
        K.layernorm_bwd(dY, X, mean, rstd, w, dX, None, 0.0, 0, pw, pb, None)
        gw = torch.zeros_like(w)
        gb = torch.zeros_like(w)
        K.colsum_reduce(pw, gw)
        K.colsum_reduce(pb, gb)
        return dX.view(ctx.shape), gw, gb, None


class ProjFunction(torch.autograd.Function):
    """y[b, off+i] = x[b, i] W^T + bias written into rows of the concatenated sequence
    buffer ``out`` [B, L, E] (one batched mmu_gemm: batch = B, row strides L_in / L)."""

    @staticmethod
    def forward(ctx, x, w, b, out, off):
        B, Li, Ein = x.shape
        E, L = w.shape[0], out.shape[1]
        X = x.contiguous().to(bf16)
        W16 = w.to(bf16)
        dst = out[:, off:off + Li]
        K.gemm(X, Ein, True, W16, Ein, True, dst, E, Li, E, Ein, epi=K.epilogue(K.EPI_STORE, bias=b), batch=B,
               sA=Li * Ein, sB=0, sC=L * E)
        ctx.save_for_backward(X)
        ctx.meta = (off, Li, w.shape)
        ctx.mark_dirty(out)
        return out

    @staticmethod
    def backward(ctx, dout):
        (X,) = ctx.saved_tensors
        off, Li, wshape = ctx.meta
        B = X.shape[0]
        E, Ein = wshape
        dY = dout[:, off:off + Li].contiguous().to(bf16).view(B * Li, E)
        gw = torch.empty(wshape, dtype=torch.float32, device=X.device)
        K.gemm(dY, E, False, X.view(B * Li, Ein), Ein, False, gw, Ein, E, Ein, B * Li, epi=K.epilogue(K.EPI_STORE))
        gb = torch.empty(E, dtype=torch.float32, device=X.device)
        K.colsum_bf16(dY, gb)
        return None, gw, gb, dout, None


def _mlp_seed(train, drop):
    if not train or drop <= 0.0:
        return 0
    return int(torch.randint(0, 2 ** 62, (1,), dtype=torch.int64))


class BlockFunction(torch.autograd.Function):
    """One pre-LN ResidualAttentionBlock (src/model.py:188-212) on x [B, L, E] bf16."""

    @staticmethod
    def forward(ctx, x, heads, drop, seed, win, bin_, wo, bo, l1w, l1b, w1, b1, w2, b2, l2w, l2b):
        e0 = _enc._mark()
        B, L, E = x.shape
        M, dev = B * L, x.device
        X = _rows(x.contiguous())
        f32 = torch.float32
        h1 = torch.empty(M, E, dtype=bf16, device=dev)
        m1, r1 = torch.empty(M, dtype=f32, device=dev), torch.empty(M, dtype=f32, device=dev)
        K.layernorm_fwd(X, l1w, l1b, h1, m1, r1, LN_EPS)
        Win, Wo, W1, W2 = (t.to(bf16) for t in (win, wo, w1, w2))
        # K-major copies for the data-gradient products dX = dY W and dZ = dT W2 (B = W^T
        # K-contiguous: the GEMM's faster B path, as the BERT layers' transposed copies,
        # DESIGN.md §2); only when a backward will run (not in no-grad inference passes)
        if any(ctx.needs_input_grad):
            Wint, Wot, W1t, W2t = (t.t().contiguous() for t in (Win, Wo, W1, W2))
        else:
            Wint = Wot = W1t = W2t = None
        qkv = torch.empty(M, 3 * E, dtype=bf16, device=dev)
        K.gemm(h1, E, True, Win, E, True, qkv, 3 * E, M, 3 * E, E, epi=K.epilogue(K.EPI_STORE, bias=bin_))
        O = torch.empty(M, E, dtype=bf16, device=dev)
        lse2 = torch.empty(L * heads, B, dtype=f32, device=dev)
        K.seqattn_fwd(qkv, O, lse2, B, L, heads)
        x1 = torch.empty(M, E, dtype=bf16, device=dev)
        K.gemm(O, E, True, Wo, E, True, x1, E, M, E, E, epi=K.epilogue(K.EPI_BIAS_DROP_RES, bias=bo, residual=X))
        h2 = torch.empty(M, E, dtype=bf16, device=dev)
        m2, r2 = torch.empty(M, dtype=f32, device=dev), torch.empty(M, dtype=f32, device=dev)
        K.layernorm_fwd(x1, l2w, l2b, h2, m2, r2, LN_EPS)
        Hh = torch.empty(M, 4 * E, dtype=bf16, device=dev)
        Zd = torch.empty(M, 4 * E, dtype=bf16, device=dev)  # dH/dz of dropout + QuickGELU
        K.gemm(h2, E, True, W1, E, True, Hh, 4 * E, M, 4 * E, E,
               epi=K.epilogue(K.EPI_BIAS_DROP_QGELU, bias=b1, aux=Zd, drop_p=drop, seed=seed))
        y = torch.empty(M, E, dtype=bf16, device=dev)
        K.gemm(Hh, 4 * E, True, W2, 4 * E, True, y, E, M, E, 4 * E,
               epi=K.epilogue(K.EPI_BIAS_DROP_RES, bias=b2, residual=x1))
        ctx.save_for_backward(X, h1, m1, r1, qkv, O, lse2, x1, h2, m2, r2, Hh, Zd, Wint, Wot, W1t, W2t, l1w, l2w)
        ctx.meta = (B, L, E, heads)
        if e0 is not None:
            _enc._block_events.append((e0, _enc._mark()))
        return y.view(B, L, E)

    @staticmethod
    def backward(ctx, dy):
        (X, h1, m1, r1, qkv, O, lse2, x1, h2, m2, r2, Hh, Zd, Wint, Wot, W1t, W2t, l1w, l2w) = ctx.saved_tensors
        B, L, E, heads = ctx.meta
        e0 = _enc._mark()
        M, dev, f32 = B * L, X.device, torch.float32
        dY = _rows(dy.contiguous()).to(bf16)
        st = K.epilogue(K.EPI_STORE)  # weight gradients: f32 C written (no zero fill + accumulate)
        g = {k: None for k in ("win", "bin", "wo", "bo", "l1w", "l1b", "w1", "b1", "w2", "b2", "l2w", "l2b")}
        # ---- c_proj (its input gradient is dy: no trailing dropout)
        dT = dY
        g["b2"] = torch.empty(E, dtype=f32, device=dev)
        K.colsum_bf16(dT, g["b2"])
        g["w2"] = torch.empty(E, 4 * E, dtype=f32, device=dev)
        K.gemm(dT, E, False, Hh, 4 * E, False, g["w2"], 4 * E, E, 4 * E, M, epi=st)
        dZ = torch.empty(M, 4 * E, dtype=bf16, device=dev)
        g["b1"] = torch.zeros(4 * E, dtype=f32, device=dev)
        K.gemm(dT, E, True, W2t, E, True, dZ, 4 * E, M, 4 * E, E,
               epi=K.epilogue(K.EPI_DGELU, aux=Zd, colsum=g["b1"]))
        g["w1"] = torch.empty(4 * E, E, dtype=f32, device=dev)
        K.gemm(dZ, 4 * E, False, h2, E, False, g["w1"], E, 4 * E, E, M, epi=st)
        dh2 = torch.empty(M, E, dtype=bf16, device=dev)
        K.gemm(dZ, 4 * E, True, W1t, 4 * E, True, dh2, E, M, E, 4 * E)
        # ---- ln_2 (+ the residual stream): dx1 = LN2'(dh2) + dy; its column sums = d out_proj.bias
        P = K.ln_parts(M)
        pw, pb, pbias = (torch.empty(P, E, dtype=f32, device=dev) for _ in range(3))
        dx1 = torch.empty(M, E, dtype=bf16, device=dev)
        K.layernorm_bwd_res(dh2, x1, m2, r2, l2w, dY, dx1, pw, pb, pbias)
        for k, part in (("l2w", pw), ("l2b", pb), ("bo", pbias)):
            g[k] = torch.empty(E, dtype=f32, device=dev)
            K.colsum_reduce(part, g[k])
        g["wo"] = torch.empty(E, E, dtype=f32, device=dev)
        K.gemm(dx1, E, False, O, E, False, g["wo"], E, E, E, M, epi=st)
        dO = torch.empty(M, E, dtype=bf16, device=dev)
        K.gemm(dx1, E, True, Wot, E, True, dO, E, M, E, E)
        # ---- attention over the sample axis + in_proj
        dqkv = torch.empty(M, 3 * E, dtype=bf16, device=dev)
        delta = torch.empty(L * heads, B, dtype=f32, device=dev)
        K.seqattn_bwd(qkv, O, dO, lse2, delta, dqkv, B, L, heads)
        g["bin"] = torch.empty(3 * E, dtype=f32, device=dev)
        K.colsum_bf16(dqkv, g["bin"])
        g["win"] = torch.empty(3 * E, E, dtype=f32, device=dev)
        K.gemm(dqkv, 3 * E, False, h1, E, False, g["win"], E, 3 * E, E, M, epi=st)
        dh1 = torch.empty(M, E, dtype=bf16, device=dev)
        K.gemm(dqkv, 3 * E, True, Wint, 3 * E, True, dh1, E, M, E, 3 * E)
        # ---- ln_1 (+ the residual stream)
        dx = torch.empty(M, E, dtype=bf16, device=dev)
        pw1, pb1 = (torch.empty(P, E, dtype=f32, device=dev) for _ in range(2))
        K.layernorm_bwd_res(dh1, X, m1, r1, l1w, dx1, dx, pw1, pb1, None)
        for k, part in (("l1w", pw1), ("l1b", pb1)):
            g[k] = torch.empty(E, dtype=f32, device=dev)
            K.colsum_reduce(part, g[k])
        if e0 is not None:
            _enc._block_events.append((e0, _enc._mark()))
        return (dx.view(B, L, E), None, None, None, g["win"], g["bin"], g["wo"], g["bo"], g["l1w"], g["l1b"],
                g["w1"], g["b1"], g["w2"], g["b2"], g["l2w"], g["l2b"])


# ------------------------------------------------------------------------------ modules
class ResidualAttentionBlock(nn.Module):
    """src/model.py:188-212 (parameters / keys identical; compute = BlockFunction)."""

    def __init__(self, d_model: int, n_head: int, attn_mask: torch.Tensor = None, drop: float = 0.0):
        super().__init__()
        self.attn = nn.MultiheadAttention(d_model, n_head)
        self.ln_1 = LayerNorm(d_model)
        self.mlp = nn.Sequential(OrderedDict([
            ("c_fc", nn.Linear(d_model, d_model * 4)),
            ("dropout", nn.Dropout(drop)),
            ("gelu", QuickGELU()),
            ("c_proj", nn.Linear(d_model * 4, d_model)),
            ("dropout", nn.Dropout(drop))
        ]))
        self.ln_2 = LayerNorm(d_model)
        self.attn_mask = attn_mask
        self.n_head = n_head
        self.drop = drop
        if attn_mask is not None:
            raise NotImplementedError("attn_mask: the reference fusion transformer passes None (src/model.py:214)")

    def forward(self, x: torch.Tensor):
        K._dev_check(x)
        p_drop = self.mlp.dropout.p if self.training else 0.0
        seed = _mlp_seed(self.training, p_drop)
        a, m = self.attn, self.mlp
        return BlockFunction.apply(x.to(bf16), self.n_head, p_drop, seed, a.in_proj_weight, a.in_proj_bias,
                                   a.out_proj.weight, a.out_proj.bias, self.ln_1.weight, self.ln_1.bias,
                                   m.c_fc.weight, m.c_fc.bias, m.c_proj.weight, m.c_proj.bias,
                                   self.ln_2.weight, self.ln_2.bias)


class Transformer(nn.Module):
    def __init__(self, width: int, layers: int, heads: int, attn_mask: torch.Tensor = None, drop: float = 0.0):
        super().__init__()
        self.width = width
        self.layers = layers
        self.resblocks = nn.Sequential(*[ResidualAttentionBlock(width, heads, attn_mask, drop) for _ in range(layers)])

    def forward(self, x: torch.Tensor):
        return self.resblocks(x)


class FlavaFusionTransfomer(nn.Module):
    """src/model.py:225-304: project, concatenate, ln_pre, 3 fusion blocks, ln_post, heads."""

    def __init__(self, out_dim: int = 1, num_classes: int = 2, image_hidden_size: int = 768,
                 text_hidden_size: int = 768, multimodal_hidden_size: int = 768,
                 multimodal_num_attention_heads: int = 3, multimodal_num_hidden_layers: int = 3,
                 drop: float = 0.0, **kwargs: Any):
        super().__init__()
        self.mm_encoder = Transformer(width=multimodal_hidden_size, layers=multimodal_num_hidden_layers,
                                      heads=multimodal_num_attention_heads, attn_mask=None, drop=drop)
        self.ln_pre = nn.LayerNorm(multimodal_hidden_size)
        self.ln_post = nn.LayerNorm(multimodal_hidden_size)
        self.image_to_mm_projection = nn.Linear(image_hidden_size, multimodal_hidden_size)
        self.text_to_mm_projection = nn.Linear(text_hidden_size, multimodal_hidden_size)
        self.output_layers = nn.ModuleList([nn.Linear(multimodal_hidden_size, num_classes) for i in range(out_dim)])
        self.loss = torch.nn.CrossEntropyLoss()
        self.avg_pool = kwargs["avg_pool"]
        self.n_cls_tokens = 0

    # the concatenated, projected sequence [B, n_cls + L_img + L_txt, E] (bf16)
    def _embed(self, image_features, text_features):
        if image_features is None or text_features is None:
            # the reference reads both shapes before its None checks (src/model.py:270)
            raise AttributeError("'NoneType' object has no attribute 'shape'")
        K._dev_check(image_features, text_features)
        B, Li, _ = image_features.shape
        Lt = text_features.shape[1]
        E = self.image_to_mm_projection.weight.shape[0]
        c = self.n_cls_tokens
        x = torch.empty(B, c + Li + Lt, E, dtype=bf16, device=image_features.device)
        if c:
            x = torch.cat([self.class_embeddings.t().to(bf16).unsqueeze(0).expand(B, -1, -1),
                           x[:, c:]], dim=1)
        pi, pt = self.image_to_mm_projection, self.text_to_mm_projection
        x = ProjFunction.apply(image_features, pi.weight, pi.bias, x, c)
        x = ProjFunction.apply(text_features, pt.weight, pt.bias, x, c + Li)
        return x, Li, Lt

    def _trunk(self, x):
        x = LNFunction.apply(x, self.ln_pre.weight, self.ln_pre.bias, self.ln_pre.eps)
        x = self.mm_encoder(x)
        return LNFunction.apply(x, self.ln_post.weight, self.ln_post.bias, self.ln_post.eps).float()

    def forward(self, x):
        image_features, text_features = x
        mm_x, l_img, l_txt = self._embed(image_features, text_features)
        out = self._trunk(mm_x)
        out_list = []
        if self.avg_pool:
            out_list.append(self.output_layers[0](out[:, :l_img, :].mean(1)))
            out_list.append(self.output_layers[1](out[:, l_img:(l_txt + l_img), :].mean(1)))
        else:
            for i, fc in enumerate(self.output_layers):
                out_list.append(fc(out[:, i, :]))
        return torch.stack(out_list, dim=1)  # (batch_size, ensemble_size, num_classes)

    def compute_loss(self, y_hat, y, eval=False):
        assert y.shape[0] == y_hat.shape[0]
        y = y.view(-1)
        if not eval:
            y_hat = y_hat.view(-1, y_hat.shape[2])  # loss per ensemble member
        else:
            y_hat = y_hat.mean(1)  # ensemble mean of the predictions
        return self.loss(y_hat, y)


class FlavaFusionTransfomerwithCLSToken(FlavaFusionTransfomer):
    """src/model.py:306-374: out_dim learned class tokens prepended; head i reads token i."""

    def __init__(self, out_dim: int = 1, num_classes: int = 2, image_hidden_size: int = 768,
                 text_hidden_size: int = 768, multimodal_hidden_size: int = 768,
                 multimodal_num_attention_heads: int = 3, multimodal_num_hidden_layers: int = 3,
                 drop: float = 0.1, **kwargs: Any):
        super().__init__(out_dim, num_classes, image_hidden_size, text_hidden_size, multimodal_hidden_size,
                         multimodal_num_attention_heads, multimodal_num_hidden_layers, drop, **kwargs)
        scale = multimodal_hidden_size ** -0.5
        self.class_embeddings = nn.Parameter(scale * torch.randn(multimodal_hidden_size, out_dim))
        self.out_dim = out_dim
        self.n_cls_tokens = out_dim

    def forward(self, x):
        image_features, text_features = x
        mm_x, _, _ = self._embed(image_features, text_features)
        out = self._trunk(mm_x)
        out_list = []
        for i, fc in enumerate(self.output_layers):
            out_list.append(fc(out[:, i, :]))
        return torch.stack(out_list, dim=1)


# ------------------------------------------------------------------ FashionMNIST MIMO family
# BASELINE config 1 (train_fashionmnist.py, CPU plumbing).  Same class names, constructor
# arguments, module trees and state_dict keys as the reference src/model.py:8-171.
model_configure = {  # model_type -> (emb_dim = views stacked as channels, out_dim = heads)
    "Vanilla": (4, 1),
    "MIMO-shuffle-instance": (4, 4),
    "MIMO-shuffle-view": (4, 4),
    "MultiHead": (4, 4),
    "MIMO-shuffle-all": (4, 4),
    "single-model-weight-sharing": (1, 1),
}


class ResNet(nn.Module):
    """src/model.py:17-56: 3x3 stem (stride 1, no max-pool), layer1 / layer2 of ``block``,
    AvgPool2d(4); convs N(0, sqrt(2 / (k*k*out))), BN gamma 1 beta 0."""

    def __init__(self, num_channels, block, layers):
        self.inplanes = 64
        super().__init__()
        self.conv1 = nn.Conv2d(num_channels, 64, kernel_size=3, stride=1, padding=1, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.avgpool = nn.AvgPool2d(4)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                fan = m.kernel_size[0] * m.kernel_size[1] * m.out_channels
                m.weight.data.normal_(0, (2.0 / fan) ** 0.5)
            elif isinstance(m, nn.BatchNorm2d):
                m.weight.data.fill_(1)
                m.bias.data.zero_()

    def _make_layer(self, block, planes, blocks, stride=1):
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = nn.Sequential(
                nn.Conv2d(self.inplanes, planes * block.expansion, kernel_size=1, stride=stride, bias=False),
                nn.BatchNorm2d(planes * block.expansion))
        mods = [block(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes * block.expansion
        mods += [block(self.inplanes, planes) for _ in range(1, blocks)]
        return nn.Sequential(*mods)


class MultiHeadFC(nn.Module):
    """src/model.py:58-70: one Linear with out_dim * num_classes outputs -> [B, out_dim, C]."""

    def __init__(self, input_dim, num_classes, out_dim):
        super().__init__()
        self.num_classes = num_classes
        self.fc = nn.Linear(input_dim, num_classes * out_dim)

    def forward(self, x):
        out = self.fc(x)
        return out.view(*out.shape[:-1], -1, self.num_classes)  # == stack(split(out, C, -1), 1)


def _mimo_loss(loss_fn, y_hat, y, eval):
    """src/model.py:102-112 / 161-171: per-head CE in training, CE of the head mean in eval."""
    assert y.shape[0] == y_hat.shape[0]
    y = y.view(-1)
    y_hat = y_hat.reshape(-1, y_hat.shape[2]) if not eval else y_hat.mean(1)
    return loss_fn(y_hat, y)


class MIMOResNet(ResNet):
    """src/model.py:72-112.  The views (or ensemble members) of x [B, E, C, H, W] are stacked
    as channels; a 4-D input is the weight-sharing model's [B*E, C, H, W]."""

    def __init__(self, num_channels, emb_dim, out_dim, num_classes):
        from .layers import BasicBlock
        super().__init__(num_channels * emb_dim, BasicBlock, [2, 2, 2])
        self.output_layer = MultiHeadFC(128 * BasicBlock.expansion, num_classes, out_dim)
        self.loss = torch.nn.CrossEntropyLoss()

    def forward(self, x):
        if x.dim() == 5:
            x = x.reshape(x.size(0), -1, x.size(3), x.size(4))
        x = self.relu(self.bn1(self.conv1(x)))
        x = self.layer2(self.layer1(x))
        x = self.avgpool(x).flatten(1)
        return self.output_layer(x)  # [B, out_dim, num_classes]

    def compute_loss(self, y_hat, y, eval=False):
        return _mimo_loss(self.loss, y_hat, y, eval)


class MIMOTransfomer(nn.Module):
    """src/model.py:114-171: each view's 14x14 pixels -> Linear(196, hidden) token, ln_pre,
    the fusion Transformer (HIP blocks of this module: attention over the SAMPLE axis, the
    reference's batch_first=False quirk), ln_post, per-head Linear on view i's token.
    GPU only (the blocks have no CPU path)."""

    def __init__(self, out_dim, num_classes, hidden_size, image_dim=14 * 14, multimodal_num_hidden_layers=3,
                 multimodal_num_attention_heads=3, drop=0):
        super().__init__()
        self.image_to_mm_projection = nn.Linear(image_dim, hidden_size)
        self.mm_encoder = Transformer(width=hidden_size, layers=multimodal_num_hidden_layers,
                                      heads=multimodal_num_attention_heads, drop=drop)
        self.output_layers = nn.ModuleList([nn.Linear(hidden_size, num_classes) for _ in range(out_dim)])
        self.loss = torch.nn.CrossEntropyLoss()
        self.ln_pre = nn.LayerNorm(hidden_size)
        self.ln_post = nn.LayerNorm(hidden_size)

    def forward(self, x):
        K._dev_check(x)
        b, e, c, h, w = x.shape
        # Linear(196 -> E) in f32 (K = 196 rows are not 16-B aligned in bf16; 0.3 MFLOP/token)
        t = torch.nn.functional.linear(x.reshape(b, e * c, h * w).float(), self.image_to_mm_projection.weight,
                                       self.image_to_mm_projection.bias)
        t = LNFunction.apply(t.to(bf16).contiguous(), self.ln_pre.weight, self.ln_pre.bias, self.ln_pre.eps)
        t = self.mm_encoder(t)
        t = LNFunction.apply(t, self.ln_post.weight, self.ln_post.bias, self.ln_post.eps).float()
        t = t.view(b, e, c, -1).mean(2)  # [B, E, hidden]
        return torch.stack([fc(t[:, i, :]) for i, fc in enumerate(self.output_layers)], dim=1)

    def compute_loss(self, y_hat, y, eval=False):
        return _mimo_loss(self.loss, y_hat, y, eval)
