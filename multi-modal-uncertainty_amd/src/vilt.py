"""ViLT (``ViltForImagesAndTextClassification`` / ``ViltModel``) inference on the HIP kernels --
the ViLT patch-embed path of SURVEY §8f rank 4 (the reference's ``train.py:164-182``
``setup_vilt`` model, fed by ``src/dataset.py:228-285`` VILTDataset / collate_fn_vilt).

The weights are those of a ``transformers`` ViLT module (the reference loads
``dandelin/vilt-b32-mlm``, not available offline: the parity tests use a seeded random init of
the same classes).  Per ViLT pass (M = B * L token rows, L = text + 1 + patches):

  text embed    word[ids] + type[seg] + pos -> LayerNorm (mmu_layernorm_fwd_f32) + modality[0]
  patch embed   pixels [B, 3, H, W] -> im2col rows [B*gh*gw, 3*32*32] . W_patch^T + b   mmu_gemm
                (the 32 x 32 / 32 patch Conv2d as one GEMM), the reference's patch selection
                (valid patches of the pixel mask, random order / random padding patches drawn
                by torch.multinomial in the reference's order), interpolated position
                embeddings, [CLS] + pos[0], + modality[image index]
  12 x layer    pre-LN ViltLayer = the FLAVA encoder layer (src/flava_encoders._encoder_layers:
                LN, fused QKV GEMM, mmu_attention_fwd, Wo + residual (f32), LN, W1 + GELU, W2
                + residual)
  final LN      mmu_layernorm_fwd_f32; pooler tanh(dense(row 0)); classifier head (one row per
                sample: Linear, LayerNorm, GELU, Linear) in torch f32
The residual stream is f32, GEMM operands bf16 with f32 accumulation.  No CPU path: the
kernels raise on CPU tensors.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import kernels as K
from .flava_encoders import _Layer, _encoder_layers, _final_ln, patchify

bf16 = torch.bfloat16
MASK_NEG = -10000.0  # additive key mask (exp underflows to 0 exactly like the reference's dtype-min mask)


def _f32(t, dev):
    return t.detach().to(dev, torch.float32).contiguous()


def patch_mask(pixel_mask, gh, gw):
    """[B, H, W] pixel mask -> [B, gh, gw] long patch mask (nearest: pixel (i H / gh, j W / gw)),
    returned on the host (ViltEmbeddings.visual_embed's x_mask).  The sampling runs where the
    mask lives and only the patch grid crosses to the host (copying the full-resolution mask
    was 11 ms of a 22 ms batch-128 step, tools/vilt_profile.py)."""
    return F.interpolate(pixel_mask[:, None].float(), size=(gh, gw)).long()[:, 0].cpu()


def image_length(xm, max_image_length):
    """number of image tokens per sample: the largest valid extent, capped by max_image_length
    when that is a non-negative int (visual_embed's max_image_length rule)"""
    eff = int((xm.sum(1)[:, 0] * xm.sum(2)[:, 0]).max())
    if max_image_length is None or not isinstance(max_image_length, int) or max_image_length < 0:
        return eff
    return min(eff, max_image_length)


def select_patches(xm, max_len):
    """ViltEmbeddings.visual_embed's patch selection on the host, sample by sample in the
    reference's order with the same torch.multinomial draws from the global CPU generator: a
    sample with at least max_len valid patches keeps max_len of them in random order, one with
    fewer keeps all (in row-major order) and pads with valid-mask-0 patches drawn with
    replacement.  xm: [B, P] long patch mask.  Returns the flat indices b * P + p of the chosen
    patches ([B * max_len]) and their mask values [B, max_len]."""
    B, P = xm.shape
    n_valid = xm.sum(1)
    nv0 = int(n_valid[0])
    if 0 < max_len <= nv0 and bool((n_valid == nv0).all()):
        # every sample keeps max_len of its nv0 valid patches: the B per-sample draws in one
        # [B, nv0] multinomial call, which consumes the generator exactly as the B calls in
        # sample order do (tests/test_vilt.py checks the two against each other)
        v = xm.nonzero(as_tuple=False)[:, 1].view(B, nv0)
        pick = torch.gather(v, 1, torch.multinomial(torch.ones(B, nv0).float(), max_len))
        flat = (pick + torch.arange(B).unsqueeze(1) * P).flatten()
        return flat, xm.flatten()[flat].view(B, -1)
    v_all = torch.split(xm.nonzero(as_tuple=False)[:, 1], n_valid.tolist())
    nv_all = torch.split((1 - xm).nonzero(as_tuple=False)[:, 1], (P - n_valid).tolist())
    sel = []
    for b in range(B):
        v, nv = v_all[b], nv_all[b]
        if v.numel() == 0:  # (the reference iterates the samples that have a valid patch)
            continue
        pad = max_len - v.shape[0]
        if pad <= 0:
            pick = v[torch.multinomial(torch.ones(v.shape[0]).float(), max_len)]
        else:
            pick = torch.cat([v, nv[torch.multinomial(torch.ones(nv.shape[0]).float(), pad, replacement=True)]])
        sel.append(pick + b * P)
    flat = torch.cat(sel, 0)
    return flat, xm.flatten()[flat].view(B, -1)



def _check_head_dim(cfg, who):
    """The attention kernels read head h's Q / K / V at columns 64 h of the fused QKV rows
    (head_dim 64, as every BERT-base-shaped ViLT): another head width would pass the C-ABI's
    row-stride check and read the wrong columns, so it is refused here."""
    if cfg.hidden_size != cfg.num_attention_heads * 64:
        raise NotImplementedError(f"{who}: hidden_size {cfg.hidden_size} / {cfg.num_attention_heads} heads is not "
                                  "head_dim 64 (mmu_attention_fwd / _bwd)")

class ViltHIP:
    """``ViltForImagesAndTextClassification`` (or a bare ``ViltModel``) on the HIP kernels.

    ``__call__(input_ids, attention_mask, token_type_ids, pixel_values, pixel_mask)`` returns
    the classifier logits (the reference's ``outputs.logits``) for a classification model,
    ``(last_hidden_state, pooler_output)`` for a ViltModel; ``pixel_values`` is
    [B, num_images, 3, H, W] (or [B, 3, H, W] for one image), ``pixel_mask`` likewise without
    the channel axis."""

    def __init__(self, model, device="cuda"):
        dev = torch.device(device)
        vm = model.vilt if hasattr(model, "vilt") else model
        cfg = vm.config
        _check_head_dim(cfg, "ViltHIP")
        self.config = cfg
        emb = vm.embeddings
        te = emb.text_embeddings
        self.word = _f32(te.word_embeddings.weight, dev)
        self.pos_txt = _f32(te.position_embeddings.weight, dev)
        self.typ = _f32(te.token_type_embeddings.weight, dev)
        ln = te.LayerNorm
        self.txt_ln = (_f32(ln.weight, dev), _f32(ln.bias, dev), ln.eps)
        self.modality = _f32(emb.token_type_embeddings.weight, dev)
        proj = emb.patch_embeddings.projection
        self.patch = proj.kernel_size[0]
        w = proj.weight
        self.w_patch = w.reshape(w.shape[0], -1).to(dev, bf16).contiguous()
        self.b_patch = _f32(proj.bias, dev)
        self.cls = _f32(emb.cls_token, dev)                  # [1, 1, H]
        self.pos_img = _f32(emb.position_embeddings, dev)    # [1, 1 + P, H]
        self.layers = [_Layer(lyr, dev) for lyr in vm.encoder.layer]
        fl = vm.layernorm
        self.final_ln = (_f32(fl.weight, dev), _f32(fl.bias, dev), fl.eps)
        self.pool_w, self.pool_b = _f32(vm.pooler.dense.weight, dev), _f32(vm.pooler.dense.bias, dev)
        self.head = None
        if hasattr(model, "classifier"):
            c = model.classifier
            self.head = (_f32(c[0].weight, dev), _f32(c[0].bias, dev), _f32(c[1].weight, dev), _f32(c[1].bias, dev),
                         c[1].eps, _f32(c[3].weight, dev), _f32(c[3].bias, dev))
        self.device = dev

    # ------------------------------------------------------------------ embeddings
    def _text(self, input_ids, token_type_ids):
        B, Lt = input_ids.shape
        H = self.word.shape[1]
        if token_type_ids is None:
            token_type_ids = torch.zeros_like(input_ids)
        E = self.word[input_ids] + self.typ[token_type_ids] + self.pos_txt[:Lt].unsqueeze(0)
        X = torch.empty(B * Lt, H, dtype=torch.float32, device=input_ids.device)
        h = torch.empty(B * Lt, H, dtype=bf16, device=input_ids.device)
        K.layernorm_fwd_f32(E.reshape(B * Lt, H).contiguous(), self.txt_ln[0], self.txt_ln[1], h, X,
                            eps=self.txt_ln[2])
        return X.view(B, Lt, H) + self.modality[0]

    def _visual(self, pixel_values, pixel_mask, type_idx):
        """ViltEmbeddings.visual_embed (transformers modeling_vilt): patch GEMM, then the
        reference's patch selection and interpolated position embeddings (index bookkeeping on
        the host, the same torch.multinomial draws in the same order)."""
        B, C, Hh, Ww = pixel_values.shape
        p = self.patch
        gh, gw = Hh // p, Ww // p
        H = self.w_patch.shape[0]
        rows = patchify(pixel_values.float(), p).to(bf16).contiguous()
        x = torch.empty(B * gh * gw, H, dtype=torch.float32, device=rows.device)
        K.gemm(rows, rows.shape[1], True, self.w_patch, rows.shape[1], True, x, H, B * gh * gw, H, rows.shape[1],
               epi=K.epilogue(K.EPI_STORE, bias=self.b_patch))
        x = x.view(B, gh * gw, H)
        # pixel mask -> patch mask (nearest), valid extents per sample
        xm = patch_mask(pixel_mask, gh, gw)
        x_h = xm.sum(1)[:, 0]
        x_w = xm.sum(2)[:, 0]
        pd = self.config.image_size // self.config.patch_size
        spatial = self.pos_img[:, 1:, :].transpose(1, 2).reshape(1, H, pd, pd)
        # one interpolated position grid per distinct valid extent (a batch of full-size
        # images shares one), gathered per sample
        ext = [(int(h), int(w)) for h, w in zip(x_h, x_w)]
        uniq = sorted(set(ext))
        grids = torch.cat([F.pad(F.interpolate(spatial, size=e, mode="bilinear", align_corners=True),
                                 (0, gw - e[1], 0, gh - e[0])) for e in uniq], 0)
        grids = grids.flatten(2).transpose(1, 2)  # [U, gh*gw, H]
        max_len = image_length(xm, self.config.max_image_length)
        P = gh * gw
        flat, mask = select_patches(xm.flatten(1), max_len)
        mask = mask.to(x.device)
        flat = flat.to(x.device)
        x = x.reshape(B * P, H)[flat].view(B, -1, H)
        gid = torch.tensor([uniq.index(e) for e in ext], device=x.device)
        pos = grids.reshape(-1, H)[(gid * P).repeat_interleave(max_len) + flat % P].view(B, -1, H)
        x = torch.cat([self.cls.expand(B, -1, -1), x], 1)
        pos = torch.cat([self.pos_img[:, :1].expand(B, -1, -1), pos], 1)
        mask = torch.cat([torch.ones(B, 1, dtype=mask.dtype, device=x.device), mask], 1)
        return x + pos + self.modality[type_idx], mask

    # ------------------------------------------------------------------ forward
    @torch.no_grad()
    def vilt(self, input_ids, attention_mask, token_type_ids, pixel_values, pixel_mask, type_idx=1):
        """ViltModel.forward -> (last_hidden_state [B, L, H] f32, pooler_output [B, H])"""
        K._dev_check(input_ids)
        B, Lt = input_ids.shape
        if attention_mask is None:
            attention_mask = torch.ones_like(input_ids)
        if pixel_mask is None:
            pixel_mask = torch.ones(B, pixel_values.shape[-2], pixel_values.shape[-1], device=input_ids.device)
        txt = self._text(input_ids, token_type_ids)
        img, img_mask = self._visual(pixel_values, pixel_mask, type_idx)
        X = torch.cat([txt, img], 1)
        L, H = X.shape[1], X.shape[2]
        mask = torch.cat([attention_mask.to(img_mask.dtype), img_mask], 1)
        keymask = ((1.0 - mask.float()) * MASK_NEG).contiguous()
        X = _encoder_layers(X.reshape(B * L, H).contiguous(), keymask, self.layers, B, L)
        seq = _final_ln(X, self.final_ln, B, L)
        pooled = torch.tanh(F.linear(seq[:, 0], self.pool_w, self.pool_b))
        return seq, pooled

    @torch.no_grad()
    def __call__(self, input_ids, attention_mask=None, token_type_ids=None, pixel_values=None, pixel_mask=None):
        if pixel_values.dim() == 4:
            pixel_values = pixel_values[:, None]
            pixel_mask = None if pixel_mask is None else pixel_mask[:, None]
        n = pixel_values.shape[1]
        pooled = []
        last = None
        for i in range(n):
            last, p = self.vilt(input_ids, attention_mask, token_type_ids, pixel_values[:, i],
                                None if pixel_mask is None else pixel_mask[:, i], type_idx=i + 1)
            pooled.append(p)
        if self.head is None:
            return last, pooled[0]
        w0, b0, lw, lb, eps, w1, b1 = self.head
        h = F.linear(torch.cat(pooled, -1), w0, b0)
        h = F.gelu(F.layer_norm(h, (h.shape[-1],), lw, lb, eps))
        return F.linear(h, w1, b1)


# ---------------------------------------------------------------------------------- training
# The reference trains ViltForImagesAndTextClassification (train.py:164-182 setup_vilt: AdamW over
# model.parameters(); src/framework.py:262-300: outputs = model(**batch), outputs.loss.backward()).
# ViltTrainHIP runs that forward and backward on the HIP kernels with the transformers module as
# the parameter container (same nn.Parameters, state_dict keys and optimizer target):
#   text embed    torch (gathers + LayerNorm in f32: 0.1 ms of a step)
#   patch embed   mmu_gemm (32x32 / 32 patch Conv2d as one GEMM; weight grad mmu_gemm, bias grad
#                 mmu_colsum), the reference's patch selection / interpolated positions in torch
#   12 x layer    _ViltLayerFunction: the inference layer (f32 residual stream, bf16 GEMM
#                 operands) plus its backward -- DGELU-epilogue data grads, f32 weight grads,
#                 mmu_attention_bwd (+ fused Q/K/V bias grads), mmu_layernorm_bwd_f32; the stream
#                 gradient stays f32
#   final LN, pooler, classifier, loss   torch f32 on the [CLS] rows
class _PatchGemm(torch.autograd.Function):
    """x = rows W^T + b (f32 out): the patch Conv2d as one GEMM; grads for W and b only (the
    pixels are data)."""

    @staticmethod
    def forward(ctx, rows, w, b):
        M, Kp = rows.shape
        H = w.shape[0]
        x = torch.empty(M, H, dtype=torch.float32, device=rows.device)
        K.gemm(rows, Kp, True, w.reshape(H, -1).to(bf16).contiguous(), Kp, True, x, H, M, H, Kp,
               epi=K.epilogue(K.EPI_STORE, bias=b.float().contiguous()))
        ctx.save_for_backward(rows)
        ctx.wshape = w.shape
        return x

    @staticmethod
    def backward(ctx, dx):
        (rows,) = ctx.saved_tensors
        M, Kp = rows.shape
        dxb = dx.contiguous().to(bf16)
        H = dxb.shape[1]
        gw = torch.empty(H, Kp, dtype=torch.float32, device=rows.device)
        K.gemm(dxb, H, False, rows, Kp, False, gw, Kp, H, Kp, M, epi=K.epilogue(K.EPI_STORE))
        return None, gw.view(ctx.wshape), dx.sum(0)


class _ViltLayerFunction(torch.autograd.Function):
    """One pre-LN ViltLayer (transformers modeling_vilt ViltLayer: x + attn(LN_before(x)), then
    + FFN(LN_after(.))) on the f32 residual stream X [B*L, H]."""

    @staticmethod
    def forward(ctx, X, keymask, B, L, heads, eps1, eps2, wq, wk, wv, bq, bk, bv, wo, bo, l1w, l1b, w1, b1, w2, b2,
                l2w, l2b):
        M, H = X.shape
        Fd = w1.shape[0]
        dev, f32 = X.device, torch.float32
        Wqkv = torch.cat([wq, wk, wv]).to(bf16).contiguous()
        bqkv = torch.cat([bq, bk, bv]).float().contiguous()
        Wo, W1, W2 = (w.to(bf16).contiguous() for w in (wo, w1, w2))
        h1 = torch.empty(M, H, dtype=bf16, device=dev)
        m1, r1 = torch.empty(M, dtype=f32, device=dev), torch.empty(M, dtype=f32, device=dev)
        K.layernorm_fwd_f32(X, l1w, l1b, h1, None, m1, r1, eps=eps1)
        qkv = torch.empty(M, 3 * H, dtype=bf16, device=dev)
        K.gemm(h1, H, True, Wqkv, H, True, qkv, 3 * H, M, 3 * H, H, epi=K.epilogue(K.EPI_STORE, bias=bqkv))
        O = torch.empty(M, H, dtype=bf16, device=dev)
        lse = torch.empty(B * heads, L, dtype=f32, device=dev)
        K.attention_fwd(qkv, keymask, O, lse, B, L, heads, 0.0, 0, None)
        S = torch.empty(M, H, dtype=f32, device=dev)
        K.gemm(O, H, True, Wo, H, True, S, H, M, H, H, epi=K.epilogue(K.EPI_BIAS_DROP_RES, bias=bo, residual=X))
        h2 = torch.empty(M, H, dtype=bf16, device=dev)
        m2, r2 = torch.empty(M, dtype=f32, device=dev), torch.empty(M, dtype=f32, device=dev)
        K.layernorm_fwd_f32(S, l2w, l2b, h2, None, m2, r2, eps=eps2)
        G = torch.empty(M, Fd, dtype=bf16, device=dev)
        Z = torch.empty(M, Fd, dtype=bf16, device=dev)  # gelu'(.) for the backward's DGELU epilogue
        K.gemm(h2, H, True, W1, H, True, G, Fd, M, Fd, H, epi=K.epilogue(K.EPI_BIAS_GELU, bias=b1, aux=Z))
        Y = torch.empty(M, H, dtype=f32, device=dev)
        K.gemm(G, Fd, True, W2, Fd, True, Y, H, M, H, Fd, epi=K.epilogue(K.EPI_BIAS_DROP_RES, bias=b2, residual=S))
        ctx.save_for_backward(X, keymask, h1, m1, r1, qkv, O, lse, S, h2, m2, r2, G, Z, Wqkv, Wo, W1, W2, l1w, l2w)
        ctx.meta = (B, L, heads)
        return Y

    @staticmethod
    def backward(ctx, dY):
        (X, keymask, h1, m1, r1, qkv, O, lse, S, h2, m2, r2, G, Z, Wqkv, Wo, W1, W2, l1w, l2w) = ctx.saved_tensors
        B, L, heads = ctx.meta
        M, H = X.shape
        Fd = W1.shape[0]
        dev, f32 = X.device, torch.float32
        st = K.epilogue(K.EPI_STORE)
        dY = dY.contiguous().float()
        dYb = dY.to(bf16)
        # ---- FFN: Y = S + gelu(LN2(S) W1^T + b1) W2^T + b2
        g_w2 = torch.empty(H, Fd, dtype=f32, device=dev)
        K.gemm(dYb, H, False, G, Fd, False, g_w2, Fd, H, Fd, M, epi=st)
        dZ = torch.empty(M, Fd, dtype=bf16, device=dev)
        g_b1 = torch.zeros(Fd, dtype=f32, device=dev)
        K.gemm(dYb, H, True, W2.t().contiguous(), H, True, dZ, Fd, M, Fd, H,
               epi=K.epilogue(K.EPI_DGELU, aux=Z, colsum=g_b1))
        g_w1 = torch.empty(Fd, H, dtype=f32, device=dev)
        K.gemm(dZ, Fd, False, h2, H, False, g_w1, H, Fd, H, M, epi=st)
        dh2 = torch.empty(M, H, dtype=bf16, device=dev)
        K.gemm(dZ, Fd, True, W1.t().contiguous(), Fd, True, dh2, H, M, H, Fd)
        P = K.ln_parts(M)
        pw, pb = (torch.empty(P, H, dtype=f32, device=dev) for _ in range(2))
        dln = torch.empty(M, H, dtype=bf16, device=dev)
        K.layernorm_bwd(dh2, S, m2, r2, l2w, dln, None, 0.0, 0, pw, pb, None)
        g_l2w, g_l2b = torch.empty(H, dtype=f32, device=dev), torch.empty(H, dtype=f32, device=dev)
        K.colsum_reduce(pw, g_l2w)
        K.colsum_reduce(pb, g_l2b)
        dS = dY + dln  # the stream gradient stays f32 (bf16 + f32 promotes in the one add)
        dSb = dS.to(bf16)
        # ---- attention: S = X + attn(LN1(X)) Wo^T + bo
        g_wo = torch.empty(H, H, dtype=f32, device=dev)
        K.gemm(dSb, H, False, O, H, False, g_wo, H, H, H, M, epi=st)
        dO = torch.empty(M, H, dtype=bf16, device=dev)
        K.gemm(dSb, H, True, Wo.t().contiguous(), H, True, dO, H, M, H, H)
        dqkv = torch.empty(M, 3 * H, dtype=bf16, device=dev)
        delta = torch.empty(B * heads, L, dtype=f32, device=dev)
        parts = K.attention_dbias_parts(B, L, heads, dev)
        K.attention_bwd(qkv, keymask, O, dO, lse, delta, dqkv, B, L, heads, 0.0, 0, None, parts)
        g_bqkv = torch.zeros(3 * H, dtype=f32, device=dev)
        K.attention_dbias_reduce(parts, B, L, g_bqkv, heads)
        g_wqkv = torch.empty(3 * H, H, dtype=f32, device=dev)
        K.gemm(dqkv, 3 * H, False, h1, H, False, g_wqkv, H, 3 * H, H, M, epi=st)
        dh1 = torch.empty(M, H, dtype=bf16, device=dev)
        K.gemm(dqkv, 3 * H, True, Wqkv.t().contiguous(), 3 * H, True, dh1, H, M, H, 3 * H)
        pw1, pb1 = (torch.empty(P, H, dtype=f32, device=dev) for _ in range(2))
        K.layernorm_bwd(dh1, X, m1, r1, l1w, dln, None, 0.0, 0, pw1, pb1, None)
        g_l1w, g_l1b = torch.empty(H, dtype=f32, device=dev), torch.empty(H, dtype=f32, device=dev)
        K.colsum_reduce(pw1, g_l1w)
        K.colsum_reduce(pb1, g_l1b)
        dX = dS + dln
        gq, gk, gv = g_wqkv.split(H)
        gbq, gbk, gbv = g_bqkv.split(H)
        return (dX, None, None, None, None, None, None, gq, gk, gv, gbq, gbk, gbv, g_wo, dS.sum(0), g_l1w, g_l1b,
                g_w1, g_b1, g_w2, dY.sum(0), g_l2w, g_l2b)


class ViltTrainHIP(nn.Module):
    """``ViltForImagesAndTextClassification`` forward + backward on the HIP kernels for training
    (the reference's ``outputs = model(**batch); outputs.loss.backward()``).  ``model`` is the
    transformers module itself: its parameters are the ones trained (optimize ``model``'s
    parameters, save ``model.state_dict()``).  ``forward(**batch)`` returns the transformers
    output type (``loss``, ``logits``).  Dropout-free configurations only (ViltConfig's default
    hidden / attention-probs dropout is 0.0); the patch selection draws from the global CPU
    generator in the reference's order (select_patches)."""

    def __init__(self, model):
        super().__init__()
        cfg = model.config
        if cfg.hidden_dropout_prob or cfg.attention_probs_dropout_prob:
            raise NotImplementedError("ViltTrainHIP: hidden / attention-probs dropout > 0 is not built "
                                      "(ViltConfig's defaults are 0.0)")
        if cfg.hidden_act != "gelu":
            raise NotImplementedError(f"ViltTrainHIP: hidden_act {cfg.hidden_act!r} (the GEMM epilogue is erf GELU)")
        _check_head_dim(cfg, "ViltTrainHIP")
        self.model = model
        self.config = cfg

    def _text(self, emb, input_ids, token_type_ids):
        te = emb.text_embeddings
        Lt = input_ids.shape[1]
        if token_type_ids is None:
            token_type_ids = torch.zeros_like(input_ids)
        # F.embedding, not tensor indexing: the indexing backward serialises repeated indices
        # (every token's type row is row 0), 5 ms of a 36 ms batch-128 step
        E = F.embedding(input_ids, te.word_embeddings.weight) + F.embedding(token_type_ids, te.token_type_embeddings.weight) \
            + te.position_embeddings.weight[:Lt].unsqueeze(0)
        ln = te.LayerNorm
        X = F.layer_norm(E.float(), (E.shape[-1],), ln.weight, ln.bias, ln.eps)
        return X + emb.token_type_embeddings.weight[0]

    def _visual(self, emb, pixel_values, pixel_mask, type_idx):
        cfg = self.config
        B, C, Hh, Ww = pixel_values.shape
        proj = emb.patch_embeddings.projection
        p = proj.kernel_size[0]
        gh, gw = Hh // p, Ww // p
        H = proj.weight.shape[0]
        rows = patchify(pixel_values.float(), p).to(bf16).contiguous()
        x = _PatchGemm.apply(rows, proj.weight, proj.bias).view(B, gh * gw, H)
        xm = patch_mask(pixel_mask, gh, gw)
        x_h, x_w = xm.sum(1)[:, 0], xm.sum(2)[:, 0]
        pd = cfg.image_size // cfg.patch_size
        pos_img = emb.position_embeddings
        spatial = pos_img[:, 1:, :].transpose(1, 2).reshape(1, H, pd, pd)
        ext = [(int(h), int(w)) for h, w in zip(x_h, x_w)]
        uniq = sorted(set(ext))
        grids = torch.cat([F.pad(F.interpolate(spatial, size=e, mode="bilinear", align_corners=True),
                                 (0, gw - e[1], 0, gh - e[0])) for e in uniq], 0)
        grids = grids.flatten(2).transpose(1, 2)
        max_len = image_length(xm, cfg.max_image_length)
        P = gh * gw
        flat, mask = select_patches(xm.flatten(1), max_len)
        mask, flat = mask.to(x.device), flat.to(x.device)
        x = F.embedding(flat, x.reshape(B * P, H)).view(B, -1, H)
        gid = torch.tensor([uniq.index(e) for e in ext], device=x.device)
        pos = F.embedding((gid * P).repeat_interleave(max_len) + flat % P, grids.reshape(-1, H)).view(B, -1, H)
        x = torch.cat([emb.cls_token.expand(B, -1, -1), x], 1)
        pos = torch.cat([pos_img[:, :1].expand(B, -1, -1), pos], 1)
        mask = torch.cat([torch.ones(B, 1, dtype=mask.dtype, device=x.device), mask], 1)
        return x + pos + emb.token_type_embeddings.weight[type_idx], mask

    def _pooled(self, input_ids, attention_mask, token_type_ids, pixel_values, pixel_mask, type_idx):
        vm = self.model.vilt if hasattr(self.model, "vilt") else self.model
        emb = vm.embeddings
        B = input_ids.shape[0]
        if attention_mask is None:
            attention_mask = torch.ones_like(input_ids)
        if pixel_mask is None:
            pixel_mask = torch.ones(B, pixel_values.shape[-2], pixel_values.shape[-1], device=input_ids.device)
        txt = self._text(emb, input_ids, token_type_ids)
        img, img_mask = self._visual(emb, pixel_values, pixel_mask, type_idx)
        X = torch.cat([txt, img], 1)
        L, H = X.shape[1], X.shape[2]
        mask = torch.cat([attention_mask.to(img_mask.dtype), img_mask], 1)
        keymask = ((1.0 - mask.float()) * MASK_NEG).contiguous()
        X = X.reshape(B * L, H).contiguous()
        for lyr in vm.encoder.layer:
            a = lyr.attention.attention
            X = _ViltLayerFunction.apply(
                X, keymask, B, L, a.num_attention_heads, lyr.layernorm_before.eps, lyr.layernorm_after.eps,
                a.query.weight, a.key.weight, a.value.weight, a.query.bias, a.key.bias, a.value.bias,
                lyr.attention.output.dense.weight, lyr.attention.output.dense.bias,
                lyr.layernorm_before.weight, lyr.layernorm_before.bias,
                lyr.intermediate.dense.weight, lyr.intermediate.dense.bias,
                lyr.output.dense.weight, lyr.output.dense.bias,
                lyr.layernorm_after.weight, lyr.layernorm_after.bias)
        cls = X.view(B, L, H)[:, 0]  # only the [CLS] rows reach the pooler
        fl = vm.layernorm
        cls = F.layer_norm(cls, (H,), fl.weight, fl.bias, fl.eps)
        return torch.tanh(F.linear(cls, vm.pooler.dense.weight, vm.pooler.dense.bias))

    def forward(self, input_ids, attention_mask=None, token_type_ids=None, pixel_values=None, pixel_mask=None,
                labels=None, **unused):
        from transformers.models.vilt.modeling_vilt import ViltForImagesAndTextClassificationOutput
        K._dev_check(input_ids)
        if pixel_values.dim() == 4:
            pixel_values = pixel_values[:, None]
            pixel_mask = None if pixel_mask is None else pixel_mask[:, None]
        n = pixel_values.shape[1]
        if n != self.config.num_images:
            raise ValueError("Make sure to match the number of images in the model with the number of images in the input.")
        pooled = [self._pooled(input_ids, attention_mask, token_type_ids, pixel_values[:, i],
                               None if pixel_mask is None else pixel_mask[:, i], i + 1) for i in range(n)]
        logits = self.model.classifier(torch.cat(pooled, -1))
        loss = None
        if labels is not None:
            loss = F.cross_entropy(logits.view(-1, self.model.num_labels), labels.to(logits.device).view(-1))
        return ViltForImagesAndTextClassificationOutput(loss=loss, logits=logits)
