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
