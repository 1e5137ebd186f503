"""FLAVA image / text encoders on the HIP kernels -- the inference path of the reference
data/encoding_with_flava.py:11-41: ``FlavaModel(**processor(...))``
whose ``image_embeddings`` [B, 197, 768] and ``text_embeddings`` [B, T, 768] are saved per
sample as the precomputed inputs of the FLAVA fusion transformer (src/model.py).

The weights are those of a ``transformers`` FlavaModel (FlavaImageModel / FlavaTextModel:
ViT-B/16 and a 12-layer text encoder, pre-LN FlavaLayers, erf GELU, final LayerNorm); the
reference loads ``facebook/flava-full``, which is not available offline, so the parity tests
use a seeded random init of the same classes.  Per encoder (M = B * L token rows):

  image embed   patches [B*196, 3*16*16] (im2col of the pixels) W_patch^T + b   mmu_gemm
                [CLS] + patches, + position embeddings -> f32 stream X
  text embed    word[ids] + type[seg] + pos -> LayerNorm -> f32 stream X (torch gather;
                the LN: mmu_layernorm_fwd_f32)
  12 x layer    h = LN_before(X)                                  mmu_layernorm_fwd_f32 -> bf16
                qkv = h Wqkv^T + bqkv                             mmu_gemm (Q | K | V fused)
                O = softmax(Q K^T / 8 + keymask) V                mmu_attention_fwd
                S = X + O Wo^T + bo                               mmu_gemm BIAS_DROP_RES, f32
                g = gelu(LN_after(S) W1^T + b1)                   mmu_layernorm_fwd_f32, mmu_gemm
                X = S + g W2^T + b2                               mmu_gemm BIAS_DROP_RES, f32
  final LN      -> f32 embeddings
The residual stream stays f32 (the pre-LN sums), GEMM operands bf16 with f32 accumulation.
There is no CPU path (the kernels raise on CPU tensors).
"""
import torch

from . import kernels as K

bf16 = torch.bfloat16
HEADS_DIM = 64


class _Layer:
    def __init__(self, layer, dev):
        a = layer.attention.attention
        self.wqkv = torch.cat([a.query.weight, a.key.weight, a.value.weight]).to(dev, bf16).contiguous()
        self.bqkv = torch.cat([a.query.bias, a.key.bias, a.value.bias]).to(dev, torch.float32).contiguous()
        o = layer.attention.output.dense
        self.wo, self.bo = o.weight.to(dev, bf16).contiguous(), o.bias.to(dev, torch.float32).contiguous()
        self.w1 = layer.intermediate.dense.weight.to(dev, bf16).contiguous()
        self.b1 = layer.intermediate.dense.bias.to(dev, torch.float32).contiguous()
        self.w2 = layer.output.dense.weight.to(dev, bf16).contiguous()
        self.b2 = layer.output.dense.bias.to(dev, torch.float32).contiguous()
        f = lambda t: t.to(dev, torch.float32).contiguous()  # noqa: E731
        self.ln1 = (f(layer.layernorm_before.weight), f(layer.layernorm_before.bias), layer.layernorm_before.eps)
        self.ln2 = (f(layer.layernorm_after.weight), f(layer.layernorm_after.bias), layer.layernorm_after.eps)
        self.heads = a.num_attention_heads
        self.hid = self.wo.shape[0]


def _encoder_layers(X, keymask, layers, B, L):
    """f32 stream X [B*L, H] through the pre-LN FlavaLayers; returns the final f32 stream."""
    M, H = X.shape
    dev = X.device
    h = torch.empty(M, H, dtype=bf16, device=dev)
    for lw in layers:
        K.layernorm_fwd_f32(X, lw.ln1[0], lw.ln1[1], h, eps=lw.ln1[2])
        qkv = torch.empty(M, 3 * H, dtype=bf16, device=dev)
        K.gemm(h, H, True, lw.wqkv, H, True, qkv, 3 * H, M, 3 * H, H, epi=K.epilogue(K.EPI_STORE, bias=lw.bqkv))
        O = torch.empty(M, H, dtype=bf16, device=dev)
        lse = torch.empty(B * lw.heads, L, dtype=torch.float32, device=dev)
        K.attention_fwd(qkv, keymask, O, lse, B, L, lw.heads, 0.0, 0, None)
        S = torch.empty(M, H, dtype=torch.float32, device=dev)
        K.gemm(O, H, True, lw.wo, H, True, S, H, M, H, H, epi=K.epilogue(K.EPI_BIAS_DROP_RES, bias=lw.bo, residual=X))
        K.layernorm_fwd_f32(S, lw.ln2[0], lw.ln2[1], h, eps=lw.ln2[2])
        F = lw.w1.shape[0]
        g = torch.empty(M, F, dtype=bf16, device=dev)
        K.gemm(h, H, True, lw.w1, H, True, g, F, M, F, H, epi=K.epilogue(K.EPI_BIAS_GELU, bias=lw.b1))
        Xn = torch.empty(M, H, dtype=torch.float32, device=dev)
        K.gemm(g, F, True, lw.w2, F, True, Xn, H, M, H, F, epi=K.epilogue(K.EPI_BIAS_DROP_RES, bias=lw.b2, residual=S))
        X = Xn
    return X


def _final_ln(X, ln, B, L):
    M, H = X.shape
    h = torch.empty(M, H, dtype=bf16, device=X.device)
    out = torch.empty(M, H, dtype=torch.float32, device=X.device)
    K.layernorm_fwd_f32(X, ln[0], ln[1], h, out, eps=ln[2])
    return out.view(B, L, H)


def patchify(pixel_values, patch):
    """[B, C, H, W] -> [B * (H/p) * (W/p), C * p * p] rows in Conv2d(kernel = stride = p) weight
    order (c, kh, kw): the patch-embedding convolution as one GEMM."""
    B, C, Hh, Ww = pixel_values.shape
    gh, gw = Hh // patch, Ww // patch
    x = pixel_values.reshape(B, C, gh, patch, gw, patch).permute(0, 2, 4, 1, 3, 5)
    return x.reshape(B * gh * gw, C * patch * patch)


class FlavaEncodersHIP:
    """Image and text encoders of a transformers FlavaModel (``model.image_model`` /
    ``model.text_model``) on the HIP kernels; ``__call__`` mirrors the two outputs the
    reference keeps: ``(image_embeddings, text_embeddings)``."""

    def __init__(self, flava_model, device="cuda"):
        dev = torch.device(device)
        im, tx = flava_model.image_model, flava_model.text_model
        pe = im.embeddings.patch_embeddings
        self.patch = pe.projection.kernel_size[0]
        w = pe.projection.weight
        self.w_patch = w.reshape(w.shape[0], -1).to(dev, bf16).contiguous()
        self.b_patch = pe.projection.bias.to(dev, torch.float32).contiguous()
        self.cls = im.embeddings.cls_token.detach().to(dev, torch.float32)
        self.pos_img = im.embeddings.position_embeddings.detach().to(dev, torch.float32)
        self.img_layers = [_Layer(lyr, dev) for lyr in im.encoder.layer]
        f = lambda ln: (ln.weight.to(dev, torch.float32).contiguous(), ln.bias.to(dev, torch.float32).contiguous(),  # noqa: E731
                        ln.eps)
        self.img_ln = f(im.layernorm)
        te = tx.embeddings
        self.word = te.word_embeddings.weight.detach().to(dev, torch.float32)
        self.typ = te.token_type_embeddings.weight.detach().to(dev, torch.float32)
        self.pos_txt = te.position_embeddings.weight.detach().to(dev, torch.float32)
        self.txt_emb_ln = f(te.LayerNorm)
        self.txt_layers = [_Layer(lyr, dev) for lyr in tx.encoder.layer]
        self.txt_ln = f(tx.layernorm)
        self.device = dev

    @torch.no_grad()
    def encode_image(self, pixel_values):
        K._dev_check(pixel_values)
        B = pixel_values.shape[0]
        rows = patchify(pixel_values.float(), self.patch).to(bf16).contiguous()
        P, H = rows.shape[0] // B, self.w_patch.shape[0]
        emb = torch.empty(B * P, H, dtype=torch.float32, device=rows.device)
        K.gemm(rows, rows.shape[1], True, self.w_patch, rows.shape[1], True, emb, H, B * P, H, rows.shape[1],
               epi=K.epilogue(K.EPI_STORE, bias=self.b_patch))
        X = torch.cat([self.cls.expand(B, 1, H), emb.view(B, P, H)], 1) + self.pos_img
        L = P + 1
        keymask = torch.zeros(B, L, dtype=torch.float32, device=rows.device)
        X = _encoder_layers(X.reshape(B * L, H).contiguous(), keymask, self.img_layers, B, L)
        return _final_ln(X, self.img_ln, B, L)

    @torch.no_grad()
    def encode_text(self, input_ids, attention_mask=None, token_type_ids=None):
        K._dev_check(input_ids)
        B, L = input_ids.shape
        H = self.word.shape[1]
        if token_type_ids is None:
            token_type_ids = torch.zeros_like(input_ids)
        if attention_mask is None:
            attention_mask = torch.ones_like(input_ids)
        E = self.word[input_ids] + self.typ[token_type_ids] + self.pos_txt[:L].unsqueeze(0)
        X = torch.empty(B * L, H, dtype=torch.float32, device=input_ids.device)
        h = torch.empty(B * L, H, dtype=bf16, device=input_ids.device)
        ln = self.txt_emb_ln
        K.layernorm_fwd_f32(E.reshape(B * L, H).contiguous(), ln[0], ln[1], h, X, eps=ln[2])
        # additive key mask, the reference's (1 - mask) * large-negative (BERT's -10000: exp underflows alike)
        keymask = ((1.0 - attention_mask.float()) * -10000.0).contiguous()
        X = _encoder_layers(X, keymask, self.txt_layers, B, L)
        return _final_ln(X, self.txt_ln, B, L)

    def __call__(self, pixel_values=None, input_ids=None, attention_mask=None, token_type_ids=None):
        img = self.encode_image(pixel_values) if pixel_values is not None else None
        txt = self.encode_text(input_ids, attention_mask, token_type_ids) if input_ids is not None else None
        return img, txt
