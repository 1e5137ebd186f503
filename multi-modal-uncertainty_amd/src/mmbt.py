"""MMBT (BERT-base + ResNet-152) on the MI355X HIP kernels -- drop-in for the
reference ``src/mmbt.py`` (classes, methods, argument order, state_dict keys).

Reference API kept (src/mmbt.py:15-262):
  ImageEncoder(args)                 .forward(img) -> [B, N, 2048]
  ImageBertEmbeddings(args, emb)     .forward(feats, token_type_ids) -> [B, N+2, 768]
  MultimodalBertEncoder(args)        .forward / forward_img_only / forward_txt_only / forward_control
  MultimodalBertClf(args)            same + .compute_loss(y_hat, y, eval=False)
  sub-modules enc.txt_embeddings, enc.img_embeddings, enc.img_encoder, enc.encoder, enc.pooler, clf

What runs where on the GPU:
  ResNet-152 trunk      MIOpen (PyTorch-ROCm), bf16 autocast, channels-last
  row pooling           mmu_row_pool_fwd/bwd           (AdaptiveAvgPool2d((N,1)) + transpose)
  image projection      torch f32 linear (2048->768, 3 rows per sample)
  token embed + concat  mmu_embed_fwd/bwd             (one pass; variants = index gather)
  12 BERT layers        src/encoder.py                 (MFMA GEMMs + flash attention + LN)
  pooler + classifier   torch f32 (768x768, 768x101 on one row per sample)
No CPU fallback: the encoder path raises on CPU tensors.
"""
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import kernels as K
from .encoder import LayerWeights, encoder_stack
from .params import ParamStore
from .resnet import StoreConv2d, resnet152_trunk

# the encoder hands the pooler only the last layer's [CLS] rows (MMU_CLS_ONLY=0: all rows, round 5)
CLS_ONLY = os.environ.get("MMU_CLS_ONLY", "1") != "0"

BERT_CONFIGS = {
    # name: (layers, hidden, heads, intermediate, vocab, max_pos, type_vocab)
    "bert-base-uncased": (12, 768, 12, 3072, 30522, 512, 2),
}
HIDDEN_DROPOUT = 0.1     # bert-base-uncased hidden_dropout_prob
ATTN_DROPOUT = 0.1       # bert-base-uncased attention_probs_dropout_prob
LN_EPS = 1e-12


def _bert_shape(args):
    name = getattr(args, "bert_model", "bert-base-uncased")
    if name not in BERT_CONFIGS:
        raise NotImplementedError(f"{name}: the HIP path is built for bert-base (768 hidden, 12 x 64 heads)")
    layers, hid, heads, inter, vocab, max_pos, tv = BERT_CONFIGS[name]
    layers = getattr(args, "bert_layers", layers)
    vocab = getattr(args, "vocab_size", vocab)
    if getattr(args, "hidden_sz", hid) != hid:
        raise NotImplementedError("hidden_sz must be 768 for bert-base")
    return layers, hid, heads, inter, vocab, max_pos, tv


def _seed():
    return int(torch.randint(0, 2 ** 62, (1,)).item())


def _mix(seed, k):
    return (seed ^ (0x9E3779B97F4A7C15 * (k + 1))) & 0xFFFFFFFFFFFFFFFF


# ----------------------------------------------------------------------------- BERT modules
class BertLayerNorm(nn.Module):
    def __init__(self, hid, eps=LN_EPS):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(hid))
        self.bias = nn.Parameter(torch.zeros(hid))
        self.eps = eps


class BertEmbeddings(nn.Module):
    """word + position + token-type embeddings, LayerNorm, dropout (pytorch_pretrained_bert 0.6.x names)."""

    def __init__(self, vocab, hid, max_pos, type_vocab):
        super().__init__()
        self.word_embeddings = nn.Embedding(vocab, hid)
        self.position_embeddings = nn.Embedding(max_pos, hid)
        self.token_type_embeddings = nn.Embedding(type_vocab, hid)
        self.LayerNorm = BertLayerNorm(hid)
        self.dropout = nn.Dropout(HIDDEN_DROPOUT)
        self._owner = None

    def forward(self, input_ids, token_type_ids=None):
        """Text-only embedding [B, T, 768] (inference helper; training uses the fused model path)."""
        return self._owner._text_embeddings(input_ids, token_type_ids)


class _Linear(nn.Linear):
    pass


class BertSelfAttention(nn.Module):
    def __init__(self, hid):
        super().__init__()
        self.query, self.key, self.value = nn.Linear(hid, hid), nn.Linear(hid, hid), nn.Linear(hid, hid)
        self.dropout = nn.Dropout(ATTN_DROPOUT)


class BertSelfOutput(nn.Module):
    def __init__(self, hid):
        super().__init__()
        self.dense = nn.Linear(hid, hid)
        self.LayerNorm = BertLayerNorm(hid)
        self.dropout = nn.Dropout(HIDDEN_DROPOUT)


class BertAttention(nn.Module):
    def __init__(self, hid):
        super().__init__()
        self.self = BertSelfAttention(hid)
        self.output = BertSelfOutput(hid)


class BertIntermediate(nn.Module):
    def __init__(self, hid, inter):
        super().__init__()
        self.dense = nn.Linear(hid, inter)


class BertOutput(nn.Module):
    def __init__(self, hid, inter):
        super().__init__()
        self.dense = nn.Linear(inter, hid)
        self.LayerNorm = BertLayerNorm(hid)
        self.dropout = nn.Dropout(HIDDEN_DROPOUT)


class BertLayer(nn.Module):
    def __init__(self, hid, inter):
        super().__init__()
        self.attention = BertAttention(hid)
        self.intermediate = BertIntermediate(hid, inter)
        self.output = BertOutput(hid, inter)


class BertEncoder(nn.Module):
    def __init__(self, n_layers, hid, inter):
        super().__init__()
        self.layer = nn.ModuleList([BertLayer(hid, inter) for _ in range(n_layers)])
        self._owner = None

    def forward(self, hidden_states, attention_mask, output_all_encoded_layers=True):
        """0.6.x call contract: hidden [B,L,768], additive mask [B,1,1,L] -> list of [B,L,768]."""
        return self._owner._run_encoder_api(hidden_states, attention_mask, output_all_encoded_layers)


class BertPooler(nn.Module):
    def __init__(self, hid):
        super().__init__()
        self.dense = nn.Linear(hid, hid)
        self.activation = nn.Tanh()

    def forward(self, hidden_states):
        return self.activation(self.dense(hidden_states[:, 0].float()))


def init_bert_weights(module, std=0.02):
    for m in module.modules():
        if isinstance(m, (nn.Linear, nn.Embedding)):
            m.weight.data.normal_(0.0, std)
        if isinstance(m, nn.Linear) and m.bias is not None:
            m.bias.data.zero_()
        if isinstance(m, BertLayerNorm):
            m.weight.data.fill_(1.0)
            m.bias.data.zero_()


# ----------------------------------------------------------------------------- autograd glue
class RowPoolFunction(torch.autograd.Function):
    """AdaptiveAvgPool2d((n,1)) + flatten + transpose of the NHWC bf16 ResNet map -> f32 [B,n,C]."""

    @staticmethod
    def forward(ctx, fmap, n):
        nhwc = fmap.permute(0, 2, 3, 1)
        if not nhwc.is_contiguous():
            nhwc = nhwc.contiguous()
        B, Hh, Ww, C = nhwc.shape
        out = torch.empty(B, n, C, dtype=torch.float32, device=fmap.device)
        K.row_pool_fwd(nhwc, n, out)
        ctx.shape, ctx.n, ctx.dtype = (B, Hh, Ww, C), n, fmap.dtype
        return out

    @staticmethod
    def backward(ctx, dout):
        B, Hh, Ww, C = ctx.shape
        d = torch.empty(B, Hh, Ww, C, dtype=torch.bfloat16, device=dout.device)
        K.row_pool_bwd(dout.contiguous().float(), ctx.n, d)
        g = d.permute(0, 3, 1, 2)
        return (g if ctx.dtype == torch.bfloat16 else g.to(ctx.dtype)), None


class EmbedFunction(torch.autograd.Function):
    """[CLS] | Linear(img) | [SEP] | text -> LayerNorm'ed encoder input + key mask (identity variant)."""

    @staticmethod
    def forward(ctx, proj, word_anchor, enc, ids, seg, txt_mask, drop_txt, drop_img, seed):
        B, T = ids.shape
        n = proj.shape[1]
        L = n + 2 + T
        dev = proj.device
        X = torch.empty(B * L, 768, dtype=torch.bfloat16, device=dev)
        X32 = torch.empty(B * L, 768, dtype=torch.float32, device=dev)
        km = torch.empty(B, L, dtype=torch.float32, device=dev)
        mean = torch.empty(B * L, dtype=torch.float32, device=dev)
        rstd = torch.empty(B * L, dtype=torch.float32, device=dev)
        e = enc.txt_embeddings
        K.embed_fwd(ids, seg, txt_mask, proj, e.word_embeddings.weight, e.position_embeddings.weight,
                    e.token_type_embeddings.weight, e.LayerNorm.weight, e.LayerNorm.bias, LN_EPS, enc.cls_id,
                    enc.sep_id, None, 1, B, T, n, L, X, km, mean, rstd, drop_txt, drop_img, seed, X32=X32)
        ctx.save_for_backward(proj, ids, seg, mean, rstd)
        ctx.meta = (enc, B, T, n, drop_txt, drop_img, seed)
        # the gradient of the encoder input arrives on the bf16 X (BertLayerFunction returns
        # the whole input gradient there); X32 is the same values in f32
        ctx.mark_non_differentiable(X32, km)
        return X, X32, km

    @staticmethod
    def backward(ctx, dX, _dX32, _dkm):
        proj, ids, seg, mean, rstd = ctx.saved_tensors
        enc, B, T, n, drop_txt, drop_img, seed = ctx.meta
        e = enc.txt_embeddings
        st = enc._store
        d_proj = torch.empty_like(proj)
        pre = "enc.txt_embeddings." if enc._prefix == "enc." else "txt_embeddings."
        K.embed_bwd(dX.contiguous(), ids, seg, proj, e.word_embeddings.weight, e.position_embeddings.weight,
                    e.token_type_embeddings.weight, e.LayerNorm.weight, mean, rstd, enc.cls_id, enc.sep_id, B, T, n,
                    st.grad_of(pre + "word_embeddings.weight"), st.grad_of(pre + "position_embeddings.weight"),
                    st.grad_of(pre + "token_type_embeddings.weight"), st.grad_of(pre + "LayerNorm.weight"),
                    st.grad_of(pre + "LayerNorm.bias"), d_proj, drop_txt, drop_img, seed)
        if enc._grad_ready_hook is not None:
            enc._grad_ready_hook("embeddings")
        return d_proj, None, None, None, None, None, None, None, None


class ProjectFunction(torch.autograd.Function):
    """img_embeddings Linear(2048 -> 768) on the pooled features (reference src/mmbt.py:61,70).
    Its backward accumulates dW / db straight into the flat gradient store and only then
    reports the "proj" gradient segment done (src/dp.py), so the segment's all-reduce is
    ordered after the accumulation on the compute stream (an AccumulateGrad node of
    autograd's own would run at an unspecified point after the embedding hook)."""

    @staticmethod
    def forward(ctx, feats, weight, bias, enc):
        ctx.save_for_backward(feats, weight)
        ctx.enc = enc
        return F.linear(feats, weight, bias)

    @staticmethod
    def backward(ctx, d):
        feats, weight = ctx.saved_tensors
        enc = ctx.enc
        d2 = d.reshape(-1, d.shape[-1]).float()
        dfeats = (d2 @ weight).view(feats.shape) if ctx.needs_input_grad[0] else None
        st, pre = enc._store, enc._prefix + "img_embeddings.img_embeddings."
        if ctx.needs_input_grad[1]:
            st.grad_of(pre + "weight").addmm_(d2.t(), feats.reshape(-1, feats.shape[-1]))
        if ctx.needs_input_grad[2]:
            st.grad_of(pre + "bias").add_(d2.sum(0))
        if enc._grad_ready_hook is not None:
            enc._grad_ready_hook("proj")
        return dfeats, None, None, None


# ----------------------------------------------------------------------------- image side
class ImageEncoder(nn.Module):
    def __init__(self, args):
        super().__init__()
        self.args = args
        self.model = resnet152_trunk(tuple(getattr(args, "resnet_blocks", (3, 8, 36, 3))))
        n = args.num_image_embeds
        pool = nn.AdaptiveAvgPool2d if args.img_embed_pool_type == "avg" else nn.AdaptiveMaxPool2d
        grid = {4: (2, 2), 6: (3, 2), 8: (4, 2), 9: (3, 3)}.get(n, (n, 1))
        self.pool = pool(grid)
        # the HIP row-pool covers the default (avg, N x 1 bins); other configs use torch pooling
        self._hip_pool = args.img_embed_pool_type == "avg" and grid[1] == 1
        # "bf16": the product / bench trunk (HIP stem, BatchNorm, implicit convs, 1x1 GEMMs, pools;
        # MIOpen for the rest); "fp32": exact-precision torch trunk for parity runs;
        # "torch_bf16": TEST COMPARATOR only -- the same bf16 arithmetic on PyTorch's own ops
        # (MIOpen bf16 convs under autocast, torch batch_norm / pools), which measures the noise
        # floor any bf16 trunk has against the fp32 reference (tests/test_mmbt_gpu.py)
        self.precision = getattr(args, "img_precision", "bf16")
        assert self.precision in ("bf16", "fp32", "torch_bf16"), self.precision

    def trunk(self, x):
        from . import resnet as R
        train_params = any(p.requires_grad for p in self.model.parameters())
        grad = torch.is_grad_enabled() and (train_params or x.requires_grad)
        bf16 = self.precision in ("bf16", "torch_bf16")
        # bf16 trunk: the image is cast once here (what autocast would do inside the stem conv),
        # so the stem runs on mmu_stem_conv_* with the store's bf16 filter copy
        x = x.to(torch.bfloat16 if bf16 else x.dtype, memory_format=torch.channels_last)
        with torch.set_grad_enabled(grad), torch.autocast("cuda", dtype=torch.bfloat16, enabled=bf16), \
                R.torch_ops_only(self.precision == "torch_bf16"):
            return self.model(x)

    def forward(self, x):
        if not x.is_cuda:
            raise K.N.NativeError("ImageEncoder: the MI355X path needs the image batch on a HIP device")
        f = self.trunk(x)
        if self._hip_pool and f.dtype == torch.bfloat16 and self.precision == "bf16":
            return RowPoolFunction.apply(f, self.args.num_image_embeds)
        return torch.flatten(self.pool(f.float()), start_dim=2).transpose(1, 2).contiguous()


class ImageBertEmbeddings(nn.Module):
    def __init__(self, args, embeddings):
        super().__init__()
        self.args = args
        self.img_embeddings = nn.Linear(args.img_hidden_sz, args.hidden_sz)
        self.position_embeddings = embeddings.position_embeddings
        self.token_type_embeddings = embeddings.token_type_embeddings
        self.word_embeddings = embeddings.word_embeddings
        self.LayerNorm = embeddings.LayerNorm
        self.dropout = nn.Dropout(p=args.dropout)
        self._owner = None

    def project(self, feats):
        w, b = self.img_embeddings.weight, self.img_embeddings.bias
        if torch.is_grad_enabled() and self._owner is not None and self._owner._store is not None and (
                feats.requires_grad or w.requires_grad or b.requires_grad):
            return ProjectFunction.apply(feats.float(), w, b, self._owner)
        return F.linear(feats.float(), w, b)

    def forward(self, input_imgs, token_type_ids=None):
        """[B,N,2048] -> [B,N+2,768] (reference forward, src/mmbt.py:58-83)."""
        return self._owner._image_embeddings(self.project(input_imgs))


# ----------------------------------------------------------------------------- encoder
class MultimodalBertEncoder(nn.Module):
    def __init__(self, args):
        super().__init__()
        self.args = args
        layers, hid, heads, inter, vocab, max_pos, tv = _bert_shape(args)
        self.txt_embeddings = BertEmbeddings(vocab, hid, max_pos, tv)
        self.img_embeddings = ImageBertEmbeddings(args, self.txt_embeddings)
        self.img_encoder = ImageEncoder(args)
        self.encoder = BertEncoder(layers, hid, inter)
        self.pooler = BertPooler(hid)
        init_bert_weights(self.txt_embeddings)
        init_bert_weights(self.encoder)
        init_bert_weights(self.pooler)
        init_bert_weights(self.img_embeddings.img_embeddings)
        self.cls_id = int(args.vocab.stoi["[CLS]"])
        self.sep_id = int(args.vocab.stoi["[SEP]"])
        self.n_img = int(args.num_image_embeds)
        self.hidden_dropout = float(getattr(args, "bert_hidden_dropout", HIDDEN_DROPOUT))
        self.attn_dropout = float(getattr(args, "bert_attn_dropout", ATTN_DROPOUT))
        self.mc_dropout = False  # keep BERT dropout sites active in eval (MC-dropout passes)
        self._grad_ready_hook = None
        self._store = None
        self._prefix = ""
        self._lw = []
        for m in (self.txt_embeddings, self.img_embeddings, self.encoder):
            object.__setattr__(m, "_owner", self)  # back-reference, not a registered sub-module

    # ---------------------------------------------------------------- storage
    def _flat_entries(self, prefix):
        named = dict(self.named_parameters(prefix=prefix.rstrip(".")) if prefix else self.named_parameters())
        order = []
        for i in reversed(range(len(self.encoder.layer))):
            p = f"{prefix}encoder.layer.{i}."
            for s in ("query", "key", "value"):
                order.append(f"{p}attention.self.{s}.weight")
            for s in ("query", "key", "value"):
                order.append(f"{p}attention.self.{s}.bias")
            order += [f"{p}attention.output.dense.weight", f"{p}attention.output.dense.bias",
                      f"{p}attention.output.LayerNorm.weight", f"{p}attention.output.LayerNorm.bias",
                      f"{p}intermediate.dense.weight", f"{p}intermediate.dense.bias",
                      f"{p}output.dense.weight", f"{p}output.dense.bias",
                      f"{p}output.LayerNorm.weight", f"{p}output.LayerNorm.bias"]
        head = [f"{prefix}pooler.dense.weight", f"{prefix}pooler.dense.bias"]
        emb = [f"{prefix}txt_embeddings.{n}" for n in ("word_embeddings.weight", "position_embeddings.weight",
                                                         "token_type_embeddings.weight", "LayerNorm.weight",
                                                         "LayerNorm.bias")]
        emb += [f"{prefix}img_embeddings.img_embeddings.weight", f"{prefix}img_embeddings.img_embeddings.bias"]
        res = [n for n in named if n.startswith(f"{prefix}img_encoder.")][::-1]
        order = head + order + emb + res
        assert len(order) == len(named) and set(order) == set(named), "flat layout misses parameters"
        compute = []
        for i in range(len(self.encoder.layer)):
            p = f"{prefix}encoder.layer.{i}."
            compute += [f"{p}attention.self.{s}.weight" for s in ("query", "key", "value")]
            compute += [f"{p}attention.output.dense.weight", f"{p}intermediate.dense.weight", f"{p}output.dense.weight"]
        # bf16 conv filters for the trunk (read by StoreConv2d instead of an autocast cast per step)
        compute += [n for n in res if named[n].dim() == 4]
        return [(n, named[n]) for n in order], compute

    def _attach_store(self, store, prefix):
        self._store, self._prefix = store, prefix
        self._lw = [LayerWeights(store, f"{prefix}encoder.layer.{i}.", lyr) for i, lyr in enumerate(self.encoder.layer)]
        for name, m in self.img_encoder.named_modules(prefix=f"{prefix}img_encoder"):
            if isinstance(m, StoreConv2d) and f"{name}.weight" in store.coffsets:
                m.attach_compute(store, f"{name}.weight")

    def _refresh_views(self):
        for lw in self._lw:
            lw.refresh()

    def _prepare(self):
        if self._store is None:
            entries, compute = self._flat_entries("")
            self._attach_store(ParamStore(entries, compute), "")
        st = self._store
        if not st.check_views():
            st.build()
            self._refresh_views()
        st.maybe_sync_compute()
        if torch.is_grad_enabled():
            st.ensure_grads(quick=True)

    def _apply(self, fn, *a, **k):
        out = super()._apply(fn, *a, **k)
        if self._store is not None and self._prefix == "":
            self._store.build()
            self._refresh_views()
        return out

    # ---------------------------------------------------------------- pieces
    def _dropout_active(self):
        return self.training or self.mc_dropout

    def _image_feats(self, img):
        return self.img_encoder(img)

    def _embed(self, txt, txt_mask, segment, proj, idx=None, Lout=None, V=1):
        B, T = txt.shape
        dev = proj.device
        drop_txt = self.hidden_dropout if self.training else 0.0
        drop_img = float(self.args.dropout) if self.training else 0.0
        seed = _seed() if (drop_txt > 0 or drop_img > 0) else 0
        txt, segment, txt_mask = (t.contiguous().long() for t in (txt, segment, txt_mask))
        if idx is None and torch.is_grad_enabled():
            X, X32, km = EmbedFunction.apply(proj, self.txt_embeddings.word_embeddings.weight, self, txt, segment,
                                             txt_mask, drop_txt, drop_img, seed)
            return (X, X32), km, self.n_img + 2 + T
        L = self.n_img + 2 + T if idx is None else Lout
        X = torch.empty(V * B * L, 768, dtype=torch.bfloat16, device=dev)
        X32 = torch.empty(V * B * L, 768, dtype=torch.float32, device=dev)
        km = torch.empty(V * B, L, dtype=torch.float32, device=dev)
        e = self.txt_embeddings
        K.embed_fwd(txt, segment, txt_mask, proj.contiguous(), e.word_embeddings.weight, e.position_embeddings.weight,
                    e.token_type_embeddings.weight, e.LayerNorm.weight, e.LayerNorm.bias, LN_EPS, self.cls_id,
                    self.sep_id, idx, V, B, T, self.n_img, L, X, km, drop_txt=drop_txt, drop_img=drop_img, seed=seed,
                    X32=X32)
        return (X, X32), km, L

    def _encode(self, XX, km, nb, L):
        """(X bf16, X32 f32) [nb*L, 768], km [nb, L] -> the last layer's [CLS] rows [nb, 768] f32
        (all the pooler reads of the f32 hidden stream; see src/encoder.py)."""
        X, X32 = XX
        act = self._dropout_active()
        p_attn, p_hid = (self.attn_dropout, self.hidden_dropout) if act else (0.0, 0.0)
        base = _seed() if act and (p_attn > 0 or p_hid > 0) else 0
        need_grad = torch.is_grad_enabled() and (X.requires_grad or any(lw.trainable() for lw in self._lw))
        return encoder_stack(self._lw, X, X32, km, nb, L, p_attn, p_hid,
                             lambda i: (_mix(base, 3 * i), _mix(base, 3 * i + 1), _mix(base, 3 * i + 2)),
                             need_grad, self._grad_ready_hook, cls_only=CLS_ONLY)

    def _pool(self, X, nb, L):
        """the pooler on the [CLS] rows: X is the last layer's [nb, 768] [CLS] rows (_encode) or
        its whole [nb * L, 768] output"""
        return self.pooler(X.view(nb, L, 768) if X.shape[0] != nb or L == 1 else X.view(nb, 1, 768))

    # ---------------------------------------------------------------- reference forwards
    def forward(self, input_txt, attention_mask, segment, input_img):
        self._prepare()
        B = input_txt.shape[0]
        proj = self.img_embeddings.project(self._image_feats(input_img))
        X, km, L = self._embed(input_txt, attention_mask, segment, proj)
        return self._pool(self._encode(X, km, B, L), B, L)

    def _variant(self, input_txt, attention_mask, segment, input_img, idx):
        if torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters()):
            raise NotImplementedError("variant forwards are inference passes; call them under torch.no_grad()")
        self._prepare()
        B = input_txt.shape[0]
        proj = self.img_embeddings.project(self._image_feats(input_img))
        idx = torch.as_tensor(idx, dtype=torch.long).to(proj.device)
        X, km, L = self._embed(input_txt, attention_mask, segment, proj, idx=idx, Lout=idx.numel())
        return self._pool(self._encode(X, km, B, L), B, L)

    def forward_img_only(self, input_txt, attention_mask, segment, input_img):
        return self._variant(input_txt, attention_mask, segment, input_img, torch.arange(self.n_img + 2))

    def forward_txt_only(self, input_txt, attention_mask, segment, input_img):
        T = input_txt.shape[1]
        idx = torch.cat([torch.zeros(1, dtype=torch.long), torch.arange(T) + self.n_img + 2])
        return self._variant(input_txt, attention_mask, segment, input_img, idx)

    def forward_control(self, input_txt, attention_mask, segment, input_img, control_modal):
        total_embeds = input_txt.size(1) + self.n_img + 2
        if control_modal == "image":
            num_embeds = self.n_img + 1
        elif control_modal == "text":
            num_embeds = input_txt.size(1)
        else:
            raise ValueError("control_modal must be either image or text")
        return self._variant(input_txt, attention_mask, segment, input_img,
                             control_indices(total_embeds, num_embeds))

    # ---------------------------------------------------------------- sub-module APIs
    def _run_encoder_api(self, hidden, ext_mask, all_layers):
        self._prepare()
        B, L, H = hidden.shape
        km = ext_mask.reshape(B, L).float().contiguous()
        X = hidden.reshape(B * L, H).to(torch.bfloat16).contiguous()
        X32 = hidden.reshape(B * L, H).detach().float().contiguous()
        act = self._dropout_active()
        p_attn, p_hid = (self.attn_dropout, self.hidden_dropout) if act else (0.0, 0.0)
        base = _seed() if act else 0
        outs = encoder_stack(self._lw, X, X32, km, B, L, p_attn, p_hid,
                             lambda i: (_mix(base, 3 * i), _mix(base, 3 * i + 1), _mix(base, 3 * i + 2)),
                             torch.is_grad_enabled(), None, all_layers=all_layers)
        outs = outs if all_layers else [outs]
        return [o.view(B, L, H) for o in outs]

    def _image_embeddings(self, proj):
        self._prepare()
        B = proj.shape[0]
        dummy = torch.zeros(B, 0, dtype=torch.long, device=proj.device)
        (_, X32), _, L = self._embed(dummy, dummy, dummy, proj, idx=torch.arange(self.n_img + 2, device=proj.device),
                                     Lout=self.n_img + 2)
        return X32.view(B, L, 768)

    def _text_embeddings(self, ids, token_type_ids=None):
        self._prepare()
        B, T = ids.shape
        seg = torch.zeros_like(ids) if token_type_ids is None else token_type_ids
        proj = torch.zeros(B, self.n_img, 768, device=ids.device)
        idx = torch.arange(T, device=ids.device) + self.n_img + 2
        (_, X32), _, L = self._embed(ids, torch.ones_like(ids), seg, proj, idx=idx, Lout=T)
        return X32.view(B, T, 768)


def control_indices(total_embeds, num_embeds):
    """forward_control's index draw (src/mmbt.py:198-201), from the global torch RNG."""
    indices = torch.zeros(num_embeds + 1)
    ind_sampled, _ = torch.sort(torch.randperm(total_embeds - 1)[:num_embeds] + 1)
    indices[1:] = ind_sampled
    return indices.long()


class MultimodalBertClf(nn.Module):
    def __init__(self, args):
        super().__init__()
        self.args = args
        self.enc = MultimodalBertEncoder(args)
        self.clf = nn.Linear(args.hidden_sz, args.n_classes)
        self.loss = nn.CrossEntropyLoss()
        entries, compute = self.enc._flat_entries("enc.")
        named = dict(self.named_parameters())
        entries = [("clf.weight", named["clf.weight"]), ("clf.bias", named["clf.bias"])] + entries
        self.enc._attach_store(ParamStore(entries, compute), "enc.")
        self.enc._prefix = "enc."

    @property
    def store(self):
        return self.enc._store

    def _apply(self, fn, *a, **k):
        out = super()._apply(fn, *a, **k)
        self.enc._store.build()
        self.enc._refresh_views()
        return out

    def forward(self, txt, mask, segment, img):
        return self.clf(self.enc(txt, mask, segment, img))

    def forward_img_only(self, txt, mask, segment, img):
        return self.clf(self.enc.forward_img_only(txt, mask, segment, img))

    def forward_txt_only(self, txt, mask, segment, img):
        return self.clf(self.enc.forward_txt_only(txt, mask, segment, img))

    def forward_control(self, txt, mask, segment, img, control_modal):
        return self.clf(self.enc.forward_control(txt, mask, segment, img, control_modal))

    def compute_loss(self, y_hat, y, eval=False):
        return self.loss(y_hat, y)
