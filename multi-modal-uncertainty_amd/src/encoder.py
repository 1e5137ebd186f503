"""Fused BERT layer on the HIP kernels: forward / backward kernel sequences and the
autograd Function the encoder stacks (replaces pytorch_pretrained_bert BertLayer,
called through ``self.encoder(...)`` at src/mmbt.py:124-126).

Forward per layer (M = B*L token rows, bf16 GEMM operands, f32 accumulation):
  qkv = X Wqkv^T + bqkv                       mmu_gemm  (fused Q|K|V, [M, 2304])
  O, lse = attention(qkv, keymask)            mmu_attention_fwd (dropout on P)
  S1 = R + dropout(O Wo^T + bo)               mmu_gemm  EPI_BIAS_DROP_RES, f32 residual + f32 out
  A = LN1(S1)                                 mmu_layernorm_fwd_f32 (bf16 operand)
  H  = gelu(A W1^T + b1)                      mmu_gemm  EPI_BIAS_GELU (saves Z = gelu'(.), bf16)
  S2 = LN1(S1)_f32 + dropout(H W2^T + b2)     mmu_gemm  EPI_BIAS_DROP_RES, f32, the residual LN1(S1)
                                              recomputed from S1 in the epilogue (res_ln)
  Y = LN2(S2)                                 mmu_layernorm_fwd_f32
The hidden state travels as bf16 X (the next GEMM's operand) plus its f32 residual R: the
embeddings' f32 rows for layer 0, then the previous layer's S2 with its LN statistics (the
f32 LayerNorm output is recomputed where it is added, never written).  The residual adds
and LN inputs stay f32, as in the reference's fp32 layer:
with the stream rounded to bf16 at each of the 48 LN / residual points of 12 layers the
logits drift by up to 1.6 % of their scale (CPU emulation of the rounding points,
DESIGN.md §4), with it f32 by 0.5 %.
Backward mirrors it (the gradient stream is bf16); weight gradients are written straight into the flat f32
gradient buffer (src/params.py) and skipped when the layer is frozen
(src/framework.py:284-285 toggles requires_grad).
"""

import os

import torch

from . import kernels as K

HID, FFN, HEADS = 768, 3072, 12
bf16 = torch.bfloat16


class LayerWeights:
    """Views of one BertLayer's parameters in the ParamStore (f32 masters, bf16 copies, f32 grads)."""

    def __init__(self, store, prefix, layer_module):
        self.store, self.prefix, self.module = store, prefix, layer_module
        q = [f"{prefix}attention.self.{n}.weight" for n in ("query", "key", "value")]
        qb = [f"{prefix}attention.self.{n}.bias" for n in ("query", "key", "value")]
        self._names = dict(
            wqkv=q, bqkv=qb,
            wo=[f"{prefix}attention.output.dense.weight"], bo=[f"{prefix}attention.output.dense.bias"],
            ln1w=[f"{prefix}attention.output.LayerNorm.weight"], ln1b=[f"{prefix}attention.output.LayerNorm.bias"],
            w1=[f"{prefix}intermediate.dense.weight"], b1=[f"{prefix}intermediate.dense.bias"],
            w2=[f"{prefix}output.dense.weight"], b2=[f"{prefix}output.dense.bias"],
            ln2w=[f"{prefix}output.LayerNorm.weight"], ln2b=[f"{prefix}output.LayerNorm.bias"])
        self._shapes = dict(wqkv=(3 * HID, HID), bqkv=(3 * HID,), wo=(HID, HID), bo=(HID,), ln1w=(HID,), ln1b=(HID,),
                            w1=(FFN, HID), b1=(FFN,), w2=(HID, FFN), b2=(HID,), ln2w=(HID,), ln2b=(HID,))
        self.refresh()

    def refresh(self):
        s = self.store
        for k, names in self._names.items():
            setattr(self, k, s.fused(names, self._shapes[k]))
            setattr(self, "g_" + k, s.fused_grad(names, self._shapes[k]))
        for k in ("wqkv", "wo", "w1", "w2"):
            setattr(self, k + "16", s.fused_compute(self._names[k], self._shapes[k]))
        # K-major copies for the data-gradient products dX = dY W (B = W^T): the GEMM's
        # K-contiguous B path runs 9-17 % faster than its N-contiguous one on these shapes
        # (profiles/r2_gemm_bt_ab.txt); dZ = dY2 W2 too, with 2-row tile groups (0.848 ->
        # 0.756 ms, profiles/r2_gemm_group_dz.txt)
        for k in ("wqkv", "wo", "w1", "w2"):
            setattr(self, k + "t16", s.transposed_compute(self._names[k], self._shapes[k]))
        self.anchor = s.params[self._names["wqkv"][0]]

    def trainable(self):
        return self.anchor.requires_grad


def layer_forward(lw, X, R, keymask, B, L, p_attn, p_hid, seeds, save, res_ln=None, out32=False):
    """X bf16 [M, 768] and its f32 residual -> (Y bf16, S2, mean2, rstd2, saved, Y32).

    The f32 residual is ``R`` itself (res_ln None: the embeddings' f32 rows) or the previous
    layer's output LayerNorm recomputed in the GEMM epilogue from its f32 input ``R`` = S2
    and ``res_ln`` = (mean2, rstd2, gamma, beta): the LayerNorms write only their bf16 output
    (the next GEMM operand), never an f32 copy, except Y32 when ``out32`` (the last layer's
    hidden state for the pooler / the encoder API)."""
    M = B * L
    dev = X.device
    f32 = torch.float32
    qkv = torch.empty(M, 3 * HID, dtype=bf16, device=dev)
    K.gemm(X, HID, True, lw.wqkv16, HID, True, qkv, 3 * HID, M, 3 * HID, HID, epi=K.epilogue(K.EPI_STORE, bias=lw.bqkv))
    O = torch.empty(M, HID, dtype=bf16, device=dev)
    lse = torch.empty(B * HEADS, L, dtype=torch.float32, device=dev)
    dmask = K.dropmask_empty(B, L, HEADS, dev) if (save and p_attn > 0) else None
    K.attention_fwd(qkv, keymask, O, lse, B, L, HEADS, p_attn, seeds[0], dmask)
    S1 = torch.empty(M, HID, dtype=f32, device=dev)
    K.gemm(O, HID, True, lw.wo16, HID, True, S1, HID, M, HID, HID,
           epi=K.epilogue(K.EPI_BIAS_DROP_RES, bias=lw.bo, residual=R, drop_p=p_hid, seed=seeds[1], res_ln=res_ln))
    A = torch.empty(M, HID, dtype=bf16, device=dev)
    mean1 = torch.empty(M, dtype=f32, device=dev)
    rstd1 = torch.empty(M, dtype=f32, device=dev)
    K.layernorm_fwd_f32(S1, lw.ln1w, lw.ln1b, A, None, mean1, rstd1)
    Z = torch.empty(M, FFN, dtype=bf16, device=dev) if save else None  # gelu'(A W1^T + b1), for the backward
    Hh = torch.empty(M, FFN, dtype=bf16, device=dev)
    K.gemm(A, HID, True, lw.w116, HID, True, Hh, FFN, M, FFN, HID, epi=K.epilogue(K.EPI_BIAS_GELU, bias=lw.b1, aux=Z))
    S2 = torch.empty(M, HID, dtype=f32, device=dev)
    K.gemm(Hh, FFN, True, lw.w216, FFN, True, S2, HID, M, HID, FFN,
           epi=K.epilogue(K.EPI_BIAS_DROP_RES, bias=lw.b2, residual=S1, drop_p=p_hid, seed=seeds[2],
                          res_ln=(mean1, rstd1, lw.ln1w, lw.ln1b)))
    Y = torch.empty(M, HID, dtype=bf16, device=dev)
    Y32 = torch.empty(M, HID, dtype=f32, device=dev) if out32 is True else None
    mean2 = torch.empty(M, dtype=f32, device=dev)
    rstd2 = torch.empty(M, dtype=f32, device=dev)
    K.layernorm_fwd_f32(S2, lw.ln2w, lw.ln2b, Y, Y32, mean2, rstd2)
    if out32 == "cls":  # only the [CLS] rows' f32 output (the pooler's input): the same kernel on them
        S2c = S2.view(B, L, HID)[:, 0].contiguous()
        Y32 = torch.empty(B, HID, dtype=f32, device=dev)
        K.layernorm_fwd_f32(S2c, lw.ln2w, lw.ln2b, torch.empty(B, HID, dtype=bf16, device=dev), Y32)
    saved = (X, qkv, O, lse, dmask, S1, mean1, rstd1, A, Z, Hh, S2, mean2, rstd2) if save else None
    return Y, S2, mean2, rstd2, saved, Y32


def encoder_stack(lws, X, X32, keymask, B, L, p_attn, p_hid, seeds_of, need_grad, hook=None, all_layers=False,
                  cls_only=False):
    """Run the fused layers over (X bf16, X32 f32 embedding rows); returns the f32 hidden
    state of the last layer, or of every layer (all_layers); with cls_only only the last layer's
    [CLS] rows [B, 768] (the pooler's input: no f32 copy of the other B (L - 1) rows, and no
    [B L, 768] f32 zero gradient for them in the backward)."""
    R, rln, outs = X32, None, []
    n = len(lws)
    for i, lw in enumerate(lws):
        out32 = all_layers or i == n - 1
        if out32 and cls_only and not all_layers:
            out32 = "cls"
        if need_grad:
            # (layer 0's backward is the encoder's last: it flushes the deferred weight gradients)
            X, R, mu, rs, Y32 = BertLayerFunction.apply(X, R, lw.anchor, lw, keymask, B, L, p_attn, p_hid,
                                                        seeds_of(i), hook, rln, out32, i == 0)
        else:
            X, R, mu, rs, _, Y32 = layer_forward(lw, X, R, keymask, B, L, p_attn, p_hid, seeds_of(i), False, rln,
                                                 out32)
        rln = (mu, rs, lw.ln2w, lw.ln2b)
        if out32:
            outs.append(Y32)
    return outs if all_layers else outs[-1]


DEFER_WGRAD = True
# the deferred closures keep their input tensors (dY2, Hh, dZ, A, dAo, O, dqkv, X: ~3 GB per layer
# at batch 256, L = 513) alive until the flush; above this many retained bytes the work deferred
# so far is flushed early (issued on the side stream at once), so larger batches / sequences do
# not run out of memory.  None: a quarter of the device memory.
DEFER_MAX_BYTES = None

# per device: the weight-gradient work of the layers' backwards, deferred (DEFER_WGRAD) until
# the encoder's data-gradient chain is enqueued, then issued on the side stream
_deferred = {}
_deferred_bytes = {}


def _defer_budget(dev):
    if DEFER_MAX_BYTES is not None:
        return DEFER_MAX_BYTES
    return torch.cuda.get_device_properties(dev).total_memory // 4


# INTERLEAVE (MMU_WGRAD_INTERLEAVE=1): at the end of the encoder's data-gradient chain the deferred
# work is not issued at once but item by item from the trunk's BatchNorm backwards
# (K.side_pump, called by src/resnet.py), the rest when the backward ends.  A HIP graph replays
# its nodes in capture order, so the all-at-once flush runs the ~200 weight-gradient kernels
# before the first trunk kernel even at batch 32, where they would fit beside the trunk's
# short BatchNorm / conv kernels (profiles/r6_wgrad_interleave_ab.txt).
# MMU_WGRAD_INTERLEAVE=2: the first trunk BatchNorm backward issues ALL of it, behind everything the
# main stream has enqueued by then (the embedding and image-projection backward then run without the
# side stream's weight-gradient GEMMs holding every CU)
# (default 2: -0.37 ms at batch 256, neutral at 32, profiles/r6_wgrad_flush_late_ab.txt; 0 = round 5)
INTERLEAVE = os.environ.get("MMU_WGRAD_INTERLEAVE", "2") != "0"
INTERLEAVE_ALL = os.environ.get("MMU_WGRAD_INTERLEAVE", "2") == "2"
_pending = {}  # per device: flushed items not yet issued (INTERLEAVE)


def _issue(dev, items):
    """the items on the side stream (which already waits for the encoder's dX chain)"""
    side = K.side_stream(dev)
    with torch.cuda.stream(side):
        e0 = _mark()
        for fn, tensors in items:
            for t in tensors:
                t.record_stream(side)
            fn()
        if e0 is not None:
            _block_extra.append((e0, _mark()))


def _flush_deferred(dev, interleave=False):
    """Issue the deferred weight-gradient work (and the DP hooks after it) on the side stream,
    behind everything the main stream has enqueued so far -- the whole encoder dX chain -- so
    it runs beside what follows (embedding backward, the ResNet trunk's backward); with
    `interleave` it is handed to pump_deferred instead."""
    items = _deferred.pop(dev, None)
    _deferred_bytes.pop(dev, None)
    if not items:
        return
    main = torch.cuda.current_stream(dev)
    side = K.side_stream(dev)
    side.wait_stream(main)
    if interleave:
        _pending.setdefault(dev, []).extend(items)
    else:
        _issue(dev, items)
    K.join_at_backward_end(main, side)


def pump_deferred(dev, n=1):
    """issue up to n of the flushed items (INTERLEAVE) on the side stream (INTERLEAVE_ALL: all of
    them, after the main stream's work so far)"""
    items = _pending.get(dev)
    if items:
        if INTERLEAVE_ALL:
            K.side_stream(dev).wait_stream(torch.cuda.current_stream(dev))
            n = len(items)
        _pending[dev] = items[n:]
        _issue(dev, items[:n])


K.set_side_pump(pump_deferred)


def _defer(dev, fn, tensors):
    items = _deferred.get(dev)
    if items is None:
        items = _deferred[dev] = []

        def at_end():  # (nothing may stay deferred past the backward)
            if dev in _deferred:
                _flush_deferred(dev)
            if _pending.get(dev):
                _issue(dev, _pending.pop(dev))
            torch.cuda.current_stream(dev).wait_stream(K.side_stream(dev))

        torch.autograd.Variable._execution_engine.queue_callback(at_end)
    items.append((fn, tensors))
    held = _deferred_bytes.get(dev, 0) + sum(t.numel() * t.element_size() for t in tensors)
    _deferred_bytes[dev] = held
    if held > _defer_budget(dev):  # retained inputs over budget: issue what is deferred so far
        _flush_deferred(dev)


class _Side:
    """The weight-gradient work of a layer's backward (split-K dW products, LN / bias
    column-sum reductions): with DEFER_WGRAD (CUDA) it is deferred until layer 0's backward
    has enqueued the encoder's whole data-gradient chain, then issued on the side stream
    (_flush_deferred), where it runs beside the embedding and ResNet-trunk backward -- a
    chain of short, latency-bound kernels.  Same-box A/B (profiles/r3_defer_wgrad_ab.txt):
    165.6 -> 163.3 ms per step at batch 256.  The inputs it reads stay alive until then
    (peak HBM 75 GB at batch 256), at most DEFER_MAX_BYTES of them: past that the work
    deferred so far is flushed early.  (Round 1 issued each piece on the side stream as soon as
    its inputs existed: 210 -> 207 ms, an opt-in that this replaces.)"""

    def __init__(self, dev, on):
        self.dev = dev
        self.defer = on and DEFER_WGRAD and dev.type == "cuda"

    def run(self, fn, *tensors):
        if self.defer:
            return _defer(self.dev, fn, tensors)
        return fn()


def layer_backward(lw, saved, dY, keymask, B, L, p_attn, p_hid, seeds, wgrad):
    X, qkv, O, lse, dmask, S1, mean1, rstd1, A, Z, Hh, S2, mean2, rstd2 = saved
    M = B * L
    dev = dY.device
    P = K.ln_parts(M)
    side = _Side(dev, wgrad)
    pw = pb = pbias = pw1 = pb1 = pbias1 = None
    if wgrad:  # two sets: the side stream reduces one while the main stream fills the other
        pw, pb, pbias, pw1, pb1, pbias1 = (torch.empty(P, HID, dtype=torch.float32, device=dev) for _ in range(6))
    acc = K.epilogue(K.EPI_STORE, accumulate=True)
    # ---- output LayerNorm + dropout + W2
    dS2 = torch.empty(M, HID, dtype=bf16, device=dev)
    dY2 = torch.empty(M, HID, dtype=bf16, device=dev)
    K.layernorm_bwd(dY, S2, mean2, rstd2, lw.ln2w, dS2, dY2, p_hid, seeds[2], pw, pb, pbias)
    if wgrad:
        def w2():
            K.colsum_reduce_multi([(pw, lw.g_ln2w), (pb, lw.g_ln2b), (pbias, lw.g_b2)], accumulate=True)
            K.gemm(dY2, HID, False, Hh, FFN, False, lw.g_w2, FFN, HID, FFN, M, epi=acc)
        side.run(w2, pw, pb, pbias, dY2, Hh)
    dZ = torch.empty(M, FFN, dtype=bf16, device=dev)
    # dgelu epilogue also accumulates the intermediate-bias gradient (column sums of dZ) in place
    K.gemm(dY2, HID, True, lw.w2t16, HID, True, dZ, FFN, M, FFN, HID,
           epi=K.epilogue(K.EPI_DGELU, aux=Z, colsum=lw.g_b1 if wgrad else None))
    if wgrad:
        side.run(lambda: K.gemm(dZ, FFN, False, A, HID, False, lw.g_w1, HID, FFN, HID, M, epi=acc), dZ, A)
    dA = torch.empty(M, HID, dtype=bf16, device=dev)
    K.gemm(dZ, FFN, True, lw.w1t16, FFN, True, dA, HID, M, HID, FFN, epi=K.epilogue(K.EPI_ADD_RES, residual=dS2))
    # ---- attention-output LayerNorm + dropout + Wo
    dS1 = torch.empty(M, HID, dtype=bf16, device=dev)
    dAo = torch.empty(M, HID, dtype=bf16, device=dev)
    K.layernorm_bwd(dA, S1, mean1, rstd1, lw.ln1w, dS1, dAo, p_hid, seeds[1], pw1, pb1, pbias1)
    if wgrad:
        def wo():
            K.colsum_reduce_multi([(pw1, lw.g_ln1w), (pb1, lw.g_ln1b), (pbias1, lw.g_bo)], accumulate=True)
            K.gemm(dAo, HID, False, O, HID, False, lw.g_wo, HID, HID, HID, M, epi=acc)
        side.run(wo, pw1, pb1, pbias1, dAo, O)
    dO = torch.empty(M, HID, dtype=bf16, device=dev)
    K.gemm(dAo, HID, True, lw.wot16, HID, True, dO, HID, M, HID, HID)
    # ---- attention + fused QKV
    dqkv = torch.empty(M, 3 * HID, dtype=bf16, device=dev)
    delta = torch.empty(B * HEADS, L, dtype=torch.float32, device=dev)
    # the attention backward also emits per-block column sums of dQ / dK / dV (bias grads)
    dbp = K.attention_dbias_parts(B, L, HEADS, dev) if wgrad else None
    K.attention_bwd(qkv, keymask, O, dO, lse, delta, dqkv, B, L, HEADS, p_attn, seeds[0], dmask, dbp)
    if wgrad:
        def wqkv():
            K.attention_dbias_reduce(dbp, B, L, lw.g_bqkv, HEADS)
            K.gemm(dqkv, 3 * HID, False, X, HID, False, lw.g_wqkv, HID, 3 * HID, HID, M, epi=acc)
        side.run(wqkv, dqkv, X, dbp)
    dX = torch.empty(M, HID, dtype=bf16, device=dev)
    K.gemm(dqkv, 3 * HID, True, lw.wqkvt16, 3 * HID, True, dX, HID, M, HID, 3 * HID,
           epi=K.epilogue(K.EPI_ADD_RES, residual=dS1))
    return dX, side


_block_events = None  # [(start, end)] HIP events around every fused-layer fwd / bwd while timing
_block_extra = []     # ... and around the layers' deferred weight-gradient work (side stream)


def block_timing(on):
    """Time every BertLayer forward and backward on the stream it runs on (bench.py: the
    fused-block roofline of BASELINE's north star), the deferred weight-gradient work of
    the backwards included (timed on the side stream, beside whatever it overlaps)."""
    global _block_events, _block_extra
    _block_events = [] if on else None
    _block_extra = []


def block_timing_read():
    """-> (total ms, number of layer passes) since block_timing(True); synchronises."""
    if not _block_events:
        return 0.0, 0
    torch.cuda.synchronize()
    ms = sum(a.elapsed_time(b) for a, b in _block_events) + sum(a.elapsed_time(b) for a, b in _block_extra)
    return ms, len(_block_events)


def _mark():
    if _block_events is None:
        return None
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    return e


class BertLayerFunction(torch.autograd.Function):
    """One fused BertLayer: X bf16 [B*L, 768] + its f32 residual (R, res_ln: see
    layer_forward) -> (Y, S2, mean2, rstd2, Y32).  S2 / mean2 / rstd2 (the next layer's
    residual source) are non-differentiable; the layer's whole input gradient is returned
    for X.  The output gradient arrives on Y from the next layer or on Y32 (out32: the last
    layer) from the pooler.  ``anchor`` (the layer's query weight) only makes autograd run
    backward when the layer is trainable."""

    @staticmethod
    def forward(ctx, X, R, anchor, lw, keymask, B, L, p_attn, p_hid, seeds, on_grads_ready, res_ln=None,
                out32=True, flush=False):
        ctx.set_materialize_grads(False)
        e0 = _mark()
        Y, S2, mean2, rstd2, saved, Y32 = layer_forward(lw, X, R, keymask, B, L, p_attn, p_hid, seeds, True,
                                                        res_ln, out32)
        if e0 is not None:
            _block_events.append((e0, _mark()))
        ctx.saved_bufs = saved
        ctx.meta = (lw, keymask, B, L, p_attn, p_hid, seeds, on_grads_ready, flush)
        ctx.mark_non_differentiable(S2, mean2, rstd2)
        if Y32 is None:
            Y32 = Y.new_empty(0, dtype=torch.float32)
            ctx.mark_non_differentiable(Y32)
        return Y, S2, mean2, rstd2, Y32

    @staticmethod
    def backward(ctx, dY, _dS2, _dmean2, _drstd2, dY32):
        lw, keymask, B, L, p_attn, p_hid, seeds, hook, flush = ctx.meta
        wgrad = lw.trainable()
        if dY32 is not None and dY32.numel():
            if dY32.shape[0] == B and B * L != B:  # out32 "cls": the gradient of the [CLS] rows only
                g = torch.zeros(B * L, HID, dtype=bf16, device=dY32.device) if dY is None else dY.clone()
                g.view(B, L, HID)[:, 0] += dY32.to(bf16)
                dY = g
            else:
                dY = dY32.to(bf16) if dY is None else dY + dY32.to(bf16)
        if dY is None:
            return (None,) * 14
        e0 = _mark()
        dX, side = layer_backward(lw, ctx.saved_bufs, dY.contiguous(), keymask, B, L, p_attn, p_hid, seeds, wgrad)
        if e0 is not None:
            _block_events.append((e0, _mark()))
        ctx.saved_bufs = None
        if wgrad and side.defer:
            if hook is not None:  # the bucket all-reduce follows the layer's deferred work
                _defer(side.dev, lambda: hook(lw), ())
            if flush:
                _flush_deferred(side.dev, INTERLEAVE)
        elif wgrad and hook is not None:
            hook(lw)
        return (dX,) + (None,) * 13


