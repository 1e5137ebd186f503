"""torch-tensor front-end of the HIP kernels (pointers + current HIP stream).

Every function enqueues on ``torch.cuda.current_stream()`` of the tensors'
device and raises if a tensor is not on a HIP device or has the wrong
dtype/layout -- there is no CPU fallback ("no fallback").
"""
import ctypes

import torch

from . import _native as N
from ._native import (Epilogue, EPI_STORE, EPI_BIAS_GELU, EPI_BIAS_DROP_RES, EPI_DGELU, EPI_ADD_RES,  # noqa: F401
                      EPI_BIAS_DROP_QGELU, EPI_STORE_STATS, EPI_STORE_BNB, EPI_ADD_RES_BNB)


def bn_stats_table(rows, C, device):
    """the float2 [ceil(rows / 64)][C] BatchNorm statistics table a conv's STORE_STATS epilogue
    writes (include/mmu.h MMU_EPI_STORE_STATS) -> (table, nparts)"""
    nparts = (rows + 63) // 64
    return torch.empty(nparts * C * 2, dtype=torch.float32, device=device), nparts


def _dev_check(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise N.NativeError("mmu kernels need tensors on a HIP (cuda) device; got CPU tensor "
                                f"{tuple(t.shape)} {t.dtype}")


_raw_stream = torch._C._cuda_getCurrentRawStream  # (device index) -> the current hipStream_t as an int


def _stream(t):
    # the raw handle, without building a torch.cuda.Stream object: this runs once per kernel
    # launch, ~800 times per training step
    return _raw_stream(t.get_device())


def _ptr(t):
    return None if t is None else t.data_ptr()


def _want(t, dtype, name):
    if t.dtype != dtype:
        raise N.NativeError(f"{name}: expected {dtype}, got {t.dtype}")


def epilogue(kind=EPI_STORE, bias=None, residual=None, aux=None, colsum=None, drop_p=0.0, seed=0, accumulate=False,
             ldr=0, ldx=0, bias_bstride=0, res_bstride=0, aux_bstride=0, colsum_bstride=0, res_ln=None,
             res_ln_bstride=0, bn=None, res_mask=None):
    """res_ln = (mean, rstd, w, b): with BIAS_DROP_RES into an f32 C, the residual is the LayerNorm
    output recomputed from the f32 ``residual`` rows (the previous LayerNorm's input).
    bn = (x, relu_mask or None, mean): with STORE_BNB / ADD_RES_BNB, the BatchNorm whose dY the
    product forms; colsum is then its backward reduction table (bn_stats_table of x's rows).
    res_mask (ADD_RES / ADD_RES_BNB): a ReLU mask [M*N/8] u8 gating the residual per element."""
    e = Epilogue()
    e.kind, e.accumulate = kind, int(accumulate)
    e.bias, e.bias_bstride = _ptr(bias), bias_bstride
    e.residual, e.ldr, e.res_bstride = _ptr(residual), ldr or (residual.shape[-1] if residual is not None else 0), \
        res_bstride
    e.aux, e.ldx, e.aux_bstride = _ptr(aux), ldx or (aux.shape[-1] if aux is not None else 0), aux_bstride
    e.colsum, e.colsum_bstride = _ptr(colsum), colsum_bstride
    e.drop_p, e.seed = float(drop_p), int(seed) & 0xFFFFFFFFFFFFFFFF
    e.workspace, e.workspace_floats = None, 0
    if res_ln is not None:
        for t in res_ln:
            _want(t, torch.float32, "epilogue res_ln")
            if not t.is_contiguous():
                raise N.NativeError("epilogue res_ln tensors must be contiguous")
        e.res_ln_mean, e.res_ln_rstd, e.res_ln_w, e.res_ln_b = (_ptr(t) for t in res_ln)
        e.res_ln_bstride = res_ln_bstride
    if bn is not None:
        _bnb_check(*bn, "epilogue bn")
        e.bn_x, e.bn_mask, e.bn_mean = (_ptr(t) for t in bn)
    if res_mask is not None:
        if res_mask.dtype != torch.uint8 or not res_mask.is_contiguous() or residual is None \
                or res_mask.numel() * 8 != residual.numel():
            raise N.NativeError("epilogue res_mask: contiguous uint8 with numel = residual.numel() / 8")
        e.res_mask = _ptr(res_mask)
    return e


def _bnb_check(x, mask, mean, what):
    if (x.dtype != torch.bfloat16 or mean.dtype != torch.float32 or not mean.is_contiguous()
            or mean.numel() != x.shape[1] or not x.is_contiguous(memory_format=torch.channels_last)):
        raise N.NativeError(f"{what}: (x channels-last bf16, relu_mask, mean f32 [C]) of a training BatchNorm")
    _bn_mask_check(mask, x, what)


SPLITK_WS_FLOATS = 16 << 20  # 64 MiB per (device, stream), reused stream-ordered by every split-K product
_ws = {}
_side = {}


def _splitk_workspace(dev):
    key = (dev, _raw_stream(dev.index if dev.index is not None else torch.cuda.current_device()))
    t = _ws.get(key)
    if t is None:
        t = _ws[key] = torch.empty(SPLITK_WS_FLOATS, dtype=torch.float32, device=dev)
    return t


SIDE_CU_FRAC = None  # e.g. 0.75: the side stream's kernels run on that fraction of every XCD's CUs


def _cu_masked_stream(dev, frac):
    """A stream whose dispatches are restricted to ``frac`` of the CUs (hipExtStreamCreateWithCUMask),
    so the side stream's weight-gradient GEMMs leave the rest to the main stream's chain.  The
    mask keeps whole 8-CU groups, 3 of every 4 for 0.75: balanced across the 8 XCDs whether the
    runtime numbers CUs XCD-blocked or XCD-interleaved."""
    import ctypes
    n_cu = torch.cuda.get_device_properties(dev).multi_processor_count
    groups = n_cu // 8
    keep = max(1, min(groups, round(frac * groups)))
    # spread the kept groups evenly over the group index (Bresenham)
    bits = [0] * ((n_cu + 31) // 32)
    for g in range(groups):
        if (g + 1) * keep // groups != g * keep // groups:
            for c in range(8 * g, 8 * g + 8):
                bits[c // 32] |= 1 << (c % 32)
    hip = ctypes.CDLL("libamdhip64.so.7")  # the runtime torch already loaded (same soname)
    h = ctypes.c_void_p()
    arr = (ctypes.c_uint32 * len(bits))(*bits)
    with torch.cuda.device(dev):
        err = hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), ctypes.c_uint32(len(bits)), arr)
    if err != 0:
        raise N.NativeError(f"hipExtStreamCreateWithCUMask failed ({err})")
    return torch.cuda.ExternalStream(h.value, device=dev)


def side_stream(dev):
    """The per-device stream the weight-gradient products run on, beside the data-gradient
    chain of the backward (src/encoder.py)."""
    dev = torch.device(dev)
    s = _side.get(dev)
    if s is None:
        s = _side[dev] = (_cu_masked_stream(dev, SIDE_CU_FRAC) if SIDE_CU_FRAC
                          else torch.cuda.Stream(device=dev))
    return s


_side_pump = None


def set_side_pump(fn):
    """src/encoder.py's pump_deferred: deferred side-stream work issued piecewise"""
    global _side_pump
    _side_pump = fn


def side_pump(dev, n=1):
    """issue up to n pieces of the encoder's flushed weight-gradient work (interleave mode)"""
    if _side_pump is not None:
        _side_pump(dev, n)


def side_stream_if_any(dev):
    """the device's side stream if one was created, else None"""
    return _side.get(torch.device(dev))


_pending_join = set()


def join_at_backward_end(main, side):
    """Once per backward pass: ``main`` waits for ``side`` when the autograd engine finishes,
    so every consumer of .grad (optimizer, all-reduce, tests) sees the side stream's work."""
    key = (main.cuda_stream, side.cuda_stream)
    if key in _pending_join:
        return
    _pending_join.add(key)

    def join():
        _pending_join.discard(key)
        main.wait_stream(side)

    torch.autograd.Variable._execution_engine.queue_callback(join)


def gemm(A, lda, a_kmajor, B, ldb, b_kmajor, C, ldc, M, N_, K, epi=None, batch=1, sA=0, sB=0, sC=0):
    """C[m,n] = sum_k A(m,k) B(n,k) (+ fused epilogue); see mmu_gemm in include/mmu.h."""
    _dev_check(A, B, C)
    _want(A, torch.bfloat16, "gemm A")
    _want(B, torch.bfloat16, "gemm B")
    cdt = N.MMU_F32 if C.dtype == torch.float32 else N.MMU_BF16
    if C.dtype not in (torch.float32, torch.bfloat16):
        raise N.NativeError("gemm C must be f32 or bf16")
    # the per-stream f32 scratch serves the split-K weight gradients
    if epi is None:
        epi = epilogue(EPI_STORE)
    if not epi.workspace:  # (on a copy: a caller's epilogue may be reused on another stream)
        epi = type(epi).from_buffer_copy(epi)
        ws = _splitk_workspace(C.device)
        epi.workspace, epi.workspace_floats = ws.data_ptr(), ws.numel()
    N.call("mmu_gemm", _ptr(A), lda, int(a_kmajor), _ptr(B), ldb, int(b_kmajor), _ptr(C), ldc, cdt, M, N_, K,
           batch, sA, sB, sC, ctypes.byref(epi) if epi is not None else None, _stream(C))
    if _alg["on"]:
        _count_alg(M, N_, K, batch, 4 if cdt == N.MMU_F32 else 2, epi)
    return C


def colsum_reduce_multi(jobs, accumulate=False):
    """[(partial [parts_z, N], out [N]), ...] (1..4 jobs of one width N): one launch
    (mmu_colsum_reduce_multi)"""
    n = len(jobs)
    N_ = jobs[0][0].shape[1]
    for part, out in jobs:
        _dev_check(part, out)
        if part.dtype != torch.float32 or out.dtype != torch.float32 or part.shape[1] != N_ or out.numel() != N_ \
                or not part.is_contiguous() or not out.is_contiguous():
            raise N.NativeError("colsum_reduce_multi: f32 contiguous [parts, N] partials / [N] outputs of one N")
    parts_p = (ctypes.c_void_p * n)(*[p.data_ptr() for p, _ in jobs])
    rows = (ctypes.c_int64 * n)(*[p.shape[0] for p, _ in jobs])
    outs = (ctypes.c_void_p * n)(*[o.data_ptr() for _, o in jobs])
    N.call("mmu_colsum_reduce_multi", n, ctypes.cast(parts_p, ctypes.c_void_p), ctypes.cast(rows, ctypes.c_void_p),
           ctypes.cast(outs, ctypes.c_void_p), N_, int(accumulate), _stream(jobs[0][1]))


def colsum_reduce(partial, out, accumulate=False):
    _dev_check(partial, out)
    N.call("mmu_colsum_reduce", _ptr(partial), partial.shape[0], partial.shape[1], _ptr(out), int(accumulate),
           _stream(out))


def transpose_bf16_batched(jobs, n_jobs, max_rows, max_cols, stream_of):
    """dst = src^T for every (src ptr, dst ptr, rows, cols, src pitch, dst pitch) row of the
    int64 device table ``jobs`` [n_jobs, 6] (pitch 0: dense); see mmu_transpose_bf16_batched.
    ``stream_of``: a tensor on the target device (its current stream is used)."""
    _dev_check(jobs, stream_of)
    if jobs.dtype != torch.int64 or not jobs.is_contiguous() or jobs.numel() < 6 * n_jobs:
        raise N.NativeError("transpose_bf16_batched: jobs must be a contiguous int64 [n_jobs, 6] device table")
    N.call("mmu_transpose_bf16_batched", _ptr(jobs), int(n_jobs), int(max_rows), int(max_cols), _stream(stream_of))


def colsum_bf16(X, out, accumulate=False):
    _dev_check(X, out)
    M, N_ = X.shape
    # scratch for the per-block partial rows (>= ceil(M / 64) x N f32, see mmu_colsum_bf16)
    part = torch.empty(((M + 63) // 64) * N_, dtype=torch.float32, device=X.device)
    N.call("mmu_colsum_bf16", _ptr(X), M, N_, X.stride(0), _ptr(part), _ptr(out), int(accumulate), _stream(X))


def dropmask_empty(batch, L, heads=12, device=None):
    """Keep-bit buffer of the attention-probs dropout: [batch*heads, L, ceil(L/64)] words
    (int64 storage of the kernel's u64; bit k of word j = key 64j+k kept)."""
    return torch.empty(batch * heads, L, (L + 63) // 64, dtype=torch.int64, device=device)


def dropmask_dense(mask, L):
    """[BH, L, W] keep words -> [BH, L, L] float 0/1 (test/debug helper)."""
    bits = torch.arange(64, device=mask.device, dtype=torch.int64)
    d = (mask.unsqueeze(-1) >> bits) & 1
    return d.flatten(-2)[..., :L].float()


def attention_fwd(qkv, keymask, O, lse, batch, L, heads=12, drop_p=0.0, seed=0, dropmask=None):
    _dev_check(qkv, keymask, O, lse)
    _want(qkv, torch.bfloat16, "attention qkv")
    if dropmask is not None:
        _dev_check(dropmask)
        if dropmask.numel() < batch * heads * L * ((L + 63) // 64) or not dropmask.is_contiguous():
            raise ValueError("attention_fwd: dropmask too small / not contiguous")
    N.call("mmu_attention_fwd", _ptr(qkv), qkv.stride(0), _ptr(keymask), _ptr(O), O.stride(0), _ptr(lse), batch, L,
           heads, float(drop_p), int(seed), _ptr(dropmask) if dropmask is not None else None, _stream(qkv))


def attention_dbias_parts(batch, L, heads=12, device=None):
    """Scratch for the fused Q/K/V bias-gradient column sums of attention_bwd."""
    nqb, nkb = (L + 127) // 128, (L + 63) // 64
    return torch.empty((nqb + 2 * nkb) * batch, heads * 64, dtype=torch.float32, device=device)


def attention_dbias_reduce(parts, batch, L, g_bqkv, heads=12):
    """g_bqkv [3 * heads * 64] += the column sums held in `parts` (Q | K | V row ranges)."""
    nqb, nkb = (L + 127) // 128, (L + 63) // 64
    H = heads * 64
    r0, r1 = nqb * batch, (nqb + nkb) * batch
    colsum_reduce_multi([(parts[:r0], g_bqkv[:H]), (parts[r0:r1], g_bqkv[H:2 * H]), (parts[r1:], g_bqkv[2 * H:])],
                        accumulate=True)


def attention_bwd(qkv, keymask, O, dO, lse, delta, dqkv, batch, L, heads=12, drop_p=0.0, seed=0, dropmask=None,
                  dbias_parts=None):
    """`dropmask` = the buffer the forward filled (required when drop_p > 0); `seed` is
    kept for signature symmetry with the forward; `dbias_parts` (attention_dbias_parts)
    collects the Q/K/V bias-gradient column sums."""
    _dev_check(qkv, keymask, O, dO, lse, delta, dqkv)
    if dropmask is not None:
        _dev_check(dropmask)
        if dropmask.numel() < batch * heads * L * ((L + 63) // 64) or not dropmask.is_contiguous():
            raise ValueError("attention_bwd: dropmask too small / not contiguous")
    N.call("mmu_attention_bwd", _ptr(qkv), qkv.stride(0), _ptr(keymask), _ptr(O), O.stride(0), _ptr(dO), dO.stride(0),
           _ptr(lse), _ptr(delta), _ptr(dqkv), dqkv.stride(0), batch, L, heads, float(drop_p), int(seed),
           _ptr(dropmask) if dropmask is not None else None, _ptr(dbias_parts), _stream(qkv))


def layernorm_fwd(X, w, b, Y, mean, rstd, eps=1e-12, group_rows=0, param_stride=0):
    _dev_check(X, w, b, Y, mean, rstd)
    rows, H = X.shape
    N.call("mmu_layernorm_fwd", _ptr(X), _ptr(w), _ptr(b), _ptr(Y), _ptr(mean), _ptr(rstd), rows, H, float(eps),
           int(group_rows), int(param_stride), _stream(X))


def layernorm_fwd_f32(X, w, b, Y, Y32=None, mean=None, rstd=None, eps=1e-12, group_rows=0, param_stride=0):
    """LN of the f32 hidden stream: X f32 -> Y bf16 (GEMM operand) [+ Y32 f32 (next residual)]."""
    _dev_check(X, w, b, Y)
    _want(X, torch.float32, "layernorm_fwd_f32 X")
    _want(Y, torch.bfloat16, "layernorm_fwd_f32 Y")
    if Y32 is not None:
        _want(Y32, torch.float32, "layernorm_fwd_f32 Y32")
    rows, H = X.shape
    N.call("mmu_layernorm_fwd_f32", _ptr(X), _ptr(w), _ptr(b), _ptr(Y), _ptr(Y32), _ptr(mean), _ptr(rstd), rows, H,
           float(eps), int(group_rows), int(param_stride), _stream(X))


LN_ROWS_PER_PART = 64


def layernorm_bwd(dY, X, mean, rstd, w, dX, dXdrop=None, drop_p=0.0, seed=0, part_dw=None, part_db=None,
                  part_dbias=None):
    """X: the forward's LN input, bf16 or f32 (the f32 hidden stream: mmu_layernorm_bwd_f32)."""
    _dev_check(dY, X, mean, rstd, w, dX)
    rows, H = X.shape
    N.call("mmu_layernorm_bwd_f32" if X.dtype == torch.float32 else "mmu_layernorm_bwd", _ptr(dY), _ptr(X), _ptr(mean), _ptr(rstd), _ptr(w), _ptr(dX), _ptr(dXdrop),
           float(drop_p), int(seed), _ptr(part_dw), _ptr(part_db), _ptr(part_dbias), rows, H, LN_ROWS_PER_PART,
           _stream(X))


def layernorm_bwd_res(dY, X, mean, rstd, w, dRes, dX, part_dw=None, part_db=None, part_dbias=None):
    """Pre-LN backward: dX = LN'(dY) + dRes (part_dbias = column sums of that dX)."""
    _dev_check(dY, X, mean, rstd, w, dRes, dX)
    rows, H = X.shape
    N.call("mmu_layernorm_bwd_res", _ptr(dY), _ptr(X), _ptr(mean), _ptr(rstd), _ptr(w), _ptr(dRes), _ptr(dX),
           _ptr(part_dw), _ptr(part_db), _ptr(part_dbias), rows, H, LN_ROWS_PER_PART, _stream(X))


def seqattn_fwd(qkv, O, lse2, S, N_, heads):
    """FLAVA attention over the sequence (= batch) axis; see mmu_seqattn_fwd."""
    _dev_check(qkv, O, lse2)
    _want(qkv, torch.bfloat16, "seqattn qkv")
    D = qkv.shape[1] // (3 * heads)
    if lse2.numel() < S * N_ * heads:
        raise ValueError("seqattn_fwd: lse2 too small")
    N.call("mmu_seqattn_fwd", _ptr(qkv), qkv.stride(0), _ptr(O), O.stride(0), _ptr(lse2), S, N_, heads, D,
           _stream(qkv))


def seqattn_bwd(qkv, O, dO, lse2, delta, dqkv, S, N_, heads):
    _dev_check(qkv, O, dO, lse2, delta, dqkv)
    D = qkv.shape[1] // (3 * heads)
    if delta.numel() < S * N_ * heads:
        raise ValueError("seqattn_bwd: delta too small")
    N.call("mmu_seqattn_bwd", _ptr(qkv), qkv.stride(0), _ptr(O), O.stride(0), _ptr(dO), dO.stride(0), _ptr(lse2),
           _ptr(delta), _ptr(dqkv), dqkv.stride(0), S, N_, heads, D, _stream(qkv))


def ln_parts(rows):
    return (rows + LN_ROWS_PER_PART - 1) // LN_ROWS_PER_PART


def embed_fwd(ids, seg, txt_mask, proj, word, pos, typ, ln_w, ln_b, eps, cls_id, sep_id, idx, V, B, T, n_img, Lout,
              X, keymask, mean=None, rstd=None, drop_txt=0.0, drop_img=0.0, seed=0, X32=None):
    """X32 (optional, f32 like X): the same rows in f32, the encoder's f32 hidden stream."""
    _dev_check(proj, word, pos, typ, ln_w, ln_b, X, keymask)
    if X32 is not None:
        _want(X32, torch.float32, "embed_fwd X32")
        _dev_check(X32)
    N.call("mmu_embed_fwd", _ptr(ids), _ptr(seg), _ptr(txt_mask), _ptr(proj), _ptr(word), _ptr(pos), _ptr(typ),
           _ptr(ln_w), _ptr(ln_b), float(eps), int(cls_id), int(sep_id), _ptr(idx), V, B, T, n_img, Lout, 768,
           float(drop_txt), float(drop_img), int(seed), _ptr(X), _ptr(X32), _ptr(keymask), _ptr(mean), _ptr(rstd),
           _stream(X))


def embed_bwd(dX, ids, seg, proj, word, pos, typ, ln_w, mean, rstd, cls_id, sep_id, B, T, n_img, d_word, d_pos,
              d_type, d_ln_w, d_ln_b, d_proj, drop_txt=0.0, drop_img=0.0, seed=0):
    _dev_check(dX, proj, word, d_word, d_proj)
    ws = torch.empty(N.load().mmu_embed_bwd_ws_floats(B, T, n_img), dtype=torch.float32, device=dX.device)
    N.call("mmu_embed_bwd", _ptr(dX), _ptr(ids), _ptr(seg), _ptr(proj), _ptr(word), _ptr(pos), _ptr(typ),
           _ptr(ln_w), _ptr(mean), _ptr(rstd), int(cls_id), int(sep_id), B, T, n_img, 768, float(drop_txt),
           float(drop_img), int(seed), _ptr(d_word),
           _ptr(d_pos), _ptr(d_type), _ptr(d_ln_w), _ptr(d_ln_b), _ptr(d_proj), _ptr(ws), _stream(dX))


def image_normalize(img_u8, mean, std, out):
    """uint8 HWC crops [B, H, W, 3] -> out = (x/255 - mean) / std as the channels-last
    [B, 3, H, W] image (f32 or bf16); see mmu_image_normalize."""
    _dev_check(img_u8, out)
    _want(img_u8, torch.uint8, "image_normalize input")
    if not img_u8.is_contiguous() or img_u8.shape[-1] != 3:
        raise N.NativeError("image_normalize: input must be contiguous [B, H, W, 3] uint8")
    if out.dtype not in (torch.float32, torch.bfloat16) or out.numel() != img_u8.numel() or \
            not out.is_contiguous(memory_format=torch.channels_last):
        raise N.NativeError("image_normalize: out must be a channels-last f32/bf16 [B, 3, H, W] of the same size")
    m = (ctypes.c_float * 3)(*[float(v) for v in mean])
    s = (ctypes.c_float * 3)(*[float(v) for v in std])
    N.call("mmu_image_normalize", _ptr(img_u8), img_u8.numel(), m, s, _ptr(out),
           N.MMU_F32 if out.dtype == torch.float32 else N.MMU_BF16, _stream(out))
    return out


def maxpool_fwd(x, y, argmax):
    """MaxPool2d(3, 2, 1) of a channels-last bf16 [B, C, H, W] map -> y [B, C, OH, OW]
    (channels-last) and the uint8 argmax in y's NHWC layout; see mmu_maxpool_fwd."""
    _dev_check(x, y, argmax)
    B, C, H, W = x.shape
    _maxpool_check(x, y, argmax, B, C, H, W, "x", "y")
    N.call("mmu_maxpool_fwd", _ptr(x), B, H, W, C, _ptr(y), _ptr(argmax), _stream(x))


def maxpool_bwd(dy, argmax, dx):
    _dev_check(dy, argmax, dx)
    B, C, H, W = dx.shape
    _maxpool_check(dx, dy, argmax, B, C, H, W, "dx", "dy")
    N.call("mmu_maxpool_bwd", _ptr(dy), _ptr(argmax), B, H, W, C, _ptr(dx), _stream(dx))


def _maxpool_check(full, pooled, argmax, B, C, H, W, nf, np_):
    """The kernels index raw NHWC pointers: refuse any layout / size they do not assume."""
    oshape = (B, C, (H - 1) // 2 + 1, (W - 1) // 2 + 1)
    for t, nm in ((full, nf), (pooled, np_)):
        _want(t, torch.bfloat16, f"maxpool {nm}")
        if t.dim() != 4 or not t.is_contiguous(memory_format=torch.channels_last):
            raise N.NativeError(f"maxpool: {nm} must be a channels-last [B, C, H, W] bf16 map")
    if tuple(pooled.shape) != oshape:
        raise N.NativeError(f"maxpool: {np_} is {tuple(pooled.shape)}, MaxPool2d(3, 2, 1) of "
                            f"{(B, C, H, W)} is {oshape}")
    if argmax.dtype != torch.uint8 or argmax.numel() != pooled.numel() or not argmax.is_contiguous():
        raise N.NativeError("maxpool: argmax must be a contiguous uint8 tensor with one entry per pooled element")


def row_pool_fwd(fmap_nhwc, n, out):
    _dev_check(fmap_nhwc, out)
    B, Hh, Ww, C = fmap_nhwc.shape
    N.call("mmu_row_pool_fwd", _ptr(fmap_nhwc), B, Hh, Ww, C, n, _ptr(out), _stream(out))


def row_pool_bwd(dout, n, dfmap_nhwc):
    _dev_check(dout, dfmap_nhwc)
    B, Hh, Ww, C = dfmap_nhwc.shape
    N.call("mmu_row_pool_bwd", _ptr(dout), B, Hh, Ww, C, n, _ptr(dfmap_nhwc), _stream(dout))


def _conv_out(h, w, ksize, stride):
    pad = ksize // 2
    return (h + 2 * pad - ksize) // stride + 1, (w + 2 * pad - ksize) // stride + 1


def conv_implicit(X, Wk, Y, ksize=3, stride=1, stats=None):
    """Y[p, n] = sum_{tap, c} X[input pixel of (p, tap), c] Wk[n, tap * C + c]: a ksize x ksize
    (3: pad 1, 1: pad 0) / stride conv as one implicit-im2col GEMM.  X [N, C, H, W] and Y
    [N, Nout, Ho, Wo] channels-last bf16, Wk bf16 with memory [Nout][ksize][ksize][C] (a
    channels-last [Nout, C, k, k] filter, or the flipped-transposed 3x3 one for dX).
    stats (optional, bn_stats_table of Y's rows): Y's BatchNorm statistics, written too."""
    _dev_check(X, Wk, Y)
    _want(X, torch.bfloat16, "conv_implicit X")
    _want(Wk, torch.bfloat16, "conv_implicit Wk")
    n, c, h, w = X.shape
    nout = Y.shape[1]
    ho, wo = _conv_out(h, w, ksize, stride)
    cl = torch.channels_last
    # the kernel reads Wk[n][tap * C + c]: either a [Nout, k, k, C] contiguous tensor or a
    # [Nout, C, k, k] filter whose memory is channels-last (both are [Nout][k][k][C] in memory)
    k = ksize
    wk_ok = Wk.dim() == 4 and (
        (tuple(Wk.shape) == (nout, k, k, c) and Wk.is_contiguous())
        or (tuple(Wk.shape) == (nout, c, k, k) and Wk.is_contiguous(memory_format=cl)))
    if (Y.shape != (n, nout, ho, wo) or Y.dtype != torch.bfloat16 or not wk_ok
            or not X.is_contiguous(memory_format=cl) or not Y.is_contiguous(memory_format=cl)):
        raise N.NativeError(f"conv_implicit: X channels-last bf16 [N, C, H, W], Y [N, Nout, {ho}, {wo}], "
                            f"Wk [Nout][{k}][{k}][C] bf16")
    ws = _splitk_workspace(Y.device)  # split-K slabs for small maps (few tiles)
    if stats is not None:
        if stats.dtype != torch.float32 or stats.numel() < ((n * ho * wo + 63) // 64) * nout * 2:
            raise N.NativeError("conv_implicit: stats table too small (kernels.bn_stats_table)")
        N.call("mmu_conv_implicit_stats", _ptr(X), _ptr(Wk), _ptr(Y), n, h, w, c, nout, ksize, stride, _ptr(stats),
               _ptr(ws), ws.numel(), _stream(X))
        return
    N.call("mmu_conv_implicit", _ptr(X), _ptr(Wk), _ptr(Y), n, h, w, c, nout, ksize, stride, _ptr(ws), ws.numel(),
           _stream(X))


def conv3x3_implicit(X, Wk, Y, bnb=None, table=None):
    """the 3x3 / stride-1 / pad-1 case of conv_implicit (Y and X share H, W).  bnb = (x, relu_mask,
    mean) with table (bn_stats_table of Y's rows): Y is the data gradient dY of that training
    BatchNorm, and the table receives its backward reduction (mmu_conv3x3_implicit_bnb)."""
    if bnb is None:
        conv_implicit(X, Wk, Y, 3, 1)
        return
    _dev_check(X, Wk, Y, table)
    x, mask, mean = bnb
    _bnb_check(x, mask, mean, "conv3x3_implicit bnb")
    n, c, h, w = X.shape
    nout = Y.shape[1]
    cl = torch.channels_last
    if (Y.shape != (n, nout, h, w) or x.shape != Y.shape or Y.dtype != torch.bfloat16 or X.dtype != torch.bfloat16
            or Wk.dtype != torch.bfloat16 or tuple(Wk.shape) != (nout, 3, 3, c) or not Wk.is_contiguous()
            or not X.is_contiguous(memory_format=cl) or not Y.is_contiguous(memory_format=cl)):
        raise N.NativeError("conv3x3_implicit bnb: X / Y / x channels-last bf16, Wk [Nout][3][3][C] bf16")
    if table.dtype != torch.float32 or table.numel() < ((n * h * w + 63) // 64) * nout * 2:
        raise N.NativeError("conv3x3_implicit bnb: table too small (kernels.bn_stats_table)")
    ws = _splitk_workspace(Y.device)
    N.call("mmu_conv3x3_implicit_bnb", _ptr(X), _ptr(Wk), _ptr(Y), n, h, w, c, nout, _ptr(x), _ptr(mask),
           _ptr(mean), _ptr(table), _ptr(ws), ws.numel(), _stream(X))


def _stem_check(X, what):
    if (X.dim() != 4 or X.dtype != torch.bfloat16 or X.shape[1] != 3
            or not X.is_contiguous(memory_format=torch.channels_last)):
        raise N.NativeError(f"{what}: X must be channels-last bf16 [N, 3, H, W] (got {tuple(X.shape)} {X.dtype})")


def stem_conv_fwd(X, Wk, Y):
    """Y = conv2d(X, Wk, stride 2, padding 3): the ResNet stem (7x7, 3 -> 64).  X [N, 3, H, W]
    and Y [N, 64, Ho, Wo] channels-last bf16; Wk bf16 [64, 3, 7, 7] channels-last (memory
    [64][7][7][3], the parameter store's filter copy)."""
    _dev_check(X, Wk, Y)
    _stem_check(X, "stem_conv_fwd")
    n, _, h, w = X.shape
    ho, wo = (h - 1) // 2 + 1, (w - 1) // 2 + 1
    if (tuple(Wk.shape) != (64, 3, 7, 7) or Wk.dtype != torch.bfloat16
            or not Wk.is_contiguous(memory_format=torch.channels_last)):
        raise N.NativeError("stem_conv_fwd: Wk must be channels-last bf16 [64, 3, 7, 7]")
    if (tuple(Y.shape) != (n, 64, ho, wo) or Y.dtype != torch.bfloat16
            or not Y.is_contiguous(memory_format=torch.channels_last)):
        raise N.NativeError(f"stem_conv_fwd: Y must be channels-last bf16 [{n}, 64, {ho}, {wo}]")
    N.call("mmu_stem_conv_fwd", _ptr(X), _ptr(Wk), _ptr(Y), n, h, w, _stream(X))


def stem_conv_wgrad(dY, X, dW, accumulate=False):
    """dW (+)= the stem conv's filter gradient: dY [N, 64, Ho, Wo] and X [N, 3, H, W]
    channels-last bf16, dW f32 [64, 3, 7, 7] channels-last."""
    _dev_check(dY, X, dW)
    _stem_check(X, "stem_conv_wgrad")
    n, _, h, w = X.shape
    ho, wo = (h - 1) // 2 + 1, (w - 1) // 2 + 1
    if (tuple(dY.shape) != (n, 64, ho, wo) or dY.dtype != torch.bfloat16
            or not dY.is_contiguous(memory_format=torch.channels_last)):
        raise N.NativeError(f"stem_conv_wgrad: dY must be channels-last bf16 [{n}, 64, {ho}, {wo}]")
    if (tuple(dW.shape) != (64, 3, 7, 7) or dW.dtype != torch.float32
            or not dW.is_contiguous(memory_format=torch.channels_last)):
        raise N.NativeError("stem_conv_wgrad: dW must be channels-last f32 [64, 3, 7, 7]")
    need = N.load().mmu_stem_conv_wgrad_ws_floats(n, h, w)
    ws = _splitk_workspace(X.device)
    if need < 0 or ws.numel() < need:
        raise N.NativeError(f"stem_conv_wgrad: workspace of {ws.numel()} floats, needs {need}")
    N.call("mmu_stem_conv_wgrad", _ptr(dY), _ptr(X), _ptr(dW), n, h, w, int(bool(accumulate)), _ptr(ws), ws.numel(),
           _stream(X))


def conv_wgrad(dY, X, dW, ksize=3, stride=1, accumulate=False):
    """dW (+)= weight gradient of a ksize x ksize (3: pad 1, 1: pad 0) / stride conv: X [N, Cin,
    H, W] and dY [N, Cout, Ho, Wo] channels-last bf16, dW f32 [Cout, Cin, k, k] channels-last
    (memory [Cout][k][k][Cin]).  Cin % 256 == 0, Cout % 128 == 0."""
    _dev_check(dY, X, dW)
    _want(X, torch.bfloat16, "conv_wgrad X")
    _want(dY, torch.bfloat16, "conv_wgrad dY")
    n, cin, h, w = X.shape
    cout = dY.shape[1]
    ho, wo = _conv_out(h, w, ksize, stride)
    cl = torch.channels_last
    if (dY.shape != (n, cout, ho, wo) or dW.shape != (cout, cin, ksize, ksize) or dW.dtype != torch.float32
            or not X.is_contiguous(memory_format=cl) or not dY.is_contiguous(memory_format=cl)
            or not dW.is_contiguous(memory_format=cl)):
        raise N.NativeError(f"conv_wgrad: X channels-last bf16 [N, C, H, W], dY [N, Cout, {ho}, {wo}], "
                            f"dW f32 channels-last [Cout, Cin, {ksize}, {ksize}]")
    ws = _splitk_workspace(X.device)
    N.call("mmu_conv_wgrad", _ptr(dY), _ptr(X), _ptr(dW), n, h, w, cin, cout, ksize, stride, int(bool(accumulate)),
           _ptr(ws), ws.numel(), _stream(X))


def conv3x3_wgrad(dY, X, dW, accumulate=False):
    """the 3x3 / stride-1 / pad-1 case of conv_wgrad"""
    conv_wgrad(dY, X, dW, 3, 1, accumulate)


_bn_ws = {}


def _bn_workspace(dev):
    """per-device scratch for mmu_batchnorm_*, reused stream-ordered by every call"""
    t = _bn_ws.get(dev)
    if t is None:
        nbytes = N.load().mmu_batchnorm_ws_bytes(2048)
        t = _bn_ws[dev] = torch.empty((nbytes + 3) // 4, dtype=torch.float32, device=dev)
    return t


def _bn_mask_check(mask, X, what):
    if mask is None:
        return
    C = X.shape[1]
    if mask.dtype != torch.uint8 or not mask.is_contiguous() or mask.numel() != X.numel() // 8 or C % 8:
        raise N.NativeError(f"{what}: relu_mask must be contiguous uint8 with numel = X.numel() / 8 "
                            f"(got {tuple(mask.shape)} {mask.dtype} for X {tuple(X.shape)})")
    _dev_check(mask, X)


def _bn_vec_check(name, C, *ts):
    """per-channel BatchNorm vectors must be f32 (the kernels read / write them as float[C]: a
    bf16 running_mean -- e.g. after module.to(bfloat16) -- would be written past its end).
    Only the dtype is checked per call (cheap: this runs ~300 times per train step)."""
    for t in ts:
        if t is not None and t.dtype != torch.float32:
            raise N.NativeError(f"{name}: per-channel tensors must be f32 (got {t.dtype} {tuple(t.shape)})")


def _bn_map_check(name, X, *ts):
    for t in ts:
        if t is not None and t.dtype != torch.bfloat16:
            raise N.NativeError(f"{name}: maps must be bf16 (got {t.dtype} {tuple(t.shape)})")


def _bn_res_check(name, X, *ts):
    for t in ts:
        if t is not None and (t.dtype != torch.int8 or t.numel() != X.numel() or not t.is_contiguous()):
            raise N.NativeError(f"{name}: a stream residue must be a contiguous int8 tensor of X's size")


def batchnorm_fwd(X, Y, weight, bias, running_mean, running_var, training, momentum, eps, relu=False, skip=None,
                  num_batches_tracked=None, save_mean=None, save_invstd=None, relu_mask=None, skip_res=None,
                  y_res=None, parts=None):
    """X, Y, skip: channels-last bf16 [N, C, H, W] (contiguous as [N*H*W, C]).  relu_mask
    (optional, relu only): uint8 [N*H*W*C/8] written with the bits Y > 0 for batchnorm_bwd.
    y_res / skip_res (optional, int8 of X's size): the residual stream's 8-bit residue of Y /
    of skip (include/mmu.h).  parts (training only): (table, nparts) of X's statistics from the
    conv that produced X (bn_stats_table): no statistics pass (mmu_batchnorm_fwd_parts)."""
    _dev_check(X, Y)
    _want(X, torch.bfloat16, "batchnorm X")
    _bn_mask_check(relu_mask, X, "batchnorm_fwd")
    C = X.shape[1]
    _bn_vec_check("batchnorm_fwd", C, weight, bias, running_mean, running_var, save_mean, save_invstd)
    _bn_map_check("batchnorm_fwd", X, Y, skip)
    _bn_res_check("batchnorm_fwd", X, skip_res, y_res)
    if num_batches_tracked is not None and num_batches_tracked.dtype != torch.int64:
        raise N.NativeError("batchnorm_fwd: num_batches_tracked must be int64")
    rows = X.numel() // C
    ws = _bn_workspace(X.device)
    if parts is not None:
        table, nparts = parts
        if not training or table.numel() < nparts * C * 2 or nparts != (rows + 63) // 64:
            raise N.NativeError("batchnorm_fwd: parts must be X's training statistics table (bn_stats_table)")
        N.call("mmu_batchnorm_fwd_parts", _ptr(X), _ptr(skip), _ptr(Y), rows, C, _ptr(table), nparts, _ptr(weight),
               _ptr(bias), _ptr(running_mean), _ptr(running_var), _ptr(num_batches_tracked), float(momentum),
               float(eps), int(bool(relu)), _ptr(save_mean), _ptr(save_invstd), _ptr(relu_mask), _ptr(skip_res),
               _ptr(y_res), _ptr(ws), ws.numel() * 4, _stream(X))
        return
    N.call("mmu_batchnorm_fwd", _ptr(X), _ptr(skip), _ptr(Y), rows, C, _ptr(weight), _ptr(bias), _ptr(running_mean),
           _ptr(running_var), _ptr(num_batches_tracked), int(bool(training)), float(momentum), float(eps),
           int(bool(relu)), _ptr(save_mean), _ptr(save_invstd), _ptr(relu_mask), _ptr(skip_res), _ptr(y_res),
           _ptr(ws), ws.numel() * 4, _stream(X))


def batchnorm_bwd(dY, Y, X, weight, save_mean, save_invstd, relu, dX, dSkip=None, dweight=None, dbias=None,
                  relu_mask=None, parts=None):
    """relu: g = dY * [Y > 0] from relu_mask (batchnorm_fwd's) when given, else from Y.  parts:
    (table, nparts) of the reduction the product that formed dY wrote (STORE_BNB / ADD_RES_BNB,
    conv3x3_implicit bnb): no reduction pass (mmu_batchnorm_bwd_parts)."""
    _dev_check(dY, X, dX)
    _want(X, torch.bfloat16, "batchnorm_bwd X")
    _bn_mask_check(relu_mask, X, "batchnorm_bwd")
    C = X.shape[1]
    _bn_vec_check("batchnorm_bwd", C, weight, save_mean, save_invstd, dweight, dbias)
    _bn_map_check("batchnorm_bwd", X, dY, Y, dX, dSkip)
    rows = X.numel() // C
    ws = _bn_workspace(X.device)
    if parts is not None:
        table, nparts = parts
        if table.numel() < nparts * C * 2 or nparts != (rows + 63) // 64:
            raise N.NativeError("batchnorm_bwd: parts must be dY's reduction table (bn_stats_table)")
        N.call("mmu_batchnorm_bwd_parts", _ptr(dY), _ptr(Y), _ptr(relu_mask), _ptr(X), rows, C, _ptr(table), nparts,
               _ptr(weight), _ptr(save_mean), _ptr(save_invstd), int(bool(relu)), _ptr(dX), _ptr(dSkip),
               _ptr(dweight), _ptr(dbias), _ptr(ws), ws.numel() * 4, _stream(X))
        return
    N.call("mmu_batchnorm_bwd", _ptr(dY), _ptr(Y), _ptr(relu_mask), _ptr(X), rows, C, _ptr(weight), _ptr(save_mean),
           _ptr(save_invstd), int(bool(relu)), _ptr(dX), _ptr(dSkip), _ptr(dweight), _ptr(dbias), _ptr(ws),
           ws.numel() * 4, _stream(X))


def bn_sums_buffer(C, device):
    """[2C+1] f64: the per-channel sums of one cross-rank BatchNorm pass + its row count"""
    return torch.empty(2 * C + 1, dtype=torch.float64, device=device)


def batchnorm_stats(X, sums):
    """cross-rank BatchNorm, forward first half: sums = {sum x, sum x^2, rows} over X's rows"""
    _dev_check(X, sums)
    _want(X, torch.bfloat16, "batchnorm_stats X")
    C = X.shape[1]
    _bn_sums_check("batchnorm_stats", sums, C)
    _bn_map_check("batchnorm_stats", X)
    ws = _bn_workspace(X.device)
    N.call("mmu_batchnorm_stats", _ptr(X), X.numel() // C, C, _ptr(sums), _ptr(ws), ws.numel() * 4, _stream(X))


def batchnorm_fwd_sums(X, Y, sums, weight, bias, running_mean, running_var, momentum, eps, relu=False, skip=None,
                       num_batches_tracked=None, save_mean=None, save_invstd=None, relu_mask=None, skip_res=None,
                       y_res=None):
    """cross-rank BatchNorm, forward second half: batchnorm_fwd (training) with the statistics
    of the exchanged sums"""
    _dev_check(X, Y, sums)
    _want(X, torch.bfloat16, "batchnorm X")
    _bn_mask_check(relu_mask, X, "batchnorm_fwd_sums")
    C = X.shape[1]
    _bn_sums_check("batchnorm_fwd_sums", sums, C)
    _bn_vec_check("batchnorm_fwd_sums", C, weight, bias, running_mean, running_var, save_mean, save_invstd)
    _bn_map_check("batchnorm_fwd_sums", X, Y, skip)
    _bn_res_check("batchnorm_fwd_sums", X, skip_res, y_res)
    if num_batches_tracked is not None and num_batches_tracked.dtype != torch.int64:
        raise N.NativeError("batchnorm_fwd_sums: num_batches_tracked must be int64")
    ws = _bn_workspace(X.device)
    N.call("mmu_batchnorm_fwd_sums", _ptr(X), _ptr(skip), _ptr(Y), X.numel() // C, C, _ptr(sums), _ptr(weight),
           _ptr(bias), _ptr(running_mean), _ptr(running_var), _ptr(num_batches_tracked), float(momentum), float(eps),
           int(bool(relu)), _ptr(save_mean), _ptr(save_invstd), _ptr(relu_mask), _ptr(skip_res), _ptr(y_res),
           _ptr(ws), ws.numel() * 4, _stream(X))


def batchnorm_bwd_reduce(dY, Y, X, save_mean, save_invstd, relu, sums, dweight=None, dbias=None, relu_mask=None):
    """cross-rank BatchNorm, backward first half: sums = {sum g, sum g*(x-mean), rows};
    dweight / dbias += this rank's"""
    _dev_check(dY, X, sums)
    _want(X, torch.bfloat16, "batchnorm_bwd X")
    _bn_mask_check(relu_mask, X, "batchnorm_bwd_reduce")
    C = X.shape[1]
    _bn_sums_check("batchnorm_bwd_reduce", sums, C)
    _bn_vec_check("batchnorm_bwd_reduce", C, save_mean, save_invstd, dweight, dbias)
    _bn_map_check("batchnorm_bwd_reduce", X, dY, Y)
    ws = _bn_workspace(X.device)
    N.call("mmu_batchnorm_bwd_reduce", _ptr(dY), _ptr(Y), _ptr(relu_mask), _ptr(X), X.numel() // C, C,
           _ptr(save_mean), _ptr(save_invstd), int(bool(relu)), _ptr(sums), _ptr(dweight), _ptr(dbias), _ptr(ws),
           ws.numel() * 4, _stream(X))


def batchnorm_bwd_sums(dY, Y, X, sums, weight, save_mean, save_invstd, relu, dX, dSkip=None, relu_mask=None):
    """cross-rank BatchNorm, backward second half: dX (, dSkip) from the exchanged sums"""
    _dev_check(dY, X, dX, sums)
    _want(X, torch.bfloat16, "batchnorm_bwd X")
    _bn_mask_check(relu_mask, X, "batchnorm_bwd_sums")
    C = X.shape[1]
    _bn_sums_check("batchnorm_bwd_sums", sums, C)
    _bn_vec_check("batchnorm_bwd_sums", C, weight, save_mean, save_invstd)
    _bn_map_check("batchnorm_bwd_sums", X, dY, Y, dX, dSkip)
    ws = _bn_workspace(X.device)
    N.call("mmu_batchnorm_bwd_sums", _ptr(dY), _ptr(Y), _ptr(relu_mask), _ptr(X), X.numel() // C, C, _ptr(sums),
           _ptr(weight), _ptr(save_mean), _ptr(save_invstd), int(bool(relu)), _ptr(dX), _ptr(dSkip), _ptr(ws),
           ws.numel() * 4, _stream(X))


def _bn_sums_check(who, sums, C):
    if sums.dtype != torch.float64 or sums.numel() != 2 * C + 1 or not sums.is_contiguous():
        raise N.NativeError(f"{who}: sums must be a contiguous float64 [2C+1] = [{2 * C + 1}] tensor")


def bertadam_step(params, grads, m, v, bf16_copy, table, steps, n_tensors, n_chunks, lr_decay, lr_nodecay, wd,
                  warmup, t_total, b1, b2, eps, max_grad_norm, ws, grad_scale=1.0):
    _dev_check(params, grads, m, v, table, steps, ws)
    N.call("mmu_bertadam_step", _ptr(params), _ptr(grads), _ptr(m), _ptr(v), _ptr(bf16_copy), _ptr(table),
           _ptr(steps), n_tensors, n_chunks, float(lr_decay), float(lr_nodecay), float(wd), float(warmup),
           float(t_total), float(b1), float(b2), float(eps), float(max_grad_norm), float(grad_scale), _ptr(ws),
           ws.numel(), _stream(params))


def uncertainty(logits, y, p_bar, nll, conf, correct):
    _dev_check(logits, y, p_bar, nll, conf, correct)
    S, R, C = logits.shape
    N.call("mmu_uncertainty", _ptr(logits), _ptr(y), S, R, C, _ptr(p_bar), _ptr(nll), _ptr(conf), _ptr(correct),
           _stream(logits))


def ece_bins(conf, correct, n_bins, out):
    _dev_check(conf, correct, out)
    N.call("mmu_ece_bins", _ptr(conf), _ptr(correct), conf.numel(), n_bins, _ptr(out), _stream(conf))


_alg = {"on": False, "bytes": 0.0, "n": 0}


_seed_counter = None


def set_seed_offset(counter):
    """Dropout seeds under HIP-graph replay (include/mmu.h mmu_set_seed_offset): ``counter`` = a
    1-element int64 device tensor every later dropout launch folds into its seed when it runs
    (None = off).  The tensor is kept referenced here while it is set."""
    global _seed_counter
    if counter is not None:
        _want(counter, torch.int64, "seed counter")
        if counter.numel() != 1 or not counter.is_cuda:
            raise N.NativeError("seed counter: a 1-element int64 CUDA tensor")
    _seed_counter = counter
    N.call("mmu_set_seed_offset", _ptr(counter) if counter is not None else None)


def timing_enable(on=True):
    """HIP-event timing of every mmu_gemm launch (and a count of its algorithmic bytes)."""
    N.call("mmu_timing_enable", int(on))
    _alg.update(on=bool(on), bytes=0.0, n=0)


class timing_paused:
    """Context: mmu_gemm launches inside are neither event-timed nor counted (bench.py's
    GEMM roofline covers the BERT-layer products only)."""

    def __enter__(self):
        self.was = _alg["on"]
        if self.was:
            N.call("mmu_timing_pause", 1)
            _alg["on"] = False
        return self

    def __exit__(self, *exc):
        if self.was:
            N.call("mmu_timing_pause", 0)
            _alg["on"] = True
        return False


def timing_read():
    ms, n, fl = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double()
    N.call("mmu_timing_read", ctypes.byref(ms), ctypes.byref(n), ctypes.byref(fl))
    return ms.value, n.value, fl.value


def timing_alg_bytes():
    """(algorithmic HBM bytes, launches) of the timed GEMMs: operands read once, C written
    once (read too when accumulating), residual / aux streams of the fused epilogues."""
    return _alg["bytes"], _alg["n"]


def _count_alg(M, N_, K, batch, c_bytes, epi):
    b = 2.0 * (M * K + N_ * K) + c_bytes * M * N_
    if epi is not None:
        if epi.accumulate:
            b += c_bytes * M * N_
        if epi.residual:  # f32 residual with an f32 BIAS_DROP_RES output (the hidden stream)
            b += (4.0 if (c_bytes == 4 and epi.kind == EPI_BIAS_DROP_RES) else 2.0) * M * N_
        if epi.aux:
            b += 2.0 * M * N_
    _alg["bytes"] += b * batch
    _alg["n"] += 1
