"""Kernel-level parity of the HIP path against plain PyTorch fp32 on the same inputs.

Tolerances: bf16 inputs with fp32 accumulation; outputs compared at bf16
resolution (rel 1e-2 of the output scale) unless stated.
"""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def K():
    from src import kernels
    return kernels


def rnd(*shape, dev, scale=1.0, dtype=torch.bfloat16, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(dev).to(dtype)


def close(a, b, rtol=1e-2, atol_frac=1e-2):
    a, b = a.float(), b.float()
    scale = b.abs().max().item() + 1e-6
    err = (a - b).abs().max().item()
    assert err <= atol_frac * scale + rtol * 0, f"max err {err:.3e} vs scale {scale:.3e}"


def op(t, kmajor, rows, K_):
    """logical [rows, K] operand from a stored tensor (K-major: [rows,K]; else [K,rows])"""
    return t.float() if kmajor else t.float().t()


@pytest.mark.parametrize("ak,bk", [(True, True), (True, False), (False, False), (False, True)])
@pytest.mark.parametrize("M,N,Kd", [(256, 128, 64), (384, 256, 192)])
def test_gemm_layouts(dev, ak, bk, M, N, Kd):
    k = K()
    A = rnd(M, Kd, dev=dev, seed=1) if ak else rnd(Kd, M, dev=dev, seed=1)
    B = rnd(N, Kd, dev=dev, seed=2) if bk else rnd(Kd, N, dev=dev, seed=2)
    C = torch.empty(M, N, dtype=torch.float32, device=dev)
    k.gemm(A, A.shape[1], ak, B, B.shape[1], bk, C, N, M, N, Kd)
    ref = op(A, ak, M, Kd) @ op(B, bk, N, Kd).t()
    torch.testing.assert_close(C, ref, rtol=1e-4, atol=1e-3)


def test_gemm_m_tail_bias_bf16(dev):
    k = K()
    M, N, Kd = 200, 256, 128
    A, B = rnd(M, Kd, dev=dev, seed=3), rnd(N, Kd, dev=dev, seed=4)
    bias = torch.randn(N, device=dev)
    C = torch.full((M + 8, N), 7.0, dtype=torch.bfloat16, device=dev)
    k.gemm(A, Kd, True, B, Kd, True, C, N, M, N, Kd, epi=k.epilogue(k.EPI_STORE, bias=bias))
    ref = A.float() @ B.float().t() + bias
    close(C[:M], ref)
    assert (C[M:] == 7.0).all(), "rows beyond M were written"


def test_gemm_k_tail_weight_grad(dev):
    k = K()
    Ktok, M, N = 1000, 256, 384  # dW = dY^T X over a token count that is not a tile multiple
    dY, X = rnd(Ktok, M, dev=dev, seed=5), rnd(Ktok, N, dev=dev, seed=6)
    C = torch.ones(M, N, dtype=torch.float32, device=dev)
    k.gemm(dY, M, False, X, N, False, C, N, M, N, Ktok, epi=k.epilogue(k.EPI_STORE, accumulate=True))
    ref = dY.float().t() @ X.float() + 1.0
    torch.testing.assert_close(C, ref, rtol=1e-4, atol=2e-3)


@pytest.mark.parametrize("accumulate", [True, False])
def test_gemm_splitk_weight_grad(dev, accumulate):
    """long-K / few-tile product takes the split-K path (slabs + ordered reduce): same result, deterministic."""
    k = K()
    Ktok, M, N = 20000, 256, 128
    dY, X = rnd(Ktok, M, dev=dev, seed=31), rnd(Ktok, N, dev=dev, seed=32)
    C = torch.full((M, N), 0.5, dtype=torch.float32, device=dev)
    k.gemm(dY, M, False, X, N, False, C, N, M, N, Ktok, epi=k.epilogue(k.EPI_STORE, accumulate=accumulate))
    ref = dY.float().t() @ X.float() + (0.5 if accumulate else 0.0)
    torch.testing.assert_close(C, ref, rtol=1e-4, atol=1e-2)
    C2 = torch.full((M, N), 0.5, dtype=torch.float32, device=dev)
    k.gemm(dY, M, False, X, N, False, C2, N, M, N, Ktok, epi=k.epilogue(k.EPI_STORE, accumulate=accumulate))
    assert torch.equal(C, C2)


def test_gemm_gelu_dgelu_colsum(dev):
    k = K()
    M, N, Kd = 300, 256, 128
    A, B = rnd(M, Kd, dev=dev, seed=7), rnd(N, Kd, dev=dev, seed=8, scale=0.2)
    bias = torch.randn(N, device=dev) * 0.5
    Z = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    Hh = torch.empty_like(Z)
    k.gemm(A, Kd, True, B, Kd, True, Hh, N, M, N, Kd, epi=k.epilogue(k.EPI_BIAS_GELU, bias=bias, aux=Z))
    z = (A.float() @ B.float().t() + bias).requires_grad_(True)
    gz = torch.nn.functional.gelu(z)  # erf form
    (dgz,) = torch.autograd.grad(gz.sum(), z)
    close(Hh, gz.detach())
    close(Z, dgz)  # aux = gelu'(z)
    # dgelu with column sums: C = acc * aux
    G = rnd(M, Kd, dev=dev, seed=9)
    W = rnd(Kd, N, dev=dev, seed=10, scale=0.2)  # stored [K][N] -> MN-major B
    out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    cs = torch.full((N,), 1.0, device=dev)  # the epilogue ADDS its column sums (bias-grad accumulation)
    k.gemm(G, Kd, True, W, N, False, out, N, M, N, Kd, epi=k.epilogue(k.EPI_DGELU, aux=Z, colsum=cs))
    g = (G.float() @ W.float()) * dgz
    close(out, g)
    torch.testing.assert_close(cs, g.sum(0) + 1.0, rtol=2e-2, atol=2e-2 * g.abs().sum(0).max().item() / 50)


@pytest.mark.parametrize("ak,bk", [(True, True), (True, False), (False, False), (False, True)])
@pytest.mark.parametrize("M,N,Kd", [(512, 256, 128), (700, 768, 192), (1024, 384, 4096)])
def test_gemm_big_tiles(dev, ak, bk, M, N, Kd):
    """256x256 LDS-DMA tiling (M, N >= 256): all layouts, ragged M/N tails, deep K."""
    k = K()
    if not ak and M % 128:
        pytest.skip("M-major A needs M % 128 == 0")
    A = rnd(M, Kd, dev=dev, seed=41) if ak else rnd(Kd, M, dev=dev, seed=41)
    B = rnd(N, Kd, dev=dev, seed=42) if bk else rnd(Kd, N, dev=dev, seed=42)
    C = torch.full((M, N), 3.0, dtype=torch.float32, device=dev)
    k.gemm(A, A.shape[1], ak, B, B.shape[1], bk, C, N, M, N, Kd, epi=k.epilogue(k.EPI_STORE, accumulate=True))
    ref = op(A, ak, M, Kd) @ op(B, bk, N, Kd).t() + 3.0
    torch.testing.assert_close(C, ref, rtol=1e-4, atol=5e-3)


def test_gemm_big_tiles_epilogues(dev):
    k = K()
    M, N, Kd = 777, 768, 256
    A, B = rnd(M, Kd, dev=dev, seed=51), rnd(N, Kd, dev=dev, seed=52, scale=0.1)
    bias = torch.randn(N, device=dev) * 0.1
    R = rnd(M, N, dev=dev, seed=53)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    k.gemm(A, Kd, True, B, Kd, True, out, N, M, N, Kd, epi=k.epilogue(k.EPI_BIAS_DROP_RES, bias=bias, residual=R))
    close(out, R.float() + A.float() @ B.float().t() + bias)
    Z = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    k.gemm(A, Kd, True, B, Kd, True, out, N, M, N, Kd, epi=k.epilogue(k.EPI_BIAS_GELU, bias=bias, aux=Z))
    z = (A.float() @ B.float().t() + bias).requires_grad_(True)
    gz = torch.nn.functional.gelu(z)
    close(out, gz.detach())
    close(Z, torch.autograd.grad(gz.sum(), z)[0])
    out2 = torch.empty_like(out)  # aux is optional (inference)
    k.gemm(A, Kd, True, B, Kd, True, out2, N, M, N, Kd, epi=k.epilogue(k.EPI_BIAS_GELU, bias=bias))
    assert torch.equal(out, out2)


def test_transpose_bf16_batched(dev):
    """mmu_transpose_bf16_batched: several jobs of different (ragged) shapes in one launch,
    bit-exact against torch's transpose; bytes outside each destination untouched."""
    k = K()
    shapes = [(2304, 768), (768, 3072), (100, 70), (65, 129), (1, 8)]
    srcs = [rnd(r, c, dev=dev, seed=70 + i) for i, (r, c) in enumerate(shapes)]
    dsts = [torch.full((c + 1, r), 5.0, dtype=torch.bfloat16, device=dev) for r, c in shapes]  # +1 guard row
    jobs = torch.tensor([[s_.data_ptr(), d.data_ptr(), r, c, 0, 0] for s_, d, (r, c) in zip(srcs, dsts, shapes)],
                        dtype=torch.int64).to(dev)
    k.transpose_bf16_batched(jobs, len(shapes), max(r for r, _ in shapes), max(c for _, c in shapes), srcs[0])
    for s_, d, (r, c) in zip(srcs, dsts, shapes):
        assert torch.equal(d[:c], s_.t()), (r, c)
        assert (d[c:] == 5.0).all(), "wrote past the destination"


def test_transpose_bf16_strided_flipped_filter(dev):
    """strided jobs (row pitches): the 9 per-tap jobs the parameter store uses for the flipped
    [Cin][3][3][Cout] copy of a channels-last 3x3 filter, bit-exact vs flip + permute."""
    k = K()
    O, I = 384, 256
    w = rnd(O, I, 3, 3, dev=dev, seed=3).contiguous(memory_format=torch.channels_last)
    dst = torch.full((I, 3, 3, O), 7.0, dtype=torch.bfloat16, device=dev)
    rows = [[w.data_ptr() + 2 * t * I, dst.data_ptr() + 2 * (8 - t) * O, O, I, 9 * I, 9 * O] for t in range(9)]
    jobs = torch.tensor(rows, dtype=torch.int64).to(dev)
    k.transpose_bf16_batched(jobs, 9, O, I, w)
    assert torch.equal(dst, w.flip(2, 3).permute(1, 2, 3, 0))


@pytest.mark.parametrize("Kd", [256, 768])
def test_gemm_partial_last_wave(dev, Kd):
    """M = 256 * 257 rows x 3 column tiles = 771 tiles (a partial last wave of 3 tiles on 256
    CUs, the N = 768 BERT products' shape class): every epilogue against torch on the last
    tile row, the dropout quads of BIAS_DROP_RES recovered from a zero residual."""
    k = K()
    M, N = 256 * 257, 768
    A, B = rnd(M, Kd, dev=dev, seed=61), rnd(N, Kd, dev=dev, seed=62, scale=0.1)
    bias = torch.randn(N, device=dev) * 0.1
    R = rnd(M, N, dev=dev, seed=63)
    Zr = torch.zeros(M, N, dtype=torch.bfloat16, device=dev)
    aux = (torch.rand(M, N, device=dev) + 0.5).to(torch.bfloat16)
    ref = A.float() @ B.float().t()
    tl = slice(M - 256, M)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    k.gemm(A, Kd, True, B, Kd, True, out, N, M, N, Kd,
           epi=k.epilogue(k.EPI_BIAS_DROP_RES, bias=bias * 0, residual=Zr, drop_p=0.1, seed=77))
    kept = out.float()[tl] != 0
    frac = kept.float().mean().item()
    assert 0.88 < frac < 0.92, frac
    close(out.float()[tl][kept], (ref[tl] / 0.9)[kept])
    for kind, kw, want in ((k.EPI_STORE, {"bias": bias}, ref + bias), (k.EPI_DGELU, {"aux": aux}, ref * aux.float()),
                           (k.EPI_ADD_RES, {"residual": R}, ref + R.float())):
        cs = torch.zeros(N, device=dev)
        out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        k.gemm(A, Kd, True, B, Kd, True, out, N, M, N, Kd, epi=k.epilogue(kind, colsum=cs, **kw))
        close(out.float()[tl], want[tl])
        torch.testing.assert_close(cs, want.sum(0), rtol=2e-2, atol=2e-2 * want.abs().sum(0).max().item() / 100)
    f = torch.full((M, N), 0.25, dtype=torch.float32, device=dev)
    k.gemm(A, Kd, True, B, Kd, True, f, N, M, N, Kd, epi=k.epilogue(k.EPI_STORE, accumulate=True))
    close(f[tl], ref[tl] + 0.25)


def _keep_np(seed, idx, p):
    """numpy restatement of mmu_keep4 / mmu_keep1 (csrc/mmu_common.h): the keep decision of
    element idx of a dropout stream"""
    import numpy as np
    M32 = np.uint64(0xFFFFFFFF)

    def lb(x):
        x = x.astype(np.uint64) & M32
        x ^= x >> np.uint64(16)
        x = (x * np.uint64(0x7FEB352D)) & M32
        x ^= x >> np.uint64(15)
        x = (x * np.uint64(0x846CA68B)) & M32
        x ^= x >> np.uint64(16)
        return x
    s32 = lb(np.uint64(seed & 0xFFFFFFFF) ^ lb(np.uint64((seed >> 32) ^ 0x68BC21EB)))
    idx = np.asarray(idx, dtype=np.uint64)
    quad = idx >> np.uint64(2)
    x = (((quad << np.uint64(1)) & M32) ^ (((quad >> np.uint64(31)) * np.uint64(0x9E3779B8)) & M32)) ^ s32
    h0, h1 = lb(x), lb(x ^ np.uint64(1))
    e = idx & np.uint64(3)
    draw = np.where(e == 0, h0 & np.uint64(0xFFFF), np.where(e == 1, h0 >> np.uint64(16),
                    np.where(e == 2, h1 & np.uint64(0xFFFF), h1 >> np.uint64(16))))
    return draw >= np.uint64(int(p * 65536.0 + 0.5))


@pytest.mark.parametrize("M,N", [(256 * 257, 768), (256 * 64 + 32, 3072)])
def test_gemm_epilogues_exact_first_and_last_tile_rows(dev, M, N):
    """M = 256 * 257 rows x 3 column tiles = 771 tiles (3 whole rounds of 256 CUs + a partial
    one), the epilogues' row addressing (per-lane row bases + wave-uniform row offsets) checked
    on the first and the last tile row against torch: the f32 hidden-stream epilogue with the
    residual LayerNorm recomputed and dropout -- keep decisions equal to a numpy restatement
    of mmu_keep4 at the element's global index --, GELU + gelu' aux, and FLAVA's dropout +
    QuickGELU with its derivative aux.  M = 16416, N = 3072 is batch 32's FFN1 shape (its
    last tile row holds 32 live rows); the bias-gradient column sums of the dGELU product and
    a bf16 residual add are checked over all rows."""
    import numpy as np
    k = K()
    Kd = 768
    A, B = rnd(M, Kd, dev=dev, seed=131), rnd(N, Kd, dev=dev, seed=132, scale=0.1)
    bias = torch.randn(N, device=dev) * 0.1
    y = A.float() @ B.float().t() + bias
    rows = [slice(0, 256), slice(M - 256, M)]
    idx = {r.start: (np.arange(r.start, r.stop)[:, None] * N + np.arange(N)[None, :]) for r in rows}
    # f32 hidden stream: C = LN(S) + dropout(A B^T + b)
    S = torch.randn(M, N, device=dev) * 2.0 + 0.7
    mean = S.mean(-1).contiguous()
    rstd = torch.rsqrt(S.var(-1, unbiased=False) + 1e-12).contiguous()
    w, b = torch.randn(N, device=dev), torch.randn(N, device=dev)
    R32 = (S - mean[:, None]) * rstd[:, None] * w + b
    p, seed = 0.1, 4242
    out = torch.empty(M, N, dtype=torch.float32, device=dev)
    k.gemm(A, Kd, True, B, Kd, True, out, N, M, N, Kd,
           epi=k.epilogue(k.EPI_BIAS_DROP_RES, bias=bias, residual=S, drop_p=p, seed=seed, res_ln=(mean, rstd, w, b)))
    for r in rows:
        keep = torch.from_numpy(_keep_np(seed, idx[r.start], p)).to(dev)
        want = R32[r] + torch.where(keep, y[r] / (1 - p), torch.zeros_like(y[r]))
        torch.testing.assert_close(out[r], want, rtol=1e-5, atol=3e-5 * (R32.abs().max() + y.abs().max()).item())
    # GELU + derivative aux
    Z = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    H = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    k.gemm(A, Kd, True, B, Kd, True, H, N, M, N, Kd, epi=k.epilogue(k.EPI_BIAS_GELU, bias=bias, aux=Z))
    for r in rows:
        z = y[r].clone().requires_grad_(True)
        g = torch.nn.functional.gelu(z)
        close(H[r], g.detach())
        close(Z[r], torch.autograd.grad(g.sum(), z)[0])
    # FLAVA: u = dropout(z), C = u * sigmoid(1.702 u), aux = keep * scale * d/du
    k.gemm(A, Kd, True, B, Kd, True, H, N, M, N, Kd,
           epi=k.epilogue(k.EPI_BIAS_DROP_QGELU, bias=bias, aux=Z, drop_p=p, seed=seed + 1))
    for r in rows:
        keep = torch.from_numpy(_keep_np(seed + 1, idx[r.start], p)).to(dev).float()
        u = y[r] * keep / (1 - p)
        sg = torch.sigmoid(1.702 * u)
        close(H[r], u * sg)
        close(Z[r], keep / (1 - p) * (sg + 1.702 * u * sg * (1 - sg)))
    # dGELU (aux = the forward's gelu') + bias-gradient column sums over every row; bf16 residual add
    Zin = rnd(M, N, dev=dev, seed=133)
    cs = torch.zeros(N, device=dev)
    k.gemm(A, Kd, True, B, Kd, True, H, N, M, N, Kd, epi=k.epilogue(k.EPI_DGELU, aux=Zin, colsum=cs))
    dg = (y - bias) * Zin.float()
    close(H, dg)
    torch.testing.assert_close(cs, dg.sum(0), rtol=2e-3, atol=2e-3 * dg.abs().sum(0).max().item())
    R16 = rnd(M, N, dev=dev, seed=134)
    k.gemm(A, Kd, True, B, Kd, True, H, N, M, N, Kd, epi=k.epilogue(k.EPI_ADD_RES, residual=R16))
    close(H, y - bias + R16.float())


@pytest.mark.parametrize("ak,bk", [(True, True), (True, False), (False, False), (False, True)])
def test_gemm_many_tiles_every_element(dev, ak, bk):
    """More tiles than CUs (40 x 9 = 360 tiles; batch 2 x 20 x 9 = 360 items), a ragged last
    wave, checked on EVERY element (not just the last tile row) for a bf16 epilogue and for
    f32 accumulate, in every operand layout."""
    k = K()
    M, N, Kd = 256 * 40 - 96, 2304, 320
    Ma = M if ak else 256 * 40
    A = rnd(Ma, Kd, dev=dev, seed=81) if ak else rnd(Kd, Ma, dev=dev, seed=81)
    B = rnd(N, Kd, dev=dev, seed=82, scale=0.1) if bk else rnd(Kd, N, dev=dev, seed=82, scale=0.1)
    bias = torch.randn(N, device=dev) * 0.1
    ref = op(A, ak, Ma, Kd) @ op(B, bk, N, Kd).t()
    out = torch.empty(Ma, N, dtype=torch.bfloat16, device=dev)
    k.gemm(A, A.shape[1], ak, B, B.shape[1], bk, out, N, Ma, N, Kd, epi=k.epilogue(k.EPI_STORE, bias=bias))
    close(out, ref + bias)
    f = torch.full((Ma, N), -1.5, dtype=torch.float32, device=dev)
    k.gemm(A, A.shape[1], ak, B, B.shape[1], bk, f, N, Ma, N, Kd, epi=k.epilogue(k.EPI_STORE, accumulate=True))
    torch.testing.assert_close(f, ref - 1.5, rtol=1e-4, atol=5e-3)
    if ak and bk:  # batched items
        Bt, Mb = 2, 256 * 20
        A2, B2 = rnd(Bt, Mb, Kd, dev=dev, seed=83), rnd(Bt, N, Kd, dev=dev, seed=84, scale=0.1)
        C2 = torch.empty(Bt, Mb, N, dtype=torch.bfloat16, device=dev)
        k.gemm(A2, Kd, True, B2, Kd, True, C2, N, Mb, N, Kd, batch=Bt, sA=Mb * Kd, sB=N * Kd, sC=Mb * N)
        close(C2, A2.float() @ B2.float().transpose(1, 2))


@pytest.mark.parametrize("M,N,Kd", [(256 * 257, 768, 3072), (16416, 768, 3072), (16416, 3072, 768),
                                     (256 * 65 + 32, 768, 2304)])
def test_gemm_tail_round_shapes(dev, M, N, Kd):
    """The tile counts of the BERT products whose last round of 256 x 256 tiles is nearly empty:
    batch 256's N = 768 class (771 tiles = 3 rounds + 3), batch 32's (195 / 780 tiles for 256
    CUs) and a 32-row M tail (round 5's stream-K tail ran these; profiles/r5_streamk_keepin_ab.txt).
    Every element of every epilogue against torch, and bitwise-equal results from two runs."""
    k = K()
    A, B = rnd(M, Kd, dev=dev, seed=141), rnd(N, Kd, dev=dev, seed=142, scale=0.1)
    ref = A.float() @ B.float().t()
    bias = torch.randn(N, device=dev) * 0.1
    out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    k.gemm(A, Kd, True, B, Kd, True, out, N, M, N, Kd, epi=k.epilogue(k.EPI_STORE, bias=bias))
    close(out, ref + bias)
    again = torch.empty_like(out)
    k.gemm(A, Kd, True, B, Kd, True, again, N, M, N, Kd, epi=k.epilogue(k.EPI_STORE, bias=bias))
    assert torch.equal(out, again)
    # f32 hidden stream: bias + dropout(p = 0) + f32 residual
    R32 = torch.randn(M, N, device=dev)
    f = torch.empty(M, N, dtype=torch.float32, device=dev)
    k.gemm(A, Kd, True, B, Kd, True, f, N, M, N, Kd,
           epi=k.epilogue(k.EPI_BIAS_DROP_RES, bias=bias, residual=R32, drop_p=0.0, seed=3))
    torch.testing.assert_close(f, ref + bias + R32, rtol=1e-3, atol=2e-3 * ref.abs().max().item())
    # GELU + its derivative, then dGELU with the bias-gradient column sums, then a residual add
    aux = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    k.gemm(A, Kd, True, B, Kd, True, out, N, M, N, Kd, epi=k.epilogue(k.EPI_BIAS_GELU, bias=bias, aux=aux))
    z = ref + bias
    phi = 0.5 * (1 + torch.erf(z / math.sqrt(2)))
    close(out, z * phi)
    close(aux, phi + z * torch.exp(-0.5 * z * z) / math.sqrt(2 * math.pi))
    cs = torch.zeros(N, device=dev)
    k.gemm(A, Kd, True, B, Kd, True, out, N, M, N, Kd, epi=k.epilogue(k.EPI_DGELU, aux=aux, colsum=cs))
    dg = ref * aux.float()
    close(out, dg)
    torch.testing.assert_close(cs, dg.sum(0), rtol=2e-3, atol=2e-3 * dg.abs().sum(0).max().item())
    R16 = rnd(M, N, dev=dev, seed=143)
    k.gemm(A, Kd, True, B, Kd, True, out, N, M, N, Kd, epi=k.epilogue(k.EPI_ADD_RES, residual=R16))
    close(out, ref + R16.float())


def test_gemm_partial_last_wave_batched(dev):
    """batch 2 x 129 tile rows x 3 column tiles = 774 tiles, per-item bias"""
    k = K()
    Bt, M, N, Kd = 2, 256 * 129, 768, 512
    A, B = rnd(Bt, M, Kd, dev=dev, seed=64), rnd(Bt, N, Kd, dev=dev, seed=65, scale=0.1)
    bias = torch.randn(Bt, N, device=dev) * 0.1
    C = torch.empty(Bt, M, N, dtype=torch.bfloat16, device=dev)
    k.gemm(A, Kd, True, B, Kd, True, C, N, M, N, Kd, batch=Bt, sA=M * Kd, sB=N * Kd, sC=M * N,
           epi=k.epilogue(k.EPI_STORE, bias=bias, bias_bstride=N))
    close(C.float()[:, -256:], (A.float() @ B.float().transpose(1, 2) + bias[:, None, :])[:, -256:])


def test_gemm_bias_dropout_residual(dev):
    k = K()
    M, N, Kd = 512, 768, 256
    A, B = rnd(M, Kd, dev=dev, seed=11), rnd(N, Kd, dev=dev, seed=12, scale=0.1)
    bias = torch.randn(N, device=dev) * 0.1
    R = rnd(M, N, dev=dev, seed=13)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    k.gemm(A, Kd, True, B, Kd, True, out, N, M, N, Kd,
           epi=k.epilogue(k.EPI_BIAS_DROP_RES, bias=bias, residual=R, drop_p=0.0))
    y = A.float() @ B.float().t() + bias
    close(out, R.float() + y)
    p = 0.1
    k.gemm(A, Kd, True, B, Kd, True, out, N, M, N, Kd,
           epi=k.epilogue(k.EPI_BIAS_DROP_RES, bias=bias, residual=R, drop_p=p, seed=1234))
    d = out.float() - R.float()
    kept = (d - y / (1 - p)).abs() <= 0.05 * (y.abs() / (1 - p)) + 0.05
    dropped = d.abs() <= 0.02 * (R.float().abs() + 1)
    assert (kept | dropped).float().mean().item() > 0.999
    rate = (dropped & ~kept).float().mean().item()
    assert abs(rate - p) < 0.01, rate


def test_gemm_bias_dropout_residual_f32_stream(dev):
    """BIAS_DROP_RES into an f32 C reads an f32 residual (the encoder's f32 hidden stream):
    C = R32 + dropout(A B^T + bias) with no bf16 rounding of R32 or C; the dropout quads are
    the bf16-output epilogue's (same seed -> same keep pattern); batched with strides."""
    k = K()
    Bt, M, N, Kd = 2, 640, 768, 256
    A, B = rnd(Bt, M, Kd, dev=dev, seed=111), rnd(Bt, N, Kd, dev=dev, seed=112, scale=0.1)
    bias = torch.randn(Bt, N, device=dev) * 0.1
    R32 = torch.randn(Bt, M, N, device=dev) * 3.0 + 1.0 / 3.0  # not representable in bf16
    out = torch.empty(Bt, M, N, dtype=torch.float32, device=dev)
    y = A.float() @ B.float().transpose(1, 2) + bias[:, None, :]
    k.gemm(A, Kd, True, B, Kd, True, out, N, M, N, Kd, batch=Bt, sA=M * Kd, sB=N * Kd, sC=M * N,
           epi=k.epilogue(k.EPI_BIAS_DROP_RES, bias=bias, bias_bstride=N, residual=R32, res_bstride=M * N))
    torch.testing.assert_close(out, R32 + y, rtol=1e-5, atol=2e-5 * y.abs().max().item())
    p = 0.1
    k.gemm(A, Kd, True, B, Kd, True, out, N, M, N, Kd, batch=Bt, sA=M * Kd, sB=N * Kd, sC=M * N,
           epi=k.epilogue(k.EPI_BIAS_DROP_RES, bias=bias, bias_bstride=N, residual=R32, res_bstride=M * N,
                          drop_p=p, seed=99))
    ob = torch.empty(Bt, M, N, dtype=torch.bfloat16, device=dev)
    Z = torch.zeros(Bt, M, N, dtype=torch.bfloat16, device=dev)
    k.gemm(A, Kd, True, B, Kd, True, ob, N, M, N, Kd, batch=Bt, sA=M * Kd, sB=N * Kd, sC=M * N,
           epi=k.epilogue(k.EPI_BIAS_DROP_RES, bias=bias, bias_bstride=N, residual=Z, res_bstride=M * N,
                          drop_p=p, seed=99))
    d = out - R32
    keep = ob.float() != 0
    torch.testing.assert_close(d[keep], (y / (1 - p))[keep], rtol=1e-5, atol=2e-5 * y.abs().max().item())
    assert (d[~keep].abs() <= 1e-6 * R32.abs().max()).all()
    assert abs((~keep).float().mean().item() - p) < 0.01


@pytest.mark.gpu
def test_gemm_residual_recomputed_layernorm(dev):
    """res_ln: the f32 residual is LN(S) recomputed in the epilogue from the f32 rows S and
    per-row mean / rstd, per-column gamma / beta -- equal to passing the materialised LN
    output (the encoder's S2 -> next layer's residual, src/encoder.py); batched."""
    k = K()
    Bt, M, N, Kd = 2, 640, 768, 256
    A, B = rnd(Bt, M, Kd, dev=dev, seed=121), rnd(Bt, N, Kd, dev=dev, seed=122, scale=0.1)
    bias = torch.randn(Bt, N, device=dev) * 0.1
    S = torch.randn(Bt, M, N, device=dev) * 2.0 + 0.7
    mean = S.mean(-1).contiguous()
    rstd = torch.rsqrt(S.var(-1, unbiased=False) + 1e-12).contiguous()
    w, b = torch.randn(N, device=dev), torch.randn(N, device=dev)
    R32 = (S - mean[..., None]) * rstd[..., None] * w + b
    y = A.float() @ B.float().transpose(1, 2) + bias[:, None, :]
    for p in (0.0, 0.1):
        out, ref = (torch.empty(Bt, M, N, dtype=torch.float32, device=dev) for _ in range(2))
        k.gemm(A, Kd, True, B, Kd, True, out, N, M, N, Kd, batch=Bt, sA=M * Kd, sB=N * Kd, sC=M * N,
               epi=k.epilogue(k.EPI_BIAS_DROP_RES, bias=bias, bias_bstride=N, residual=S, res_bstride=M * N,
                              drop_p=p, seed=5, res_ln=(mean, rstd, w, b)))
        k.gemm(A, Kd, True, B, Kd, True, ref, N, M, N, Kd, batch=Bt, sA=M * Kd, sB=N * Kd, sC=M * N,
               epi=k.epilogue(k.EPI_BIAS_DROP_RES, bias=bias, bias_bstride=N, residual=R32, res_bstride=M * N,
                              drop_p=p, seed=5))
        torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-5 * R32.abs().max().item())
        if p == 0.0:
            torch.testing.assert_close(out, R32 + y, rtol=1e-5, atol=2e-5 * (R32.abs().max() + y.abs().max()).item())
    with pytest.raises(Exception):  # all four LN tensors or none
        k.gemm(A[0], Kd, True, B[0], Kd, True, out[0], N, M, N, Kd,
               epi=k.epilogue(k.EPI_BIAS_DROP_RES, bias=bias[0], residual=S[0], res_ln=(mean[0], rstd[0], w, None)))


def test_gemm_batched(dev):
    k = K()
    Bt, M, N, Kd = 3, 128, 128, 64
    A, B = rnd(Bt, M, Kd, dev=dev, seed=14), rnd(Bt, N, Kd, dev=dev, seed=15)
    C = torch.empty(Bt, M, N, dtype=torch.float32, device=dev)
    k.gemm(A, Kd, True, B, Kd, True, C, N, M, N, Kd, batch=Bt, sA=M * Kd, sB=N * Kd, sC=M * N)
    torch.testing.assert_close(C, A.float() @ B.float().transpose(1, 2), rtol=1e-4, atol=1e-3)


def test_gemm_rejects_bad_shapes(dev):
    k = K()
    from src._native import NativeError
    A = rnd(128, 64, dev=dev)
    B = rnd(100, 64, dev=dev)
    C = torch.empty(128, 100, device=dev)
    with pytest.raises(NativeError, match="multiple of 128"):
        k.gemm(A, 64, True, B, 64, True, C, 100, 128, 100, 64)


# ----------------------------------------------------------------------------- attention
def attn_ref(qkv, keymask, B, L, heads=12, dropmask=None, p=0.0):
    q, kk, v = qkv.float().view(B, L, 3, heads, 64).permute(2, 0, 3, 1, 4)
    s = q @ kk.transpose(-1, -2) / 8.0 + keymask.view(B, 1, 1, L)
    lse = torch.logsumexp(s, -1)
    P = torch.softmax(s, -1)
    if dropmask is not None:
        P = P * dropmask / (1 - p)
    o = (P @ v).permute(0, 2, 1, 3).reshape(B * L, heads * 64)
    return o, lse.reshape(B * heads, L)


def make_attn_inputs(dev, B, L, pad=True, seed=0, scale=1.0):
    qkv = rnd(B * L, 3 * 768, dev=dev, seed=seed, scale=scale)
    km = torch.zeros(B, L, device=dev)
    if pad and L > 6:
        km[0, L - L // 3:] = -10000.0
    return qkv, km


@pytest.mark.parametrize("B,L", [(2, 5), (2, 17), (1, 64), (2, 130), (2, 513)])
def test_attention_fwd(dev, B, L):
    k = K()
    qkv, km = make_attn_inputs(dev, B, L, seed=L, scale=2.0)
    O = torch.empty(B * L, 768, dtype=torch.bfloat16, device=dev)
    lse = torch.empty(B * 12, L, device=dev)
    k.attention_fwd(qkv, km, O, lse, B, L)
    o_ref, lse_ref = attn_ref(qkv, km, B, L)
    close(O, o_ref)
    torch.testing.assert_close(lse, lse_ref, rtol=1e-4, atol=2e-3)


@pytest.mark.parametrize("B,L", [(2, 5), (2, 17), (2, 130), (1, 513)])
def test_attention_bwd(dev, B, L):
    k = K()
    qkv, km = make_attn_inputs(dev, B, L, seed=100 + L, scale=1.5)
    O = torch.empty(B * L, 768, dtype=torch.bfloat16, device=dev)
    lse = torch.empty(B * 12, L, device=dev)
    k.attention_fwd(qkv, km, O, lse, B, L)
    dO = rnd(B * L, 768, dev=dev, seed=200 + L)
    dqkv = torch.zeros(B * L, 2304, dtype=torch.bfloat16, device=dev)
    delta = torch.empty(B * 12, L, device=dev)
    k.attention_bwd(qkv, km, O, dO, lse, delta, dqkv, B, L)
    x = qkv.float().requires_grad_(True)
    o_ref, _ = attn_ref(x, km, B, L)
    (g,) = torch.autograd.grad(o_ref, x, dO.float())
    for part in range(3):
        close(dqkv[:, 768 * part:768 * (part + 1)], g[:, 768 * part:768 * (part + 1)], atol_frac=2e-2)


def test_attention_dropout_consistent(dev):
    """Recover the kernel's dropped-P matrix with one-hot V rows (L <= 64), then check
    (a) its drop rate, (b) fwd == P*mask/(1-p) V on random V, (c) bwd matches autograd with that mask."""
    k = K()
    B, L, p, seed = 2, 60, 0.2, 99
    qkv, km = make_attn_inputs(dev, B, L, pad=False, seed=5, scale=1.0)
    probe = qkv.clone().view(B, L, 3, 12, 64)
    eye = torch.zeros(L, 64, device=dev)
    eye[torch.arange(L), torch.arange(L)] = 1.0
    probe[:, :, 2] = eye.view(1, L, 1, 64).to(torch.bfloat16)
    probe = probe.view(B * L, 2304)
    O = torch.empty(B * L, 768, dtype=torch.bfloat16, device=dev)
    lse = torch.empty(B * 12, L, device=dev)
    dm = k.dropmask_empty(B, L, 12, dev)
    k.attention_fwd(probe, km, O, lse, B, L, drop_p=p, seed=seed, dropmask=dm)
    Pd = O.float().view(B, L, 12, 64).permute(0, 2, 1, 3)[..., :L]  # [B,h,q,key] = P*mask/(1-p)
    mask = (Pd > 0).float()
    rate = 1 - mask.mean().item()
    assert abs(rate - p) < 0.02, rate
    # the emitted keep bits are exactly the mask the forward applied
    assert torch.equal(k.dropmask_dense(dm, L).view(B, 12, L, L), mask)
    # (b) forward on the real V with the recovered mask
    k.attention_fwd(qkv, km, O, lse, B, L, drop_p=p, seed=seed, dropmask=dm)
    o_ref, _ = attn_ref(qkv, km, B, L, dropmask=mask, p=p)
    close(O, o_ref, atol_frac=2e-2)
    # (c) backward
    dO = rnd(B * L, 768, dev=dev, seed=7)
    dqkv = torch.zeros(B * L, 2304, dtype=torch.bfloat16, device=dev)
    delta = torch.empty(B * 12, L, device=dev)
    k.attention_bwd(qkv, km, O, dO, lse, delta, dqkv, B, L, drop_p=p, seed=seed, dropmask=dm)
    x = qkv.float().requires_grad_(True)
    o2, _ = attn_ref(x, km, B, L, dropmask=mask, p=p)
    (g,) = torch.autograd.grad(o2, x, dO.float())
    for part in range(3):
        close(dqkv[:, 768 * part:768 * (part + 1)], g[:, 768 * part:768 * (part + 1)], atol_frac=3e-2)
    with pytest.raises(Exception):  # dropout backward without the forward's bits is refused
        k.attention_bwd(qkv, km, O, dO, lse, delta, dqkv, B, L, drop_p=p, seed=seed)


@pytest.mark.parametrize("B,L", [(2, 200), (1, 321), (2, 280)])
def test_attention_dropout_multiword(dev, B, L):
    """L > 64: several keep words per query row; fwd and bwd against autograd with the
    mask decoded from the emitted bits, plus the drop rate.  L = 280: 24 query rows past the
    last 128-row block and 24 keys past the last 64-key block (the one-wave TAIL kernels)."""
    k = K()
    p, seed = 0.1, 1234
    qkv, km = make_attn_inputs(dev, B, L, pad=True, seed=11, scale=1.0)
    O = torch.empty(B * L, 768, dtype=torch.bfloat16, device=dev)
    lse = torch.empty(B * 12, L, device=dev)
    dm = k.dropmask_empty(B, L, 12, dev)
    k.attention_fwd(qkv, km, O, lse, B, L, drop_p=p, seed=seed, dropmask=dm)
    mask = k.dropmask_dense(dm, L).view(B, 12, L, L)
    assert abs((1 - mask.mean().item()) - p) < 0.01
    o_ref, _ = attn_ref(qkv, km, B, L, dropmask=mask, p=p)
    close(O, o_ref, atol_frac=2e-2)
    dO = rnd(B * L, 768, dev=dev, seed=8)
    dqkv = torch.zeros(B * L, 2304, dtype=torch.bfloat16, device=dev)
    delta = torch.empty(B * 12, L, device=dev)
    k.attention_bwd(qkv, km, O, dO, lse, delta, dqkv, B, L, drop_p=p, seed=seed, dropmask=dm)
    x = qkv.float().requires_grad_(True)
    o2, _ = attn_ref(x, km, B, L, dropmask=mask, p=p)
    (g,) = torch.autograd.grad(o2, x, dO.float())
    for part in range(3):
        close(dqkv[:, 768 * part:768 * (part + 1)], g[:, 768 * part:768 * (part + 1)], atol_frac=3e-2)


def test_attention_dropout_joint_statistics(dev):
    """Higher-order statistics of the attention-probs dropout draws: the 16 keep decisions of a
    half-wave's 16 consecutive keys come from ONE 32-bit hash (attention.hip pair_draw: 24-bit
    multiplies of rotated windows), so beyond the per-key rate the JOINT behaviour of a group is
    tested on the forward's own keep words (1.6 M groups of 16 at B = 8, L = 513, p = 0.1):
    the kept count per group against Binomial(16, 0.9), and the 16 patterns of every aligned
    4-bit sub-group against their product probabilities -- chi-square at alpha = 1e-6."""
    from scipy import stats
    k = K()
    B, L, p = 8, 513, 0.1
    qkv, km = make_attn_inputs(dev, B, L, pad=False, seed=21, scale=1.0)
    O = torch.empty(B * L, 768, dtype=torch.bfloat16, device=dev)
    lse = torch.empty(B * 12, L, device=dev)
    dm = k.dropmask_empty(B, L, 12, dev)
    k.attention_fwd(qkv, km, O, lse, B, L, drop_p=p, seed=97, dropmask=dm)
    words = dm[:, :, : L // 64].reshape(-1)  # full 64-key tiles only (the last one holds 1 key)
    groups = torch.stack([(words >> (16 * g)) & 0xFFFF for g in range(4)], 1).reshape(-1).cpu().numpy()
    n = groups.size
    kept = np.unpackbits(groups.astype(">u2").view(np.uint8)).reshape(n, 16).sum(1)
    obs = np.bincount(kept, minlength=17).astype(np.float64)
    exp = n * stats.binom.pmf(np.arange(17), 16, 1 - p)
    lo = np.nonzero(exp >= 20)[0][0]  # pool the sparse low-count bins
    o2 = np.concatenate([[obs[:lo].sum()], obs[lo:]])
    e2 = np.concatenate([[exp[:lo].sum()], exp[lo:]])
    chi_count = float(((o2 - e2) ** 2 / e2).sum())
    crit_count = stats.chi2.ppf(1 - 1e-6, len(o2) - 1)
    nib = np.concatenate([(groups >> (4 * s)) & 0xF for s in range(4)])
    obs4 = np.bincount(nib, minlength=16).astype(np.float64)
    ones = np.array([bin(v).count("1") for v in range(16)])
    exp4 = nib.size * (1 - p) ** ones * p ** (4 - ones)
    chi_nib = float(((obs4 - exp4) ** 2 / exp4).sum())
    crit_nib = stats.chi2.ppf(1 - 1e-6, 15)
    print(f"\n[dropout joint] {n} groups: kept-count chi2 {chi_count:.1f} (crit {crit_count:.1f}), "
          f"4-bit pattern chi2 {chi_nib:.1f} (crit {crit_nib:.1f}), drop rate {1 - kept.mean() / 16:.5f}")
    assert abs(1 - kept.mean() / 16 - p) < 2e-3
    assert chi_count < crit_count and chi_nib < crit_nib


@pytest.mark.parametrize("B,L", [(2, 200), (1, 513)])
def test_attention_dropout_inference_matches_training_forward(dev, B, L):
    """MC-dropout inference (no dropmask: the forward kernel that stores no keep bits) drops
    exactly the elements the training forward drops: its dropped-P matrix, recovered 64
    keys at a time with one-hot V rows, has the zeros the training kernel's keep bits say;
    O on the real V and LSE agree with the training forward to float-ordering tolerance."""
    k = K()
    p, seed = 0.1, 77
    qkv, km = make_attn_inputs(dev, B, L, pad=False, seed=5, scale=1.0)
    O1 = torch.empty(B * L, 768, dtype=torch.bfloat16, device=dev)
    lse1, lse2 = torch.empty(B * 12, L, device=dev), torch.empty(B * 12, L, device=dev)
    dm = k.dropmask_empty(B, L, 12, dev)
    k.attention_fwd(qkv, km, O1, lse1, B, L, drop_p=p, seed=seed, dropmask=dm)
    keep = k.dropmask_dense(dm, L).view(B, 12, L, L)
    seen = torch.zeros(B, 12, L, L, device=dev)
    for c in range(0, L, 64):  # one-hot V on keys [c, c+64): O[q, d] = P[q, c+d] * keep / (1-p)
        w = min(64, L - c)
        probe = qkv.clone().view(B, L, 3, 12, 64)
        probe[:, :, 2] = 0
        probe[:, c + torch.arange(w, device=dev), 2, :, torch.arange(w, device=dev)] = 1.0
        O = torch.empty(B * L, 768, dtype=torch.bfloat16, device=dev)
        k.attention_fwd(probe.view(B * L, 2304), km, O, lse2, B, L, drop_p=p, seed=seed)
        seen[..., c:c + w] = (O.float().view(B, L, 12, 64).permute(0, 2, 1, 3)[..., :w] > 0).float()
    assert torch.equal(seen, keep)
    O2 = torch.empty_like(O1)
    k.attention_fwd(qkv, km, O2, lse2, B, L, drop_p=p, seed=seed)
    close(O2, O1.float(), atol_frac=1e-2)
    torch.testing.assert_close(lse2, lse1, rtol=1e-5, atol=1e-5)


# ----------------------------------------------------------------------------- layernorm
@pytest.mark.parametrize("H,groups,rows_per", [(768, 3, 130), (768, 2, 77), (256, 1, 9), (1024, 2, 64)])
def test_layernorm_fwd_grouped(dev, H, groups, rows_per):
    """row groups with their own affine parameters (the K ensemble members in one launch):
    both forward kernels (16-B row pairs when the group size is even or there is one group,
    else row per wave: the 77-row groups) against torch per group; odd total row counts."""
    k = K()
    rows = groups * rows_per
    X = rnd(rows, H, dev=dev, seed=31, scale=2.0)
    w = torch.randn(groups, H, device=dev) * 0.1 + 1
    b = torch.randn(groups, H, device=dev) * 0.1
    ref = torch.cat([torch.nn.functional.layer_norm(X[g * rows_per:(g + 1) * rows_per].float(), (H,), w[g], b[g],
                                                    eps=1e-12) for g in range(groups)])
    Y = torch.empty_like(X)
    mean, rstd = torch.empty(rows, device=dev), torch.empty(rows, device=dev)
    k.layernorm_fwd(X, w, b, Y, mean, rstd, group_rows=rows_per, param_stride=H)
    close(Y, ref)
    torch.testing.assert_close(mean, X.float().mean(1), rtol=1e-4, atol=1e-4)


def test_layernorm_fwd_bwd(dev):
    k = K()
    rows, H, p, seed = 333, 768, 0.1, 77
    X = rnd(rows, H, dev=dev, seed=20, scale=3.0)
    w = torch.randn(H, device=dev) * 0.1 + 1
    b = torch.randn(H, device=dev) * 0.1
    Y = torch.empty_like(X)
    mean, rstd = torch.empty(rows, device=dev), torch.empty(rows, device=dev)
    k.layernorm_fwd(X, w, b, Y, mean, rstd)
    xr = X.float().requires_grad_(True)
    wr, br = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    yr = torch.nn.functional.layer_norm(xr, (H,), wr, br, eps=1e-12)
    close(Y, yr)
    dY = rnd(rows, H, dev=dev, seed=21)
    dX, dXd = torch.empty_like(X), torch.empty_like(X)
    P = k.ln_parts(rows)
    pw, pb, pbias = (torch.empty(P, H, device=dev) for _ in range(3))
    k.layernorm_bwd(dY, X, mean, rstd, w, dX, dXd, p, seed, pw, pb, pbias)
    gx, gw, gb = torch.autograd.grad(yr, (xr, wr, br), dY.float())
    close(dX, gx)
    sw, sb, sbias = torch.empty(H, device=dev), torch.empty(H, device=dev), torch.empty(H, device=dev)
    k.colsum_reduce(pw, sw)
    k.colsum_reduce(pb, sb)
    k.colsum_reduce(pbias, sbias)
    torch.testing.assert_close(sw, gw, rtol=1e-2, atol=0.05)
    torch.testing.assert_close(sb, gb, rtol=1e-2, atol=0.05)
    # dropout backward: every element either dX/(1-p) or 0, ~p dropped, colsum matches
    dx, dd = dX.float(), dXd.float()
    kept = (dd - dx / (1 - p)).abs() <= 0.02 * dx.abs() / (1 - p) + 1e-3
    zero = dd == 0
    assert (kept | zero).all()
    assert abs(zero.float().mean().item() - p) < 0.01
    torch.testing.assert_close(sbias, dd.sum(0), rtol=1e-2, atol=0.05)


@pytest.mark.parametrize("groups", [1, 3])
def test_layernorm_f32_stream_fwd_bwd(dev, groups):
    """mmu_layernorm_fwd_f32 (f32 X -> bf16 Y + f32 Y32, grouped affine params as for the
    ensemble members) and mmu_layernorm_bwd_f32 against torch fp32 on the same f32 input."""
    k = K()
    rows_per, H, p, seed = 111, 768, 0.1, 5
    rows = groups * rows_per
    X = torch.randn(rows, H, device=dev) * 3.0 + 0.5
    w = torch.randn(groups, H, device=dev) * 0.1 + 1
    b = torch.randn(groups, H, device=dev) * 0.1
    Y = torch.empty(rows, H, dtype=torch.bfloat16, device=dev)
    Y32 = torch.empty(rows, H, device=dev)
    mean, rstd = torch.empty(rows, device=dev), torch.empty(rows, device=dev)
    k.layernorm_fwd_f32(X, w, b, Y, Y32, mean, rstd, group_rows=rows_per, param_stride=H)
    ref = torch.cat([torch.nn.functional.layer_norm(X[g * rows_per:(g + 1) * rows_per], (H,), w[g], b[g], eps=1e-12)
                     for g in range(groups)])
    torch.testing.assert_close(Y32, ref, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(Y.float(), ref, rtol=2 ** -8, atol=1e-3)  # one bf16 rounding of the f32 row
    torch.testing.assert_close(mean, X.mean(1), rtol=1e-5, atol=1e-5)
    if groups > 1:
        return
    xr, wr, br = X.clone().requires_grad_(True), w[0].clone().requires_grad_(True), b[0].clone().requires_grad_(True)
    yr = torch.nn.functional.layer_norm(xr, (H,), wr, br, eps=1e-12)
    dY = rnd(rows, H, dev=dev, seed=22)
    dX, dXd = torch.empty_like(Y), torch.empty_like(Y)
    P = k.ln_parts(rows)
    pw, pb, pbias = (torch.empty(P, H, device=dev) for _ in range(3))
    k.layernorm_bwd(dY, X, mean, rstd, w[0], dX, dXd, p, seed, pw, pb, pbias)
    gx, gw, gb = torch.autograd.grad(yr, (xr, wr, br), dY.float())
    close(dX, gx)
    sw, sb = torch.empty(H, device=dev), torch.empty(H, device=dev)
    k.colsum_reduce(pw, sw)
    k.colsum_reduce(pb, sb)
    torch.testing.assert_close(sw, gw, rtol=1e-2, atol=0.05)
    torch.testing.assert_close(sb, gb, rtol=1e-2, atol=0.05)


# ----------------------------------------------------------------------------- pooling / adam / uncertainty
def test_row_pool(dev):
    k = K()
    B, C = 3, 2048
    f = rnd(B, 2048, 7, 7, dev=dev, seed=30).contiguous(memory_format=torch.channels_last)
    out = torch.empty(B, 3, C, device=dev)
    k.row_pool_fwd(f.permute(0, 2, 3, 1), 3, out)
    fr = f.float().requires_grad_(True)
    ref = torch.nn.functional.adaptive_avg_pool2d(fr, (3, 1)).flatten(2).transpose(1, 2)
    torch.testing.assert_close(out, ref, rtol=1e-3, atol=1e-3)
    d = torch.randn(B, 3, C, device=dev)
    df = torch.empty_like(f)
    k.row_pool_bwd(d, 3, df.permute(0, 2, 3, 1))
    (g,) = torch.autograd.grad(ref, fr, d)
    close(df, g)


def test_bertadam_matches_restatement(dev):
    k = K()
    from oracle.bertadam_ref import bertadam_step
    sizes = [1000, 70000, 5, 768 * 3]
    groups = [0, 0, 1, 1]
    active = [1, 1, 1, 0]
    g = torch.Generator().manual_seed(0)
    ps = [torch.randn(n, generator=g) for n in sizes]
    gs = [torch.randn(n, generator=g) * (3.0 if i == 1 else 0.01) for i, n in enumerate(sizes)]
    offs = np.cumsum([0] + sizes)
    flat_p = torch.cat(ps).to(dev)
    flat_g = torch.cat(gs).to(dev)
    m, v = torch.zeros_like(flat_p), torch.zeros_like(flat_p)
    copy = torch.zeros(sum(sizes), dtype=torch.bfloat16, device=dev)
    CH = 4096
    chunks, tab = [], []
    for t, n in enumerate(sizes):
        first = len(chunks)
        for s in range(0, n, CH):
            chunks.append((t, s, min(CH, n - s)))
        tab.append((offs[t], n, groups[t], offs[t] if t != 2 else -1, active[t], first, len(chunks) - first))
    table = torch.tensor([x for r in tab for x in r] + [x for c in chunks for x in c], dtype=torch.int64, device=dev)
    steps = torch.zeros(len(sizes), dtype=torch.int32, device=dev)
    ws = torch.empty(len(chunks) + 2 * len(sizes), device=dev)
    rp = [p.clone() for p in ps]
    rm = [torch.zeros(n) for n in sizes]
    rv = [torch.zeros(n) for n in sizes]
    rs = [0] * len(sizes)
    lr, warm, tt = 1e-3, 0.1, 20.0
    for it in range(3):
        k.bertadam_step(flat_p, flat_g, m, v, copy, table, steps, len(sizes), len(chunks), lr, lr, 0.01, warm, tt,
                        0.9, 0.999, 1e-6, 1.0, ws)
        act = [i for i in range(len(sizes)) if active[i]]
        new = bertadam_step([rp[i] for i in act], [gs[i] for i in act], [rm[i] for i in act], [rv[i] for i in act],
                            [rs[i] for i in act], lr, [0.01 if groups[i] == 0 else 0.0 for i in act], warm, tt)
        for j, i in enumerate(act):
            rs[i] = new[j]
    torch.cuda.synchronize()
    got = flat_p.cpu()
    for t in range(len(sizes)):
        torch.testing.assert_close(got[offs[t]:offs[t + 1]], rp[t], rtol=1e-5, atol=1e-6)
    assert steps.cpu().tolist() == [3, 3, 3, 0]
    torch.testing.assert_close(copy[:sizes[0]].float().cpu(), rp[0].bfloat16().float())


def test_uncertainty_nll_ece(dev):
    k = K()
    from oracle import uncertainty_ref as U
    S, R, C = 257, 15, 101
    g = torch.Generator().manual_seed(3)
    logits = torch.randn(S, R, C, generator=g) * 3
    y = torch.randint(0, C, (S,), generator=g)
    ld, yd = logits.to(dev), y.to(dev)
    pb, nll, conf, cor = (torch.empty(S, C, device=dev), torch.empty(S, device=dev), torch.empty(S, device=dev),
                          torch.empty(S, device=dev))
    k.uncertainty(ld, yd, pb, nll, conf, cor)
    bins = torch.empty(45, device=dev)
    k.ece_bins(conf, cor, 15, bins)
    pr = U.probs_mean(logits.numpy().transpose(1, 0, 2), member_axes=(0,))
    np.testing.assert_allclose(pb.cpu().numpy(), pr, rtol=1e-4, atol=1e-6)
    assert abs(nll.mean().item() - U.nll(pr, y.numpy())) < 1e-4
    bb = bins.view(15, 3).cpu().double().numpy()
    ece = float((np.abs(bb[:, 2] - bb[:, 1]) / S).sum())
    assert abs(ece - U.ece(pr, y.numpy())) < 1e-4


# ------------------------------------------------------------------ BatchNorm (+ residual) (+ ReLU)
def _bn_ref(x, w, b, skip, relu, eps=1e-5):
    """f32 torch reference of training-mode BN [+ skip] [+ ReLU] on the same bf16 inputs"""
    y = torch.nn.functional.batch_norm(x, None, None, w, b, training=True, eps=eps)
    if skip is not None:
        y = y + skip
    return torch.relu(y) if relu else y


@pytest.mark.parametrize("N,C,H,W,skip,relu", [(4, 64, 9, 7, False, True), (3, 256, 5, 5, True, True),
                                               (2, 2048, 3, 3, False, False), (5, 96, 4, 3, True, False)])
def test_batchnorm_train_fwd_bwd(dev, N, C, H, W, skip, relu):
    k = K()
    g = torch.Generator(device=dev).manual_seed(C + H)
    cl = torch.channels_last
    x = (torch.randn(N, C, H, W, generator=g, device=dev) * 2 + 0.7).to(torch.bfloat16).contiguous(memory_format=cl)
    s = (torch.randn(N, C, H, W, generator=g, device=dev)).to(torch.bfloat16).contiguous(memory_format=cl) if skip else None
    w = torch.rand(C, generator=g, device=dev) + 0.5
    b = torch.randn(C, generator=g, device=dev) * 0.1
    rm, rv = torch.randn(C, device=dev) * 0.1, torch.rand(C, device=dev) + 0.5
    rm0, rv0 = rm.clone(), rv.clone()
    nbt = torch.zeros((), dtype=torch.int64, device=dev)
    Y = torch.empty_like(x)
    sm, si = torch.empty(C, device=dev), torch.empty(C, device=dev)
    k.batchnorm_fwd(x, Y, w, b, rm, rv, True, 0.1, 1e-5, relu=relu, skip=s, num_batches_tracked=nbt,
                    save_mean=sm, save_invstd=si)
    xf = x.float().requires_grad_(True)
    wf, bf_ = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    sf = s.float().requires_grad_(True) if skip else None
    ref = _bn_ref(xf, wf, bf_, sf, relu)
    close(Y, ref.detach(), atol_frac=1e-2)
    n = N * H * W
    mu = x.float().mean((0, 2, 3))
    var = x.float().var((0, 2, 3), unbiased=False)
    torch.testing.assert_close(sm, mu, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(si, (var + 1e-5).rsqrt(), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(rm, 0.9 * rm0 + 0.1 * mu, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(rv, 0.9 * rv0 + 0.1 * var * n / (n - 1), rtol=1e-5, atol=1e-6)
    assert int(nbt) == 1
    # backward: the mask comes from the kernel's own output, the reference uses its own
    dY = torch.randn(N, C, H, W, generator=g, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
    dX = torch.empty_like(x)
    dS = torch.empty_like(x) if skip else None
    dw = torch.full((C,), 0.25, device=dev)  # accumulated into
    db = torch.full((C,), -0.5, device=dev)
    k.batchnorm_bwd(dY, Y if relu else None, x, w, sm, si, relu, dX, dS, dw, db)
    if relu:  # the ReLU-mask path: the forward's bit mask instead of Y, bit-identical results
        mask = torch.empty(x.numel() // 8, dtype=torch.uint8, device=dev)
        Y2 = torch.empty_like(x)
        rm2, rv2 = rm0.clone(), rv0.clone()
        k.batchnorm_fwd(x, Y2, w, b, rm2, rv2, True, 0.1, 1e-5, relu=relu, skip=s, relu_mask=mask,
                        save_mean=torch.empty_like(sm), save_invstd=torch.empty_like(si))
        assert torch.equal(Y2, Y)
        bits = ((Y.permute(0, 2, 3, 1).reshape(-1, 8).float() > 0).to(torch.int32)
                << torch.arange(8, device=dev, dtype=torch.int32)).sum(1)
        assert torch.equal(mask.to(torch.int32), bits)
        dX2, dS2 = torch.empty_like(x), torch.empty_like(x) if skip else None
        dw2, db2 = torch.full((C,), 0.25, device=dev), torch.full((C,), -0.5, device=dev)
        k.batchnorm_bwd(dY, None, x, w, sm, si, relu, dX2, dS2, dw2, db2, relu_mask=mask)
        assert torch.equal(dX2, dX) and torch.equal(dw2, dw) and torch.equal(db2, db)
        if skip:
            assert torch.equal(dS2, dS)
    grads = torch.autograd.grad(ref, [xf, wf, bf_] + ([sf] if skip else []), dY.float())
    close(dX, grads[0], atol_frac=2e-2)
    torch.testing.assert_close(dw - 0.25, grads[1], rtol=2e-2, atol=2e-2 * grads[1].abs().max().item() + 1e-3)
    torch.testing.assert_close(db + 0.5, grads[2], rtol=2e-2, atol=2e-2 * grads[2].abs().max().item() + 1e-3)
    if skip:
        close(dS, grads[3], atol_frac=1e-2)


@pytest.mark.parametrize("C,skip,relu", [(64, False, True), (256, True, True), (2048, False, False)])
def test_batchnorm_cross_rank_sums_equal_whole_batch(dev, C, skip, relu):
    """mmu_batchnorm_stats / _fwd_sums / _bwd_reduce / _bwd_sums over two halves of a batch,
    their sums added (the all-reduce two ranks would do), reproduce mmu_batchnorm_fwd / _bwd on
    the whole batch: outputs, saved statistics, running statistics, dX, dSkip and the two
    halves' dweight / dbias summing to the whole batch's."""
    k = K()
    g = torch.Generator(device=dev).manual_seed(C)
    cl = torch.channels_last
    N, H, W = 6, 7, 5
    x = (torch.randn(N, C, H, W, generator=g, device=dev) * 2 + 0.7).to(torch.bfloat16).contiguous(memory_format=cl)
    s = torch.randn(N, C, H, W, generator=g, device=dev).to(torch.bfloat16).contiguous(memory_format=cl) if skip else None
    dY = torch.randn(N, C, H, W, generator=g, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
    w, b = torch.rand(C, generator=g, device=dev) + 0.5, torch.randn(C, generator=g, device=dev) * 0.1
    rm0, rv0 = torch.randn(C, device=dev) * 0.1, torch.rand(C, device=dev) + 0.5
    # whole batch
    rm, rv = rm0.clone(), rv0.clone()
    Y, sm, si = torch.empty_like(x), torch.empty(C, device=dev), torch.empty(C, device=dev)
    mask = torch.empty(x.numel() // 8, dtype=torch.uint8, device=dev) if relu else None
    k.batchnorm_fwd(x, Y, w, b, rm, rv, True, 0.1, 1e-5, relu=relu, skip=s, save_mean=sm, save_invstd=si,
                    relu_mask=mask)
    dX, dS = torch.empty_like(x), torch.empty_like(x) if skip else None
    dw, db = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
    k.batchnorm_bwd(dY, None, x, w, sm, si, relu, dX, dS, dw, db, relu_mask=mask)
    # two "ranks"
    halves = [slice(0, 4), slice(4, N)]  # ragged: 4 + 2 images
    part = lambda t, h: None if t is None else t[h].contiguous(memory_format=cl)
    sums = [k.bn_sums_buffer(C, dev) for _ in halves]
    for h, sm_ in zip(halves, sums):
        k.batchnorm_stats(part(x, h), sm_)
    assert [int(t[2 * C]) for t in sums] == [4 * H * W, 2 * H * W]
    tot = sums[0] + sums[1]
    outs = []
    for h in halves:
        rm_h, rv_h = rm0.clone(), rv0.clone()
        nbt = torch.zeros((), dtype=torch.int64, device=dev)
        xh = part(x, h)
        Yh, smh, sih = torch.empty_like(xh), torch.empty(C, device=dev), torch.empty(C, device=dev)
        mh = torch.empty(xh.numel() // 8, dtype=torch.uint8, device=dev) if relu else None
        k.batchnorm_fwd_sums(xh, Yh, tot, w, b, rm_h, rv_h, 0.1, 1e-5, relu=relu, skip=part(s, h),
                             num_batches_tracked=nbt, save_mean=smh, save_invstd=sih, relu_mask=mh)
        assert int(nbt) == 1
        torch.testing.assert_close(rm_h, rm, rtol=1e-6, atol=1e-7)
        torch.testing.assert_close(rv_h, rv, rtol=1e-6, atol=1e-7)
        torch.testing.assert_close(smh, sm, rtol=1e-6, atol=1e-7)
        torch.testing.assert_close(sih, si, rtol=1e-6, atol=1e-7)
        outs.append((xh, Yh, smh, sih, mh))
    Yc = torch.cat([o[1] for o in outs])
    assert (Yc.float() - Y.float()).abs().max() <= 1e-2 * Y.float().abs().max()
    assert (Yc != Y).float().mean() < 1e-3  # bit-identical but for a rare last-bit rounding
    bsums, dws, dbs = [k.bn_sums_buffer(C, dev) for _ in halves], [], []
    for h, bs, (xh, Yh, smh, sih, mh) in zip(halves, bsums, outs):
        dwh, dbh = torch.full((C,), 0.25, device=dev), torch.full((C,), -0.5, device=dev)
        k.batchnorm_bwd_reduce(part(dY, h), None, xh, smh, sih, relu, bs, dwh, dbh, relu_mask=mh)
        dws.append(dwh - 0.25)
        dbs.append(dbh + 0.5)
    torch.testing.assert_close(dws[0] + dws[1], dw, rtol=1e-4, atol=1e-4 * dw.abs().max().item())
    torch.testing.assert_close(dbs[0] + dbs[1], db, rtol=1e-4, atol=1e-4 * db.abs().max().item())
    btot = bsums[0] + bsums[1]
    dXs, dSs = [], []
    for h, (xh, Yh, smh, sih, mh) in zip(halves, outs):
        dXh, dSh = torch.empty_like(xh), torch.empty_like(xh) if skip else None
        k.batchnorm_bwd_sums(part(dY, h), None, xh, btot, w, smh, sih, relu, dXh, dSh, relu_mask=mh)
        dXs.append(dXh)
        dSs.append(dSh)
    dXc = torch.cat(dXs)
    assert (dXc.float() - dX.float()).abs().max() <= 1e-2 * dX.float().abs().max()
    assert (dXc != dX).float().mean() < 1e-2
    if skip:
        assert torch.equal(torch.cat(dSs), dS)


def _res_decode(hi, res):
    """value of a bf16 map + its 8-bit stream residue (include/mmu.h mmu_batchnorm_fwd y_res):
    hi + res * 2^(e - 15), e the binary exponent of hi (0 for hi == 0)"""
    h = hi.float()
    m, ex = torch.frexp(h)
    scale = torch.where(h == 0, torch.zeros_like(h), torch.ldexp(torch.ones_like(h), ex - 1 - 15))
    return h + res.view(hi.permute(0, 2, 3, 1).shape).permute(0, 3, 1, 2).float() * scale


def _res_encode(v):
    """the kernel's encoding restated: (bf16(v), rint((v - hi) * 2^15 / 2^e)) as an NHWC int8 map"""
    hi = v.to(torch.bfloat16)
    h = hi.float()
    m, ex = torch.frexp(h)
    q = torch.round((v - h) * torch.ldexp(torch.ones_like(h), 15 - (ex - 1))).clamp(-127, 127)
    q = torch.where(h == 0, torch.zeros_like(q), q)
    return hi.contiguous(memory_format=torch.channels_last), q.to(torch.int8).permute(0, 2, 3, 1).contiguous().view(-1)


@pytest.mark.parametrize("training", [True, False])
def test_batchnorm_stream_residue(dev, training):
    """The residual stream's 8-bit residue (round 5): bn3 reads its skip as bf16 + residue and
    writes the block output's residue; the downsample's BN writes its output's.  The decoded
    stream is held to 2^-14 of the f32 value (bf16 alone: 2^-8), against an f32 torch BN on the
    same bf16 conv output and the f32 skip; the C-ABI rejects a y_res without skip_res."""
    k = K()
    g = torch.Generator(device=dev).manual_seed(11)
    cl = torch.channels_last
    N, C, H, W = 3, 256, 7, 5
    x = (torch.randn(N, C, H, W, generator=g, device=dev) * 2 + 0.3).to(torch.bfloat16).contiguous(memory_format=cl)
    s32 = torch.randn(N, C, H, W, generator=g, device=dev) * 3
    s32[:, :, 0, 0] = 0.0  # exact zeros in the stream
    shi, sres = _res_encode(s32)
    assert sres.abs().max().item() <= 127
    assert (_res_decode(shi, sres) - s32).abs().max().item() <= 2.0 ** -15 * s32.abs().max().item()
    w = torch.rand(C, generator=g, device=dev) + 0.5
    b = torch.randn(C, generator=g, device=dev) * 0.1
    rm, rv = torch.randn(C, device=dev) * 0.1, torch.rand(C, device=dev) + 0.5
    Y, yres = torch.empty_like(x), torch.empty(x.numel(), dtype=torch.int8, device=dev)
    kw = dict(save_mean=torch.empty(C, device=dev), save_invstd=torch.empty(C, device=dev),
              relu_mask=torch.empty(x.numel() // 8, dtype=torch.uint8, device=dev)) if training else {}
    k.batchnorm_fwd(x, Y, w, b, rm.clone(), rv.clone(), training, 0.1, 1e-5, relu=True, skip=shi, skip_res=sres,
                    y_res=yres, **kw)
    ref = torch.relu(torch.nn.functional.batch_norm(x.float(), rm, rv, w, b, training=training, eps=1e-5) + s32)
    got = _res_decode(Y, yres)
    scale = ref.abs().max().item()
    err = (got - ref).abs().max().item()
    err_bf16 = (Y.float() - ref).abs().max().item()
    assert err <= 2.0 ** -13 * scale, (err, err_bf16, scale)
    assert err_bf16 > 8 * err  # the residue carries the bits bf16 drops
    # the downsample's BN: no skip, no ReLU, the output's residue
    Y2, yres2 = torch.empty_like(x), torch.empty(x.numel(), dtype=torch.int8, device=dev)
    kw2 = dict(save_mean=torch.empty(C, device=dev), save_invstd=torch.empty(C, device=dev)) if training else {}
    k.batchnorm_fwd(x, Y2, w, b, rm.clone(), rv.clone(), training, 0.1, 1e-5, y_res=yres2, **kw2)
    ref2 = torch.nn.functional.batch_norm(x.float(), rm, rv, w, b, training=training, eps=1e-5)
    assert (_res_decode(Y2, yres2) - ref2).abs().max().item() <= 2.0 ** -13 * ref2.abs().max().item()
    with pytest.raises(Exception, match="skip_res"):
        k.batchnorm_fwd(x, Y, w, b, rm.clone(), rv.clone(), training, 0.1, 1e-5, relu=True, skip=shi, y_res=yres, **kw)


def test_batchnorm_eval_and_module(dev):
    """the module path (train, then eval from the updated running statistics) against
    torch.nn.BatchNorm2d in f32 on the same bf16 inputs, with the fused residual + ReLU"""
    from src.resnet import BatchNorm2d
    cl = torch.channels_last
    g = torch.Generator(device=dev).manual_seed(3)
    C = 128
    bn = BatchNorm2d(C).to(dev)
    ref = torch.nn.BatchNorm2d(C).to(dev)
    with torch.no_grad():
        bn.weight.copy_(torch.rand(C, generator=g, device=dev) + 0.5)
        bn.bias.copy_(torch.randn(C, generator=g, device=dev))
        ref.load_state_dict(bn.state_dict())
    x = (torch.randn(6, C, 7, 7, generator=g, device=dev) * 3 - 1).to(torch.bfloat16).contiguous(memory_format=cl)
    sk = torch.randn(6, C, 7, 7, generator=g, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
    for _ in range(2):  # two training steps: running stats and num_batches_tracked follow torch
        y = bn(x, skip=sk, relu=True)
        yr = torch.relu(ref(x.float()) + sk.float())
        close(y, yr.detach(), atol_frac=1e-2)
    torch.testing.assert_close(bn.running_mean, ref.running_mean, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(bn.running_var, ref.running_var, rtol=1e-4, atol=1e-5)
    assert int(bn.num_batches_tracked) == int(ref.num_batches_tracked) == 2
    bn.eval()
    ref.eval()
    close(bn(x, relu=False), ref(x.float()).detach(), atol_frac=1e-2)
    # autograd through the module: weight / bias grads land in .grad
    bn.train()
    ref.train()
    xr = x.float().requires_grad_(True)
    xb = x.clone().requires_grad_(True)
    y = bn(xb, relu=True)
    y.float().pow(2).sum().backward()
    torch.relu(ref(xr)).pow(2).sum().backward()
    close(xb.grad, xr.grad, atol_frac=3e-2)
    torch.testing.assert_close(bn.weight.grad, ref.weight.grad, rtol=3e-2, atol=3e-2 * ref.weight.grad.abs().max().item())
    torch.testing.assert_close(bn.bias.grad, ref.bias.grad, rtol=3e-2, atol=3e-2 * ref.bias.grad.abs().max().item())


@pytest.mark.parametrize("B,L,p", [(2, 130, 0.0), (3, 513, 0.1), (1, 17, 0.0)])
def test_attention_bwd_fused_bias_grad(dev, B, L, p):
    """the Q/K/V bias-gradient column sums emitted by the backward kernels equal the
    column sums of the dQKV they write (f32 accumulators vs bf16-stored rows)"""
    k = K()
    qkv, km = make_attn_inputs(dev, B, L, pad=True, seed=21, scale=1.0)
    O = torch.empty(B * L, 768, dtype=torch.bfloat16, device=dev)
    lse = torch.empty(B * 12, L, device=dev)
    dm = k.dropmask_empty(B, L, 12, dev) if p > 0 else None
    k.attention_fwd(qkv, km, O, lse, B, L, drop_p=p, seed=5, dropmask=dm)
    dO = rnd(B * L, 768, dev=dev, seed=22)
    dqkv = torch.zeros(B * L, 2304, dtype=torch.bfloat16, device=dev)
    delta = torch.empty(B * 12, L, device=dev)
    parts = k.attention_dbias_parts(B, L, 12, dev).fill_(float("nan"))  # every element must be written
    k.attention_bwd(qkv, km, O, dO, lse, delta, dqkv, B, L, drop_p=p, seed=5, dropmask=dm, dbias_parts=parts)
    assert not torch.isnan(parts).any()
    g = torch.full((2304,), 0.5, device=dev)
    k.attention_dbias_reduce(parts, B, L, g)
    ref = dqkv.float().sum(0) + 0.5
    torch.testing.assert_close(g, ref, rtol=1e-2, atol=1e-2 * ref.abs().max().item())


def _keep_bits_formula(seed, bh, q, L, p):
    """the attention dropout stream restated (attention.hip seed_for / lowbias32 / pair_draw and the
    tile body's register layout): keep decision of every key of query row q, head-row bh"""
    M32 = 0xFFFFFFFF

    def lowbias32(x):
        x = np.asarray(x, dtype=np.uint64) & M32
        x ^= x >> 16
        x = (x * 0x7FEB352D) & M32
        x ^= x >> 15
        x = (x * 0x846CA68B) & M32
        x ^= x >> 16
        return x

    mul = [0x9E3779, 0x85EBCB, 0xC2B2AF, 0xA7D4EB, 0x965667, 0xD3A265, 0xFD7047, 0xB55A4F]
    sbh = int(lowbias32((seed & M32) ^ int(lowbias32(((seed >> 32) + 0x9E3779B9 * (bh + 1)) & M32))))
    nkv = (L + 63) // 64
    thr = int(p * 65536.0 + 0.5)
    k = np.arange(nkv * 64, dtype=np.uint64)
    hb = lowbias32(sbh + 4 * q * nkv + 2 * ((k >> 4) & 1) + 4 * (k >> 6) + ((k >> 5) & 1))
    i = (k & 15) >> 1
    src = np.where(i > 0, ((hb >> (4 * i)) | (hb << (32 - 4 * i))) & M32, hb)
    x = ((src & 0xFFFFFF) * np.array(mul, dtype=np.uint64)[i]) & M32
    hsh = x ^ (x >> 16)
    return np.where(k & 1, hsh >= (thr << 16), (hsh & 0xFFFF) >= thr)[:L]


@pytest.mark.parametrize("L", [513, 390])
def test_attention_dropout_tail_rows_follow_the_stream(dev, L):
    """The forward's keep words are the restated dropout stream bit for bit (attention.hip
    seed_for / pair_draw over the tile body's register layout), for rows of full query blocks and
    for the rows past the last full 128-row block (L = 513: one; 390: six); O / LSE of those tail
    rows against fp32 with the decoded mask.  (Round 6 used it to check a folded-tail forward,
    profiles/r6_attn_tailfold_ab.txt: the stream is what the backward's bits must match.)"""
    k = K()
    B, p, seed = 2, 0.1, 0x5EED1234ABCD
    qkv, km = make_attn_inputs(dev, B, L, pad=True, seed=31, scale=1.0)
    O = torch.empty(B * L, 768, dtype=torch.bfloat16, device=dev)
    lse = torch.empty(B * 12, L, device=dev)
    dm = k.dropmask_empty(B, L, 12, dev)
    k.attention_fwd(qkv, km, O, lse, B, L, drop_p=p, seed=seed, dropmask=dm)
    mask = k.dropmask_dense(dm, L).view(B * 12, L, L).cpu().numpy().astype(bool)
    tail0 = 128 * (L // 128)
    for bh in (0, 13, B * 12 - 1):
        for q in (0, 127, tail0 - 1) + tuple(range(tail0, L)):
            assert np.array_equal(mask[bh, q], _keep_bits_formula(seed, bh, q, L, p)), (bh, q)
    o_ref, lse_ref = attn_ref(qkv, km, B, L, dropmask=torch.from_numpy(mask).to(dev).view(B, 12, L, L).float(), p=p)
    rows = torch.cat([torch.arange(b * L + tail0, (b + 1) * L) for b in range(B)]).to(dev)
    close(O[rows], o_ref[rows], atol_frac=2e-2)
    torch.testing.assert_close(lse[:, tail0:], lse_ref[:, tail0:], rtol=1e-4, atol=2e-3)


@pytest.mark.parametrize("B,T", [(1, 16), (3, 17), (20, 9)])
def test_embed_bwd_matches_autograd(dev, B, T):
    """mmu_embed_bwd (round 6: position-major, position / type / [CLS] / [SEP] sums per wave and
    per block, no f32 copy of the row gradients) against autograd of the same embedding + LN in
    fp32: word (incl. [CLS] / [SEP] rows), position, token-type, LN weight / bias and image
    projection gradients.  (1, 16): S = 21 positions, a 1-wave last position group; (20, 9): two
    sample chunks per position group."""
    k = K()
    torch.manual_seed(B * 100 + T)
    n, V, H, cls_id, sep_id, eps = 3, 300, 768, 101, 102, 1e-12
    word, pos, typ = (torch.randn(V, H, device=dev) * 0.05, torch.randn(512, H, device=dev) * 0.05,
                      torch.randn(2, H, device=dev) * 0.05)
    lw, lb = 1 + 0.1 * torch.randn(H, device=dev), 0.1 * torch.randn(H, device=dev)
    proj = torch.randn(B, n, H, device=dev) * 0.05
    ids = torch.randint(200, V, (B, T), device=dev)
    seg = torch.randint(0, 2, (B, T), device=dev)
    S = n + 2 + T
    X = torch.empty(B * S, H, dtype=torch.bfloat16, device=dev)
    km = torch.empty(B, S, device=dev)
    mean, rstd = torch.empty(B * S, device=dev), torch.empty(B * S, device=dev)
    k.embed_fwd(ids, seg, torch.ones_like(ids), proj, word, pos, typ, lw, lb, eps, cls_id, sep_id, None, 1, B, T, n, S,
                X, km, mean, rstd)
    G = (torch.randn(B * S, H, device=dev)).to(torch.bfloat16)
    grads = [torch.zeros_like(t) for t in (word, pos, typ, lw, lb)]
    d_proj = torch.empty_like(proj)
    k.embed_bwd(G, ids, seg, proj, word, pos, typ, lw, mean, rstd, cls_id, sep_id, B, T, n, *grads, d_proj)
    # fp32 autograd reference of the same rows
    leaves = [t.clone().requires_grad_(True) for t in (word, pos, typ, lw, lb, proj)]
    w_, p_, t_, lw_, lb_, pr_ = leaves
    rows = []
    for b in range(B):
        rows.append(w_[cls_id] + p_[0] + t_[0])
        for s in range(n):
            rows.append(pr_[b, s] + p_[1 + s] + t_[0])
        rows.append(w_[sep_id] + p_[n + 1] + t_[0])
        for t in range(T):
            rows.append(w_[ids[b, t]] + p_[t] + t_[seg[b, t]])
    e = torch.stack(rows)
    y = torch.nn.functional.layer_norm(e, (H,), lw_, lb_, eps)
    (y * G.float()).sum().backward()
    for got, ref, name in zip(grads + [d_proj], [l_.grad for l_ in leaves], ("word", "pos", "type", "ln_w", "ln_b",
                                                                          "proj")):
        torch.testing.assert_close(got, ref, rtol=2e-3, atol=2e-3 * ref.abs().max().item(), msg=name)


def test_colsum_reduce_multi_matches_sums(dev):
    """mmu_colsum_reduce_multi (round 6): up to 4 column-sum reductions of one width in one launch,
    each with its own row count, accumulating into its own output -- the per-job sums of the
    partial rows, as separate mmu_colsum_reduce calls give them."""
    from src import kernels as K
    torch.manual_seed(0)
    N_ = 768
    parts = [torch.randn(r, N_, device=dev) for r in (5, 1, 37, 16)]
    outs = [torch.randn(N_, device=dev) for _ in parts]
    want = [o + p.sum(0) for o, p in zip(outs, parts)]
    K.colsum_reduce_multi(list(zip(parts, outs)), accumulate=True)
    for o, w in zip(outs, want):
        torch.testing.assert_close(o, w, rtol=1e-5, atol=1e-4)
    outs2 = [torch.randn(N_, device=dev) for _ in parts[:2]]
    K.colsum_reduce_multi(list(zip(parts[:2], outs2)))
    for o, p in zip(outs2, parts[:2]):
        torch.testing.assert_close(o, p.sum(0), rtol=1e-5, atol=1e-4)


# ---------------------------------------------------------------- 256 x 384 tiling (round 6)
@pytest.fixture
def wide_gemm(monkeypatch):
    """route every eligible product (both operands K-major, N % 384 == 0) to gemm_wide_kernel"""
    monkeypatch.setenv("MMU_GEMM_WIDE", "2")  # (2: the dGELU product too)
    monkeypatch.setenv("MMU_GEMM_WIDE_MIN_TILES", "1")


@pytest.mark.parametrize("M,N,Kd", [(256 * 257, 768, 3072), (16416, 3072, 768), (256 * 65 + 32, 768, 2304),
                                     (16416, 2304, 768)])
def test_gemm_wide_tail_round_shapes(dev, wide_gemm, M, N, Kd):
    test_gemm_tail_round_shapes(dev, M, N, Kd)


@pytest.mark.parametrize("M,N", [(256 * 257, 768), (256 * 64 + 32, 3072)])
def test_gemm_wide_epilogues_exact_first_and_last_tile_rows(dev, wide_gemm, M, N):
    test_gemm_epilogues_exact_first_and_last_tile_rows(dev, M, N)


def test_gemm_wide_streams_and_batches(dev, wide_gemm):
    test_gemm_many_tiles_every_element(dev, True, True)
    test_gemm_bias_dropout_residual_f32_stream(dev)
    test_gemm_residual_recomputed_layernorm(dev)
    test_gemm_partial_last_wave(dev, 768)


@pytest.mark.parametrize("M,N,Kd", [(256 * 129 + 96, 768, 768), (4096, 3072, 768), (2 * 1536, 2304, 768)])
def test_gemm_wide_bitwise_equals_big_tiles(dev, monkeypatch, M, N, Kd):
    """Every output element accumulates the same 16x16x32 MFMAs in the same k order on both
    tilings, so the 256 x 384 kernel's results equal the 256 x 256 kernel's bit for bit, for
    every epilogue (dropout draws by global element index, colsum by float atomics excepted:
    those are compared to a tolerance)."""
    k = K()
    A, B = rnd(M, Kd, dev=dev, seed=151), rnd(N, Kd, dev=dev, seed=152, scale=0.1)
    bias = torch.randn(N, device=dev) * 0.1
    R16 = rnd(M, N, dev=dev, seed=153)
    S = torch.randn(M, N, device=dev) * 2.0 + 0.7
    mean = S.mean(-1).contiguous()
    rstd = torch.rsqrt(S.var(-1, unbiased=False) + 1e-12).contiguous()
    w, b = torch.randn(N, device=dev), torch.randn(N, device=dev)
    aux_in = (torch.rand(M, N, device=dev) + 0.5).to(torch.bfloat16)

    def run():
        outs = []
        o = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        k.gemm(A, Kd, True, B, Kd, True, o, N, M, N, Kd, epi=k.epilogue(k.EPI_STORE, bias=bias))
        outs.append(o)
        o, z = torch.empty(M, N, dtype=torch.bfloat16, device=dev), torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        k.gemm(A, Kd, True, B, Kd, True, o, N, M, N, Kd, epi=k.epilogue(k.EPI_BIAS_GELU, bias=bias, aux=z))
        outs += [o, z]
        f = torch.empty(M, N, dtype=torch.float32, device=dev)
        k.gemm(A, Kd, True, B, Kd, True, f, N, M, N, Kd,
               epi=k.epilogue(k.EPI_BIAS_DROP_RES, bias=bias, residual=S, drop_p=0.1, seed=9, res_ln=(mean, rstd, w, b)))
        outs.append(f)
        o = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        k.gemm(A, Kd, True, B, Kd, True, o, N, M, N, Kd,
               epi=k.epilogue(k.EPI_BIAS_DROP_RES, bias=bias, residual=R16, drop_p=0.1, seed=10))
        outs.append(o)
        o, cs = torch.empty(M, N, dtype=torch.bfloat16, device=dev), torch.zeros(N, device=dev)
        k.gemm(A, Kd, True, B, Kd, True, o, N, M, N, Kd, epi=k.epilogue(k.EPI_DGELU, aux=aux_in, colsum=cs))
        outs += [o]
        o = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        k.gemm(A, Kd, True, B, Kd, True, o, N, M, N, Kd, epi=k.epilogue(k.EPI_ADD_RES, residual=R16))
        outs.append(o)
        f = torch.full((M, N), 0.5, dtype=torch.float32, device=dev)
        k.gemm(A, Kd, True, B, Kd, True, f, N, M, N, Kd, epi=k.epilogue(k.EPI_STORE, accumulate=True))
        outs.append(f)
        torch.cuda.synchronize()
        return outs, cs

    monkeypatch.setenv("MMU_GEMM_TAIL", "0")  # (the split tail sums K in another order)
    monkeypatch.setenv("MMU_GEMM_WIDE", "0")
    ref, cs_ref = run()
    monkeypatch.setenv("MMU_GEMM_WIDE", "2")
    monkeypatch.setenv("MMU_GEMM_WIDE_MIN_TILES", "1")
    got, cs_got = run()
    for i, (g, r) in enumerate(zip(got, ref)):
        assert torch.equal(g, r), f"output {i} differs: max {(g.float() - r.float()).abs().max().item():.3e}"
    torch.testing.assert_close(cs_got, cs_ref, rtol=1e-4, atol=1e-4 * cs_ref.abs().max().item())


@pytest.mark.parametrize("wide", ["0", "2"])
@pytest.mark.parametrize("M,N,Kd", [(256 * 257, 768, 3072), (256 * 64 + 32, 3072, 768), (256 * 65 + 32, 768, 2304)])
def test_gemm_split_tail_matches_whole_tiles(dev, monkeypatch, wide, M, N, Kd):
    """The split tail rows (the last tile row of a nearly empty last round as split-K partial
    products + splitk_epilogue_kernel) against the same product on whole tiles
    (MMU_GEMM_TAIL=0): every epilogue kind, on the tail rows and on all rows; only the f32 sum
    order of the K slices differs, so f32 outputs agree to f32 rounding and bf16 outputs to one
    bf16 rounding step.  Dropout keeps are the same draws (global element index)."""
    k = K()
    monkeypatch.setenv("MMU_GEMM_WIDE", wide)
    monkeypatch.setenv("MMU_GEMM_WIDE_MIN_TILES", "1")
    A, B = rnd(M, Kd, dev=dev, seed=161), rnd(N, Kd, dev=dev, seed=162, scale=0.1)
    bias = torch.randn(N, device=dev) * 0.1
    R16 = rnd(M, N, dev=dev, seed=163)
    S = torch.randn(M, N, device=dev) * 2.0 + 0.7
    mean = S.mean(-1).contiguous()
    rstd = torch.rsqrt(S.var(-1, unbiased=False) + 1e-12).contiguous()
    w, b = torch.randn(N, device=dev), torch.randn(N, device=dev)
    aux_in = (torch.rand(M, N, device=dev) + 0.5).to(torch.bfloat16)

    def run():
        outs = []
        o = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        k.gemm(A, Kd, True, B, Kd, True, o, N, M, N, Kd, epi=k.epilogue(k.EPI_STORE, bias=bias))
        outs.append(o)
        o, z = torch.empty(M, N, dtype=torch.bfloat16, device=dev), torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        k.gemm(A, Kd, True, B, Kd, True, o, N, M, N, Kd, epi=k.epilogue(k.EPI_BIAS_GELU, bias=bias, aux=z))
        outs += [o, z]
        f = torch.empty(M, N, dtype=torch.float32, device=dev)
        k.gemm(A, Kd, True, B, Kd, True, f, N, M, N, Kd,
               epi=k.epilogue(k.EPI_BIAS_DROP_RES, bias=bias, residual=S, drop_p=0.1, seed=9, res_ln=(mean, rstd, w, b)))
        outs.append(f)
        o, cs = torch.empty(M, N, dtype=torch.bfloat16, device=dev), torch.zeros(N, device=dev)
        k.gemm(A, Kd, True, B, Kd, True, o, N, M, N, Kd, epi=k.epilogue(k.EPI_DGELU, aux=aux_in, colsum=cs))
        outs.append(o)
        o = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        k.gemm(A, Kd, True, B, Kd, True, o, N, M, N, Kd, epi=k.epilogue(k.EPI_ADD_RES, residual=R16))
        outs.append(o)
        f2 = torch.full((M, N), 0.5, dtype=torch.float32, device=dev)
        k.gemm(A, Kd, True, B, Kd, True, f2, N, M, N, Kd, epi=k.epilogue(k.EPI_STORE, accumulate=True))
        outs.append(f2)
        torch.cuda.synchronize()
        return outs, cs

    monkeypatch.setenv("MMU_GEMM_TAIL", "0")
    ref, cs_ref = run()
    monkeypatch.setenv("MMU_GEMM_TAIL", "2")  # (2: the 256 x 256 tiling too)
    got, cs_got = run()
    tail = slice(M - 256, M)
    for i, (g, r) in enumerate(zip(got, ref)):
        g, r = g.float(), r.float()
        assert torch.equal(g[: M - 256], r[: M - 256]), f"output {i}: rows before the tail changed"
        if i in (3, 6):  # f32 outputs
            torch.testing.assert_close(g[tail], r[tail], rtol=1e-5, atol=1e-5 * r.abs().max().item())
        else:
            torch.testing.assert_close(g[tail], r[tail], rtol=1e-2, atol=1e-2 * r.abs().max().item())
    torch.testing.assert_close(cs_got, cs_ref, rtol=1e-4, atol=1e-4 * cs_ref.abs().max().item())


@pytest.mark.parametrize("M,N,Kd,wide", [(256 * 257, 3072, 768, "1"), (300, 256, 128, "1"), (256 * 64 + 32, 3072, 768, "2"),
                                         (256 * 257, 768, 3072, "2")])
def test_gemm_colsum_partial_rows_match_atomics(dev, monkeypatch, M, N, Kd, wide):
    """Column sums of the dGELU product as per-wave-block partial rows folded by one reduce launch
    (the default) against the float-atomic epilogue (MMU_GEMM_CS_PART=0), on the 256 x 256, small,
    wide and split-tail paths; the accumulate semantics (the sums are ADDED to colsum) kept."""
    k = K()
    monkeypatch.setenv("MMU_GEMM_WIDE", wide)
    monkeypatch.setenv("MMU_GEMM_WIDE_MIN_TILES", "1")
    A, B = rnd(M, Kd, dev=dev, seed=171), rnd(N, Kd, dev=dev, seed=172, scale=0.1)
    aux = (torch.rand(M, N, device=dev) + 0.5).to(torch.bfloat16)
    outs = []
    for flag in ("0", "1"):
        monkeypatch.setenv("MMU_GEMM_CS_PART", flag)
        o, cs = torch.empty(M, N, dtype=torch.bfloat16, device=dev), torch.full((N,), 1.0, device=dev)
        k.gemm(A, Kd, True, B, Kd, True, o, N, M, N, Kd, epi=k.epilogue(k.EPI_DGELU, aux=aux, colsum=cs))
        outs.append((o, cs))
    assert torch.equal(outs[0][0], outs[1][0])
    dg = (A.float() @ B.float().t()) * aux.float()
    for _, cs in outs:
        torch.testing.assert_close(cs, dg.sum(0) + 1.0, rtol=2e-3, atol=2e-3 * dg.abs().sum(0).max().item())
    torch.testing.assert_close(outs[1][1], outs[0][1], rtol=1e-4, atol=1e-4 * outs[0][1].abs().max().item())
