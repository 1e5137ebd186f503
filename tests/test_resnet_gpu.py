"""ResNet-152 Bottleneck on the bf16 training path (src/resnet.py): the 1x1 stride-1 convs on
mmu_gemm (forward, dX with the identity-skip gradient added in the GEMM epilogue, dW into
the f32 gradient) against the same block with every conv product on MIOpen and autograd
summing the skip gradient.  Shapes are chosen so that every branch of _mmu_1x1 runs:
  1024 -> 256 at 14x14, batch 128 (M = 25088): fwd, dX + skip, dW on conv1 and conv3
  256 -> 64 at 56x56, batch 4 (M = 12544): conv1 dX + skip with K = 64; the rest MIOpen
Yardstick: the same block in fp32 (PyTorch convs and batch norm) is the truth; the mmu
path's relative Frobenius error against it must be within 1.25x (+1e-3) of the all-MIOpen
bf16 path's own error.  (A fixed bound on the bf16-vs-bf16 difference is the wrong test:
both engines round, three BatchNorm backwards amplify it through their mean subtraction,
and a few ReLU masks flip at pre-activations near 0, so the difference sits at 2-3 % either
way; a max-error bound is worse still, one flipped element moves its whole gradient.)
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


class _Store:
    """stand-in for the parameter store: bf16 channels-last copies of the conv filters"""

    def __init__(self, mod):
        self.w = {n: p.detach().to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
                  for n, p in mod.named_parameters() if p.dim() == 4}

    def compute_of(self, name):
        return self.w[name]


def _run(block, x, g, fp32=False):
    from src import resnet as R
    xx = (x.float() if fp32 else x).clone().requires_grad_(True)
    for p in block.parameters():
        p.grad = None
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=not fp32):
        used_sink = block.downsample is None and block.conv1.takes_skip_grad(xx)
        y = block(xx)
    y.float().backward(g)
    assert isinstance(block.conv1, R.StoreConv2d)
    return y.float(), xx.grad.float(), {n: p.grad.float().clone() for n, p in block.named_parameters()}, used_sink


def _rel(a, b):
    return (a - b).double().norm().item() / (b.double().norm().item() + 1e-12)


def _no_worse(mmu, miopen, ref, what, slack=1.25, eps=1e-3):
    e1, e0 = _rel(mmu, ref), _rel(miopen, ref)
    assert e1 <= slack * e0 + eps, f"{what}: mmu path error {e1:.3e} vs MIOpen path error {e0:.3e} (fp32 truth)"


def _close(a, b, what, frac=2e-2):
    err = (a - b).double().norm().item()
    scale = b.double().norm().item() + 1e-12
    assert err <= frac * scale, f"{what}: |err| {err:.3e} vs |ref| {scale:.3e}"


@pytest.mark.parametrize("n,cin,cout,h,w", [(2, 256, 256, 14, 14), (3, 512, 128, 7, 5), (1, 256, 384, 9, 11),
                                             (16, 256, 256, 14, 14)])
def test_conv3x3_wgrad_matches_torch(dev, n, cin, cout, h, w):
    """mmu_conv3x3_wgrad (implicit im2col in the GEMM's B-operand DMA, split-K over pixels)
    against torch's fp32 conv weight gradient on the same bf16 inputs; accumulate and store."""
    from src import kernels as K
    cl = torch.channels_last
    g = torch.Generator(device=dev).manual_seed(cin + h)
    x = torch.randn(n, cin, h, w, generator=g, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
    dy = torch.randn(n, cout, h, w, generator=g, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
    ref = torch.nn.grad.conv2d_weight(x.float(), (cout, cin, 3, 3), dy.float(), stride=1, padding=1)
    dw = torch.full((cout, cin, 3, 3), 0.5, device=dev).contiguous(memory_format=cl)
    K.conv3x3_wgrad(dy, x, dw, accumulate=True)
    _close(dw - 0.5, ref, "dW accumulate", frac=1e-4)
    dw2 = torch.empty((cout, cin, 3, 3), device=dev).contiguous(memory_format=cl)
    K.conv3x3_wgrad(dy, x, dw2)
    _close(dw2, ref, "dW", frac=1e-4)
    assert (dw2 - ref).abs().max().item() <= 1e-3 * ref.abs().max().item()


@pytest.mark.parametrize("n,h,w", [(2, 224, 224), (3, 37, 53), (1, 7, 130), (5, 16, 16)])
def test_stem_conv_matches_torch(dev, n, h, w):
    """mmu_stem_conv_fwd / _wgrad (the 7x7 / stride-2 / pad-3 stem, 3 -> 64, LDS patch +
    16x16x32 MFMAs over taps padded to 4 channels) against torch's fp32 conv and conv weight
    gradient on the same bf16 inputs: full 224 images, odd sizes (partial column tiles, odd
    output rows), a single output row pair; accumulate and store."""
    from src import kernels as K
    cl = torch.channels_last
    g = torch.Generator(device=dev).manual_seed(h * w + n)
    x = torch.randn(n, 3, h, w, generator=g, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
    wt = (torch.randn(64, 3, 7, 7, generator=g, device=dev) * 0.1).to(torch.bfloat16).contiguous(memory_format=cl)
    ho, wo = (h - 1) // 2 + 1, (w - 1) // 2 + 1
    y = torch.full((n, 64, ho, wo), 7.0, dtype=torch.bfloat16, device=dev).contiguous(memory_format=cl)
    K.stem_conv_fwd(x, wt, y)
    ref = torch.nn.functional.conv2d(x.float(), wt.float(), stride=2, padding=3)
    assert y.shape == ref.shape
    assert (y.float() - ref).abs().max().item() <= 1e-2 * ref.abs().max().item()
    _close(y.float(), ref, "stem fwd", frac=5e-3)
    dy = torch.randn(n, 64, ho, wo, generator=g, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
    rdw = torch.nn.grad.conv2d_weight(x.float(), (64, 3, 7, 7), dy.float(), stride=2, padding=3)
    dw = torch.full((64, 3, 7, 7), 0.5, device=dev).contiguous(memory_format=cl)
    K.stem_conv_wgrad(dy, x, dw, accumulate=True)
    _close(dw - 0.5, rdw, "stem dW accumulate", frac=1e-4)
    dw2 = torch.empty((64, 3, 7, 7), device=dev).contiguous(memory_format=cl)
    K.stem_conv_wgrad(dy, x, dw2)
    assert (dw2 - rdw).abs().max().item() <= 1e-3 * rdw.abs().max().item()


@pytest.mark.parametrize("n,cin,cout,h,w", [(2, 256, 256, 14, 14), (3, 512, 512, 7, 13), (4, 64, 384, 9, 11),
                                             (16, 256, 256, 14, 14), (96, 256, 256, 28, 28), (4, 128, 128, 28, 28)])
def test_conv3x3_implicit_matches_torch(dev, n, cin, cout, h, w):
    """mmu_conv3x3_implicit (im2col gathered in the A-operand DMA) as the 3x3 conv forward
    (filter as stored, channels-last) and as its data gradient (flipped filter transposed to
    [Cin][3][3][Cout]) against torch's fp32 conv on the same bf16 inputs.  96 x 28 x 28:
    294 tiles, more than one wave of tiles on 256 CUs."""
    from src import kernels as K
    cl = torch.channels_last
    g = torch.Generator(device=dev).manual_seed(cin + w)
    x = torch.randn(n, cin, h, w, generator=g, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
    wt = (torch.randn(cout, cin, 3, 3, generator=g, device=dev) * 0.05).to(torch.bfloat16).contiguous(memory_format=cl)
    y = torch.empty(n, cout, h, w, dtype=torch.bfloat16, device=dev).contiguous(memory_format=cl)
    K.conv3x3_implicit(x, wt, y)
    ref = torch.nn.functional.conv2d(x.float(), wt.float(), padding=1)
    _close(y.float(), ref, "conv fwd", frac=5e-3)
    assert (y.float() - ref).abs().max().item() <= 1e-2 * ref.abs().max().item()
    if cin % 128 == 0:  # the data-gradient routes (_mmu_conv: layer2..4)
        dy = torch.randn(n, cout, h, w, generator=g, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
        dx = torch.empty_like(x)
        K.conv3x3_implicit(dy, wt.flip(2, 3).permute(1, 2, 3, 0).contiguous(), dx)
        rdx = torch.nn.grad.conv2d_input(x.shape, wt.float(), dy.float(), padding=1)
        _close(dx.float(), rdx, "conv dX", frac=5e-3)


@pytest.mark.parametrize("n,cin,cout,h,k,s", [(4, 128, 128, 28, 3, 2), (2, 256, 256, 28, 3, 2), (6, 512, 512, 13, 3, 2),
                                               (8, 64, 64, 16, 3, 2), (5, 256, 512, 15, 1, 2), (16, 512, 1024, 28, 1, 2),
                                               (8, 1024, 2048, 14, 1, 2)])
def test_strided_conv_matches_torch(dev, n, cin, cout, h, k, s):
    """mmu_conv_implicit / mmu_conv_wgrad on the strided convs of ResNet-152 (first block of
    layer2..4: conv2 3x3 / stride 2 / pad 1, downsample 1x1 / stride 2) against torch's fp32
    conv and conv weight gradient on the same bf16 inputs: the trunk's shapes, odd maps
    (partial output rows), the narrow 128x128-tile forward (Cout < 256), split-K filter
    gradients (many pixels) and unsplit ones (few)."""
    from src import kernels as K
    cl = torch.channels_last
    pad = k // 2
    g = torch.Generator(device=dev).manual_seed(cin * 7 + h + k)
    x = torch.randn(n, cin, h, h, generator=g, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
    wt = (torch.randn(cout, cin, k, k, generator=g, device=dev) * 0.05).to(torch.bfloat16).contiguous(memory_format=cl)
    ref = torch.nn.functional.conv2d(x.float(), wt.float(), stride=s, padding=pad)
    y = torch.full(ref.shape, 3.0, dtype=torch.bfloat16, device=dev).contiguous(memory_format=cl)
    K.conv_implicit(x, wt, y, k, s)
    _close(y.float(), ref, "strided conv fwd", frac=5e-3)
    assert (y.float() - ref).abs().max().item() <= 1e-2 * ref.abs().max().item()
    if cin % 256 == 0 and cout % 128 == 0:
        dy = torch.randn(ref.shape, generator=g, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
        rdw = torch.nn.grad.conv2d_weight(x.float(), wt.shape, dy.float(), stride=s, padding=pad)
        dw = torch.full(wt.shape, 0.25, device=dev).contiguous(memory_format=cl)
        K.conv_wgrad(dy, x, dw, k, s, accumulate=True)
        _close(dw - 0.25, rdw, "strided conv dW accumulate", frac=1e-3)
        dw2 = torch.empty(wt.shape, device=dev).contiguous(memory_format=cl)
        K.conv_wgrad(dy, x, dw2, k, s)
        _close(dw2, rdw, "strided conv dW", frac=1e-3)


@pytest.mark.parametrize("cin,width,hw,batch", [(1024, 256, 14, 128), (256, 64, 56, 4)])
def test_bottleneck_mmu_1x1_matches_miopen(dev, monkeypatch, cin, width, hw, batch):
    from src import resnet as R
    torch.manual_seed(0)
    block = R.Bottleneck(cin, width, 1)
    for m in block.modules():
        if isinstance(m, torch.nn.Conv2d):
            torch.nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
    block = block.to(dev).train()
    store = _Store(block)
    for n, m in block.named_modules():
        if isinstance(m, R.StoreConv2d):
            m.attach_compute(store, f"{n}.weight")
    g = torch.Generator().manual_seed(1)
    x = torch.randn(batch, cin, hw, hw, generator=g).clamp_(min=0).to(dev).to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    gy = torch.randn(batch, cin, hw, hw, generator=g).to(dev).contiguous(memory_format=torch.channels_last)
    M = batch * hw * hw
    assert R._mmu_1x1(cin, width, M, hw)[1]
    y1, dx1, gr1, sink1 = _run(block, x, gy)
    assert sink1, "the identity-skip gradient must go through conv1's dX GEMM"
    monkeypatch.setattr(R, "_mmu_1x1", lambda *a: (False, False, False))
    y0, dx0, gr0, sink0 = _run(block, x, gy)
    assert not sink0
    yr, dxr, grr, _ = _run(block, x, gy, fp32=True)
    _close(y1, yr, "output vs fp32", frac=2e-2)
    _no_worse(y1, y0, yr, "output")
    _no_worse(dx1, dx0, dxr, "input grad")
    for n in gr0:
        _no_worse(gr1[n], gr0[n], grr[n], f"grad {n}")


@pytest.mark.parametrize("shape", [(4, 64, 112, 112), (3, 16, 7, 9)])
def test_stem_maxpool_matches_torch(dev, shape):
    """MaxPool2d(3, 2, 1) (torchvision resnet child 3) on mmu_maxpool_fwd/bwd vs torch's
    max_pool2d on the same bf16 channels-last input: forward bit-exact (first maximum wins
    ties; post-ReLU maps are full of ties at 0), backward: the gradient of every window goes
    to the same element (sums of <= 4 bf16 values in f32, rounded once)."""
    from src import resnet as R
    g = torch.Generator().manual_seed(3)
    x = torch.randn(shape, generator=g).clamp_(min=0)
    x = (x * 4).round_() / 4                              # many exact ties
    x = x.to(dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    pool = R.MaxPool2d(3, 2, 1)
    y = pool(x)
    ref_x = x.detach().clone().requires_grad_(True)
    ref = torch.nn.functional.max_pool2d(ref_x, 3, 2, 1)
    assert y.shape == ref.shape and y.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(y.float(), ref.float())
    gy = torch.randn(ref.shape, generator=g).to(dev).to(torch.bfloat16)
    y.backward(gy)
    ref.backward(gy)
    torch.testing.assert_close(x.grad.float(), ref_x.grad.float(), rtol=1e-2, atol=1e-2)
    assert (x.grad.float() != 0).sum() == (ref_x.grad.float() != 0).sum()


def test_model_grads_with_mmu_1x1_match_miopen(dev, monkeypatch):
    """Whole small MMBT (bf16 trunk, the bench precision) at batch 64: every ResNet weight
    gradient with the stem conv on mmu_stem_conv_* and the 1x1 products on mmu_gemm -- through the parameter store's bf16
    filter copies and channels-last f32 gradient views (layer3/4 dW at 14x14 and 7x7,
    dX, the 28x28 forward) -- against the all-MIOpen path, both measured against the fp32 trunk (_no_worse)."""
    from oracle.weights import SMALL, make_state_dict
    from src import resnet as R
    from src.mmbt import MultimodalBertClf
    from src.testing import small_args, synthetic_batch
    monkeypatch.setattr(torch.backends.cudnn, "deterministic", True)
    x, y = synthetic_batch(64, 16, vocab=SMALL.vocab, seed=9)
    x, y = tuple(t.to(dev) for t in x), y.to(dev)
    sd = make_state_dict(0, SMALL)
    assert R._mmu_1x1(1024, 512, 64 * 196, 14) == (False, True, True)

    def grads(precision="bf16"):
        torch.manual_seed(0)
        m = MultimodalBertClf(small_args(bert_hidden_dropout=0.0, bert_attn_dropout=0.0, dropout=0.0,
                                         img_precision=precision))
        m.load_state_dict(sd, strict=True)
        m = m.to(dev).train()
        m.store.zero_grad()
        loss = m.compute_loss(m(*x), y)
        loss.backward()
        return loss.item(), {n: p.grad.float().clone() for n, p in m.named_parameters() if "img_encoder" in n}

    l1, g1 = grads()
    monkeypatch.setattr(R, "_mmu_1x1", lambda *a: (False, False, False))
    monkeypatch.setattr(R, "_mmu_conv", lambda *a: (False, False, False))
    monkeypatch.setattr(R, "_is_stem", lambda *a: False)
    l0, g0 = grads()
    lr, gr = grads("fp32")                          # the trunk in fp32: the truth for both
    assert abs(l1 - lr) <= 1e-2 * abs(lr)
    for n in g0:
        if n.endswith("weight") and g0[n].dim() == 4:
            _no_worse(g1[n], g0[n], gr[n], f"grad {n}")


def test_model_grads_with_side_stream_wgrad(dev, monkeypatch):
    """The trunk's filter gradients on the side stream (src/resnet.py _wgrad_run, on from
    SIDE_WGRAD_MIN_BATCH images: forced on here) give the same gradients as the main-stream
    order, and every one of them is complete when backward() returns (the end-of-backward join)."""
    from oracle.weights import SMALL, make_state_dict
    from src import resnet as R
    from src.mmbt import MultimodalBertClf
    from src.testing import small_args, synthetic_batch
    monkeypatch.setattr(torch.backends.cudnn, "deterministic", True)
    x, y = synthetic_batch(8, 16, vocab=SMALL.vocab, seed=5)
    x, y = tuple(t.to(dev) for t in x), y.to(dev)
    sd = make_state_dict(0, SMALL)

    def grads():
        torch.manual_seed(0)
        m = MultimodalBertClf(small_args(bert_hidden_dropout=0.0, bert_attn_dropout=0.0, dropout=0.0))
        m.load_state_dict(sd, strict=True)
        m = m.to(dev).train()
        m.store.zero_grad()
        m.compute_loss(m(*x), y).backward()
        # no synchronize: the clones run on the main stream after the join.  The trunk's
        # gradients only (the text embeddings' scatter-add order is not deterministic)
        return {n: p.grad.clone() for n, p in m.named_parameters() if "img_encoder" in n}

    g0 = grads()
    monkeypatch.setattr(R, "SIDE_WGRAD_MIN_BATCH", 1)
    g1 = grads()
    for n in g0:
        err = (g1[n] - g0[n]).abs().max().item()
        assert err <= 1e-5 * g0[n].abs().max().item() + 1e-12, f"{n}: side-stream gradient differs by {err:.3e}"


@pytest.mark.parametrize("train", [True, False])
def test_stream_residue_carried_through_the_trunk(dev, monkeypatch, train):
    """The residual stream's 8-bit residue (resnet.STREAM_RESIDUE, csrc/batchnorm.hip) reaches
    every Bottleneck: each block output carries ``_mmu_res`` when the block returns (train and
    eval), the next block frees it, and with it the trunk's output map lies closer to the fp32
    trunk's than without it (the 4-block small trunk at batch 8: a small but systematic gain;
    the full model's measured in tests/test_mmbt_gpu.py)."""
    from oracle.weights import SMALL, make_state_dict
    from src import resnet as R
    from src.mmbt import MultimodalBertClf
    from src.testing import small_args, synthetic_batch
    monkeypatch.setattr(torch.backends.cudnn, "deterministic", True)
    (_, _, _, img), _ = synthetic_batch(8, 16, vocab=SMALL.vocab, seed=12)
    img = img.to(dev)
    sd = make_state_dict(0, SMALL)

    def trunk(precision, residue):
        monkeypatch.setattr(R, "STREAM_RESIDUE", residue)
        torch.manual_seed(0)
        m = MultimodalBertClf(small_args(img_precision=precision))
        m.load_state_dict(sd, strict=True)
        m = m.to(dev).train(train)
        seen = []
        blocks = [mod for mod in m.modules() if isinstance(mod, R.Bottleneck)]
        hooks = [b.register_forward_hook(lambda mod, i, o: seen.append(getattr(o, "_mmu_res", None) is not None))
                 for b in blocks]
        with torch.no_grad():
            out = m.enc.img_encoder.trunk(img).float()
        for h in hooks:
            h.remove()
        return out, seen, len(blocks)

    ref, _, _ = trunk("fp32", True)
    on, seen_on, nb = trunk("bf16", True)
    off, seen_off, _ = trunk("bf16", False)
    assert seen_on == [True] * nb and seen_off == [False] * nb
    e_on, e_off = _rel(on, ref), _rel(off, ref)
    print(f"\n[stream residue, train={train}] trunk output rel err vs fp32: with {e_on:.3e}, without {e_off:.3e}")
    assert not torch.equal(on, off)
    assert e_on < e_off


def test_batchnorm_momentum_none_cumulative_average_on_device(dev):
    """momentum=None (torch's cumulative moving average): the HIP pass takes 1 / num_batches_tracked
    on the device (no host read) and matches torch.nn.BatchNorm2d's running statistics
    over three training passes."""
    from src.resnet import BatchNorm2d
    torch.manual_seed(0)
    C = 64
    hip = BatchNorm2d(C, momentum=None).to(dev).train()
    ref = torch.nn.BatchNorm2d(C, momentum=None).to(dev).train()
    for it in range(3):
        x = torch.randn(4, C, 9, 7, device=dev) * (1 + it) + it
        xb = x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        with torch.no_grad():
            hip(xb)
            ref(xb.float())
    assert int(hip.num_batches_tracked) == 3 == int(ref.num_batches_tracked)
    torch.testing.assert_close(hip.running_mean, ref.running_mean, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(hip.running_var, ref.running_var, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("n,cin,cout,h,ks,st", [(256, 256, 256, 14, 3, 1), (4, 256, 256, 14, 3, 1),
                                               (24, 128, 128, 28, 3, 1), (8, 512, 512, 13, 3, 2), (8, 64, 64, 56, 3, 1),
                                               (16, 1024, 2048, 14, 1, 2)])
def test_conv_stats_epilogue_matches_output(dev, n, cin, cout, h, ks, st):
    """mmu_conv_implicit_stats (MMU_EPI_STORE_STATS, round 6): the BatchNorm statistics table the
    conv's epilogue writes -- {sum, sum of squares} per channel and 64-row block of the bf16
    output -- against the output itself; the big-tile, small-tile (128 channels) and split-K
    (few tiles: a stats pass after the reduction) paths."""
    from src import kernels as K
    torch.manual_seed(n + cin)
    cl = torch.channels_last
    x = torch.randn(n, cin, h, h, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
    w = (torch.randn(cout, cin, ks, ks, device=dev) * (cin * ks * ks) ** -0.5).to(torch.bfloat16)
    w = w.contiguous(memory_format=cl)
    ho = (h + 2 * (ks // 2) - ks) // st + 1
    y = torch.empty(n, cout, ho, ho, dtype=torch.bfloat16, device=dev, memory_format=cl)
    M = n * ho * ho
    table, nparts = K.bn_stats_table(M, cout, dev)
    K.conv_implicit(x, w, y, ks, st, stats=table)
    yr = y.permute(0, 2, 3, 1).reshape(M, cout).float()
    t = table.view(nparts, cout, 2)
    blocks = torch.nn.functional.pad(yr, (0, 0, 0, nparts * 64 - M)).view(nparts, 64, cout)
    torch.testing.assert_close(t[..., 0], blocks.sum(1), rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(t[..., 1], (blocks * blocks).sum(1), rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("M,C,Co", [(25088, 1024, 256), (25088, 512, 128), (200, 256, 256), (12544, 2048, 512)])
def test_gemm_stats_epilogue_and_bn_parts(dev, M, C, Co):
    """the 1x1 conv forward's STORE_STATS GEMM, then mmu_batchnorm_fwd_parts on its table: the same
    BatchNorm output / saved statistics / running statistics as mmu_batchnorm_fwd's own pass
    (big tiles; 128x128 tiles for 128 output channels or < 256 rows)."""
    from src import kernels as K
    torch.manual_seed(3)
    x = torch.randn(M, C, device=dev).to(torch.bfloat16)
    w = (torch.randn(Co, C, device=dev) * C ** -0.5).to(torch.bfloat16)
    y = torch.empty(M, Co, dtype=torch.bfloat16, device=dev)
    table, nparts = K.bn_stats_table(M, Co, dev)
    K.gemm(x, C, 1, w, C, 1, y, Co, M, Co, C, epi=K.epilogue(K.EPI_STORE_STATS, colsum=table))
    torch.testing.assert_close(y.float(), x.float() @ w.float().t(), rtol=2e-2, atol=2e-2)
    t = table.view(nparts, Co, 2).sum(0)
    torch.testing.assert_close(t[:, 0], y.float().sum(0), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(t[:, 1], (y.float() ** 2).sum(0), rtol=1e-4, atol=1e-2)
    Y4 = y.view(M, 1, 1, Co).permute(0, 3, 1, 2)  # channels-last [N, C, H, W] view of the rows
    outs = []
    for parts in (None, (table, nparts)):
        Yo = torch.empty_like(Y4)
        torch.manual_seed(5)
        wgt, bias = 1 + 0.1 * torch.randn(Co, device=dev), 0.1 * torch.randn(Co, device=dev)
        rm, rv = torch.zeros(Co, device=dev), torch.ones(Co, device=dev)
        sm, si = torch.empty(Co, device=dev), torch.empty(Co, device=dev)
        K.batchnorm_fwd(Y4, Yo, wgt, bias, rm, rv, True, 0.1, 1e-5, relu=True, save_mean=sm, save_invstd=si,
                        parts=parts)
        outs.append((Yo.float(), rm, rv, sm, si))
    for a, b in zip(outs[0], outs[1]):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-2 if a.dim() == 4 else 1e-6)


def _bnb_reference(dx_rows, x_rows, mask, mean):
    """the float2 [ceil(M/64)][C] table {sum g, sum g (x - mean)}, g = dx * relu bit (mmu.h *_BNB)"""
    M, C = dx_rows.shape
    bits = ((mask.view(M, C // 8, 1).int() >> torch.arange(8, device=mask.device, dtype=torch.int32)) & 1)
    g = dx_rows.float() * bits.reshape(M, C).float()
    h = g * (x_rows.float() - mean)
    nparts = (M + 63) // 64
    pad = nparts * 64 - M
    g = torch.nn.functional.pad(g, (0, 0, 0, pad)).view(nparts, 64, C).sum(1)
    h = torch.nn.functional.pad(h, (0, 0, 0, pad)).view(nparts, 64, C).sum(1)
    return g, h


def _bn_fwd_for_bnb(dev, n, C, hw, seed):
    from src import kernels as K
    torch.manual_seed(seed)
    cl = torch.channels_last
    x = (torch.randn(n, C, hw, hw, device=dev) * 2 + 0.5).to(torch.bfloat16).contiguous(memory_format=cl)
    Y = torch.empty_like(x)
    wgt, bias = 1 + 0.1 * torch.randn(C, device=dev), 0.1 * torch.randn(C, device=dev)
    rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    sm, si = torch.empty(C, device=dev), torch.empty(C, device=dev)
    mask = torch.empty(x.numel() // 8, dtype=torch.uint8, device=dev)
    K.batchnorm_fwd(x, Y, wgt, bias, rm, rv, True, 0.1, 1e-5, relu=True, save_mean=sm, save_invstd=si,
                    relu_mask=mask)
    return x, wgt, sm, si, mask


def _check_bn_bwd_parts(dev, dx4, x, wgt, sm, si, mask, table, nparts):
    """mmu_batchnorm_bwd_parts on the epilogue's table == mmu_batchnorm_bwd's own reduction"""
    from src import kernels as K
    C = x.shape[1]
    outs = []
    for parts in (None, (table, nparts)):
        dX = torch.empty_like(x)
        dw, db = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
        K.batchnorm_bwd(dx4, None, x, wgt, sm, si, True, dX, None, dw, db, relu_mask=mask, parts=parts)
        outs.append((dX.float(), dw, db))
    torch.testing.assert_close(outs[1][1], outs[0][1], rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(outs[1][2], outs[0][2], rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(outs[1][0], outs[0][0], rtol=1e-2, atol=1e-3)


@pytest.mark.parametrize("n,C,hw,K_,skip", [(32, 256, 28, 1024, False), (32, 256, 28, 1024, True),
                                            (2, 128, 7, 512, True), (8, 512, 7, 2048, False)])
def test_gemm_bnb_epilogue_and_bn_bwd_parts(dev, n, C, hw, K_, skip):
    """the 1x1 conv data gradient dX = dY.W with the STORE_BNB / ADD_RES_BNB epilogue (round 6): dX
    bit-identical to the plain STORE / ADD_RES product, the table = the BatchNorm backward's
    reduction {sum g, sum g (x - mean)} of dX, and mmu_batchnorm_bwd_parts on it = mmu_batchnorm_bwd
    (big 256x256 tiles, and the 128x128 tiles of a 98-row map)."""
    from src import kernels as K
    x, wgt, sm, si, mask = _bn_fwd_for_bnb(dev, n, C, hw, n + C + int(skip))
    M = n * hw * hw
    dyn = torch.randn(M, K_, device=dev).to(torch.bfloat16)
    w = (torch.randn(K_, C, device=dev) * K_ ** -0.5).to(torch.bfloat16)
    res = torch.randn(M, C, device=dev).to(torch.bfloat16) if skip else None
    plain = torch.empty(M, C, dtype=torch.bfloat16, device=dev)
    K.gemm(dyn, K_, 1, w, C, 0, plain, C, M, C, K_, epi=K.epilogue(K.EPI_ADD_RES, residual=res) if skip else None)
    dx = torch.empty(M, C, dtype=torch.bfloat16, device=dev)
    table, nparts = K.bn_stats_table(M, C, dev)
    kind = K.EPI_ADD_RES_BNB if skip else K.EPI_STORE_BNB
    K.gemm(dyn, K_, 1, w, C, 0, dx, C, M, C, K_, epi=K.epilogue(kind, residual=res, colsum=table, bn=(x, mask, sm)))
    assert torch.equal(dx, plain)
    g, h = _bnb_reference(dx, x.permute(0, 2, 3, 1).reshape(M, C), mask, sm)
    t = table.view(nparts, C, 2)
    torch.testing.assert_close(t[..., 0], g, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(t[..., 1], h, rtol=1e-4, atol=1e-3)
    _check_bn_bwd_parts(dev, dx.view(n, hw, hw, C).permute(0, 3, 1, 2), x, wgt, sm, si, mask, table, nparts)


@pytest.mark.parametrize("n,C,hw", [(32, 128, 28), (64, 256, 14), (4, 256, 14), (8, 512, 7), (8, 64, 56)])
def test_conv3x3_bnb_epilogue_and_bn_bwd_parts(dev, n, C, hw):
    """mmu_conv3x3_implicit_bnb (the 3x3 conv data gradient + the backward reduction of the
    BatchNorm before the conv, round 6): dX bit-identical to mmu_conv3x3_implicit, the table against
    dX, mmu_batchnorm_bwd_parts against mmu_batchnorm_bwd -- small tiles (128 channels), big tiles,
    and split-K maps (a reduction pass over dX after the slab sum)."""
    from src import kernels as K
    x, wgt, sm, si, mask = _bn_fwd_for_bnb(dev, n, C, hw, 7 * n + C)
    cl = torch.channels_last
    dyn = torch.randn(n, C, hw, hw, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
    wf = (torch.randn(C, 3, 3, C, device=dev) * (9 * C) ** -0.5).to(torch.bfloat16).contiguous()
    plain = torch.empty(n, C, hw, hw, dtype=torch.bfloat16, device=dev, memory_format=cl)
    K.conv3x3_implicit(dyn, wf, plain)
    dx = torch.empty_like(plain)
    M = n * hw * hw
    table, nparts = K.bn_stats_table(M, C, dev)
    K.conv3x3_implicit(dyn, wf, dx, bnb=(x, mask, sm), table=table)
    assert torch.equal(dx, plain)
    g, h = _bnb_reference(dx.permute(0, 2, 3, 1).reshape(M, C), x.permute(0, 2, 3, 1).reshape(M, C), mask, sm)
    t = table.view(nparts, C, 2)
    torch.testing.assert_close(t[..., 0], g, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(t[..., 1], h, rtol=1e-4, atol=1e-3)
    _check_bn_bwd_parts(dev, dx, x, wgt, sm, si, mask, table, nparts)


@pytest.mark.parametrize("bnb", [False, True])
def test_gemm_add_res_gated_by_relu_mask(dev, bnb):
    """ADD_RES / ADD_RES_BNB with res_mask (round 6): the residual gated element-wise by a ReLU mask --
    an identity Bottleneck's skip gradient dY3 * mask3 read inside conv1's dX epilogue -- equals the
    plain epilogue on the materialised product, bit for bit, and the BNB table follows the output."""
    from src import kernels as K
    from src.resnet import _mask_bits
    torch.manual_seed(11)
    n, C, hw, K_ = 8, 256, 14, 1024
    M = n * hw * hw
    x, wgt, sm, si, mask = _bn_fwd_for_bnb(dev, n, C, hw, 5)
    dy3 = torch.randn(n, C, hw, hw, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y3 = torch.randn(n, C, hw, hw, device=dev)
    mask3 = torch.empty(M * C // 8, dtype=torch.uint8, device=dev)
    # a ReLU mask from a real BN pass on an unrelated map
    xb = y3.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    K.batchnorm_fwd(xb, torch.empty_like(xb), None, None, None, None, True, 0.1, 1e-5, relu=True,
                    save_mean=torch.empty(C, device=dev), save_invstd=torch.empty(C, device=dev), relu_mask=mask3)
    g3 = (dy3 * _mask_bits(mask3, dy3)).contiguous(memory_format=torch.channels_last)
    rows = lambda t: t.permute(0, 2, 3, 1).reshape(M, C)
    dyn = torch.randn(M, K_, device=dev).to(torch.bfloat16)
    w = (torch.randn(K_, C, device=dev) * K_ ** -0.5).to(torch.bfloat16)
    plain = torch.empty(M, C, dtype=torch.bfloat16, device=dev)
    K.gemm(dyn, K_, 1, w, C, 0, plain, C, M, C, K_, epi=K.epilogue(K.EPI_ADD_RES, residual=rows(g3)))
    out = torch.empty_like(plain)
    if bnb:
        table, nparts = K.bn_stats_table(M, C, dev)
        epi = K.epilogue(K.EPI_ADD_RES_BNB, residual=rows(dy3), res_mask=mask3, colsum=table, bn=(x, mask, sm))
    else:
        epi = K.epilogue(K.EPI_ADD_RES, residual=rows(dy3), res_mask=mask3)
    K.gemm(dyn, K_, 1, w, C, 0, out, C, M, C, K_, epi=epi)
    assert torch.equal(out, plain)
    if bnb:
        g, h = _bnb_reference(out, rows(x), mask, sm)
        t = table.view(nparts, C, 2)
        torch.testing.assert_close(t[..., 0], g, rtol=1e-4, atol=1e-3)
        torch.testing.assert_close(t[..., 1], h, rtol=1e-4, atol=1e-3)
