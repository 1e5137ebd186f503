"""ResNet-152 v1.5 image trunk (the torchvision module tree src/mmbt.py:19-21 slices).

Child order and parameter names follow torchvision's resnet152 so that
``ImageEncoder.model = Sequential(children[:-2])`` yields the reference keys
``enc.img_encoder.model.{0..7}.*``.  No pretrained weights exist offline: weights
use torchvision's default init (He-normal fan_out convs, BN gamma 1 / beta 0).
On MI355X the trunk's convs run in bf16, channels-last (ImageEncoder): the 1x1 stride-1
products through mmu_gemm where measured faster (_mmu_1x1), the rest through MIOpen; every
BatchNorm2d [+ residual] [+ ReLU] through mmu_batchnorm_fwd/bwd.  In an identity-skip
Bottleneck the block input feeds both conv1 and bn3's residual: bn3's backward hands its
skip gradient to conv1's backward (_SkipGrad), whose dX GEMM adds it in the epilogue
(EPI_ADD_RES) instead of autograd summing the two in a separate pass.
"""
import os

import torch
import torch.nn as nn

from . import kernels as K


_TORCH_ONLY = [False]

# The residual stream past bf16 (round 5): each Bottleneck's output and its downsample's
# BatchNorm output carry an 8-bit residue (int8 of the map's size, csrc/batchnorm.hip), kept as
# the ``_mmu_res`` attribute of the bf16 map; the next bn3 adds it to its skip, so the stream
# is held to ~2^-15 of its value instead of bf16's 2^-8.  The convs read the bf16 map.
# MMU_STREAM_RESIDUE=0 turns it off process-wide (the parity A/B of profiles/r6_residue_parity_ab.txt).
STREAM_RESIDUE = os.environ.get("MMU_STREAM_RESIDUE", "1") != "0"
# A training conv on the gathered / mmu_gemm products writes its output's BatchNorm statistics in
# its own epilogue (MMU_EPI_STORE_STATS), so the BatchNorm after it skips its statistics pass
# (round 6; MMU_BN_STATS_FUSION=0: the BatchNorms compute them, for A/Bs)
BN_STATS_FUSION = os.environ.get("MMU_BN_STATS_FUSION", "1") != "0"
# ... and the backward: the data-gradient product of the conv that is a training BatchNorm's only
# consumer (a Bottleneck's conv2 / conv3, an identity block's conv1) writes that BatchNorm's
# backward reduction {sum g, sum g (x - mean)} in its epilogue (MMU_EPI_STORE_BNB / ADD_RES_BNB,
# mmu_conv3x3_implicit_bnb), so the BatchNorm backward skips its reduction pass
# (round 6; MMU_BN_BWD_FUSION=0 turns it off, for A/Bs)
BN_BWD_FUSION = os.environ.get("MMU_BN_BWD_FUSION", "1") != "0"
# An identity Bottleneck's skip gradient g = dY3 * mask3 is read by conv1's dX epilogue from bn3's dY
# and ReLU mask (res_mask) instead of being written out by bn3's backward (round 6;
# MMU_SKIP_MASKED=0: the materialised dSkip, for A/Bs)
SKIP_MASKED = os.environ.get("MMU_SKIP_MASKED", "1") != "0"


class _BnStats:
    """filled by a conv Function's forward with (table, nparts) of its output's statistics"""
    __slots__ = ("parts",)

    def __init__(self):
        self.parts = None


class _BnLink:
    """A training BatchNorm's hand-off to the conv that consumes its output (BN_BWD_FUSION): the
    BatchNorm's forward fills x / mask / mean (its input, ReLU mask, batch mean), the conv's
    backward fills ``parts`` (table, nparts) from its data-gradient epilogue, the BatchNorm's
    backward consumes them.  Carried as the ``_mmu_bnb`` attribute of the BatchNorm output."""
    __slots__ = ("x", "mask", "mean", "parts")

    def __init__(self):
        self.x = self.mask = self.mean = self.parts = None

    def operands(self):
        """(x, mask, mean) for the epilogue, or None once the BatchNorm's backward has run"""
        return None if self.x is None else (self.x, self.mask, self.mean)

    def release(self):
        self.x = self.mask = self.mean = self.parts = None


class torch_ops_only:
    """Context (ImageEncoder img_precision "torch_bf16", a TEST comparator): every trunk module
    takes PyTorch's own path instead of the HIP kernels / store copies."""

    def __init__(self, on=True):
        self.on, self.prev = bool(on), None

    def __enter__(self):
        self.prev, _TORCH_ONLY[0] = _TORCH_ONLY[0], self.on or _TORCH_ONLY[0]

    def __exit__(self, *exc):
        _TORCH_ONLY[0] = self.prev


class _BatchNormAct(torch.autograd.Function):
    """Training-mode BatchNorm2d [+ residual] [+ ReLU] on channels-last bf16 via
    mmu_batchnorm_fwd / mmu_batchnorm_bwd (batch statistics, running stats updated)."""

    @staticmethod
    def forward(ctx, x, weight, bias, skip, bn, relu, sink=None, skip_res=None, y_res=None, parts=None, link=None):
        ctx.bias_ref, ctx.sink, ctx.link = bias, sink, link
        Y = torch.empty_like(x)
        C = x.shape[1]
        smean = torch.empty(C, dtype=torch.float32, device=x.device)
        sinv = torch.empty_like(smean)
        # the backward reads the ReLU mask (1 bit per element) instead of Y (16 bits)
        mask = torch.empty(x.numel() // 8, dtype=torch.uint8, device=x.device) if relu else None
        K.batchnorm_fwd(x, Y, weight, bias, bn.running_mean, bn.running_var, True, _momentum_arg(bn), bn.eps,
                        relu=relu, skip=skip, num_batches_tracked=bn.num_batches_tracked, save_mean=smean,
                        save_invstd=sinv, relu_mask=mask, skip_res=skip_res, y_res=y_res, parts=parts)
        ctx.save_for_backward(x, mask, weight, smean, sinv)
        ctx.relu, ctx.has_skip = relu, skip is not None
        if link is not None:
            link.x, link.mask, link.mean = x, mask, smean
        return Y

    @staticmethod
    def backward(ctx, dY):
        x, mask, weight, smean, sinv = ctx.saved_tensors
        K.side_pump(dY.device, WGRAD_PUMP)  # (encoder INTERLEAVE: its weight-gradient work beside ours)
        dY = dY.contiguous(memory_format=torch.channels_last)
        dX = torch.empty_like(x)
        dS = torch.empty_like(x) if ctx.has_skip and ctx.needs_input_grad[3] else None
        # an identity block's bn3 (sink + ReLU mask): the skip gradient g = dY * mask is not written
        # out; conv1's dX epilogue reads dY and the mask instead (res_mask, SKIP_MASKED)
        gated = SKIP_MASKED and dS is not None and ctx.sink is not None and mask is not None and ctx.relu
        if gated:
            dS = None
        want_w, want_b = ctx.needs_input_grad[1], ctx.needs_input_grad[2]
        # straight into the flat gradient store when it exists (no AccumulateGrad pass)
        dw = (weight.grad if weight.grad is not None else torch.zeros_like(weight)) if want_w else None
        db = None
        if want_b:
            bias = ctx.bias_ref
            db = bias.grad if bias.grad is not None else torch.zeros_like(bias)
        parts = None
        if ctx.link is not None:  # the reduction the consuming conv's dX epilogue wrote, if it did
            parts = ctx.link.parts
            ctx.link.release()
        K.batchnorm_bwd(dY, None, x, weight, smean, sinv, ctx.relu, dX, dS, dw, db, relu_mask=mask, parts=parts)
        rw = dw if (want_w and weight.grad is None) else None
        rb = db if (want_b and ctx.bias_ref.grad is None) else None
        if ctx.sink is not None and dS is not None:  # conv1's dX GEMM adds it (EPI_ADD_RES)
            ctx.sink.g, dS = dS, None
        elif gated:
            ctx.sink.g = (dY, mask)
        return dX, rw, rb, dS, None, None, None, None, None, None, None


def _momentum(bn):
    """the running-statistics factor of this training pass: bn.momentum, or for momentum=None
    (torch's cumulative moving average) 1 / num_batches_tracked after this pass's increment
    (host value: the torch-op sync path only)"""
    if bn.momentum is not None:
        return float(bn.momentum)
    return 1.0 / float(int(bn.num_batches_tracked) + 1)


def _momentum_arg(bn):
    """the kernels' momentum argument: bn.momentum, or for momentum=None -1 after counting this
    pass in num_batches_tracked ON THE DEVICE (the kernel then uses 1 / num_batches_tracked): no
    device-to-host read, so the pass stays asynchronous and graph-capturable"""
    if bn.momentum is not None:
        return float(bn.momentum)
    bn.num_batches_tracked.add_(1)
    return -1.0


class _SyncBatchNormAct(torch.autograd.Function):
    """Training-mode BatchNorm2d [+ residual] [+ ReLU] with statistics over the batch of every
    rank of ``group`` (the reference's whole-batch normalisation, src/mmbt.py:19-21, kept under
    data parallelism; torch.nn.SyncBatchNorm's exchange): each pass sums its per-channel
    reductions locally, all-reduces {s1[C], s2[C], rows} (2C+1 f64), then normalises / forms
    dX from the global sums.  The weight / bias gradients stay this rank's (the DP gradient
    all-reduce sums them).  bf16 channels-last GPU maps run mmu_batchnorm_stats /
    _fwd_sums / _bwd_reduce / _bwd_sums; anything else (fp32 parity runs, CPU) the same
    arithmetic in torch ops."""

    @staticmethod
    def forward(ctx, x, weight, bias, skip, bn, relu, sink, group, hip, skip_res=None, y_res=None):
        import torch.distributed as dist
        ctx.bias_ref, ctx.sink, ctx.group, ctx.hip = bias, sink, group, hip
        ctx.relu, ctx.has_skip = relu, skip is not None
        C = x.shape[1]
        if hip:
            sums = K.bn_sums_buffer(C, x.device)
            K.batchnorm_stats(x, sums)
            dist.all_reduce(sums, group=group)
            Y = torch.empty_like(x)
            smean = torch.empty(C, dtype=torch.float32, device=x.device)
            sinv = torch.empty_like(smean)
            mask = torch.empty(x.numel() // 8, dtype=torch.uint8, device=x.device) if relu else None
            K.batchnorm_fwd_sums(x, Y, sums, weight, bias, bn.running_mean, bn.running_var, _momentum_arg(bn), bn.eps,
                                 relu=relu, skip=skip, num_batches_tracked=bn.num_batches_tracked, save_mean=smean,
                                 save_invstd=sinv, relu_mask=mask, skip_res=skip_res, y_res=y_res)
            ctx.save_for_backward(x, mask, weight, smean, sinv)
            return Y
        xd = x.double()
        red = [0, 2, 3]
        sums = torch.cat([xd.sum(red), (xd * xd).sum(red), xd.new_tensor([x.numel() // C])])
        dist.all_reduce(sums, group=group)
        n = sums[2 * C]
        mean = sums[:C] / n
        var = (sums[C:2 * C] / n - mean * mean).clamp_min(0)
        invstd = (var + bn.eps).rsqrt()
        if bn.running_mean is not None:
            with torch.no_grad():
                m = _momentum(bn)
                bn.running_mean.mul_(1 - m).add_(m * mean.to(bn.running_mean.dtype))
                bn.running_var.mul_(1 - m).add_(m * (var * n / (n - 1)).to(bn.running_var.dtype))
                bn.num_batches_tracked.add_(1)
        shape = (1, C, 1, 1)
        scale = invstd * (weight.double() if weight is not None else 1.0)
        shift = (bias.double() if bias is not None else 0.0) - mean * scale
        y = (xd * scale.view(shape) + shift.view(shape)).to(x.dtype)
        if skip is not None:
            y = y + skip
        if relu:
            y = torch.relu(y)
        ctx.save_for_backward(x, y if relu else None, weight, mean, invstd)
        return y

    @staticmethod
    def backward(ctx, dY):
        import torch.distributed as dist
        x, saved, weight, mean, invstd = ctx.saved_tensors
        K.side_pump(x.device, WGRAD_PUMP)
        C = x.shape[1]
        want_w, want_b = ctx.needs_input_grad[1], ctx.needs_input_grad[2]
        bias = ctx.bias_ref
        if ctx.hip:
            dY = dY.contiguous(memory_format=torch.channels_last)
            dw = (weight.grad if weight.grad is not None else torch.zeros_like(weight)) if want_w else None
            db = (bias.grad if bias.grad is not None else torch.zeros_like(bias)) if want_b else None
            sums = K.bn_sums_buffer(C, x.device)
            K.batchnorm_bwd_reduce(dY, None, x, mean, invstd, ctx.relu, sums, dw, db, relu_mask=saved)
            dist.all_reduce(sums, group=ctx.group)
            dX = torch.empty_like(x)
            dS = torch.empty_like(x) if ctx.has_skip and ctx.needs_input_grad[3] else None
            K.batchnorm_bwd_sums(dY, None, x, sums, weight, mean, invstd, ctx.relu, dX, dS, relu_mask=saved)
            rw = dw if (want_w and weight.grad is None) else None
            rb = db if (want_b and bias.grad is None) else None
        else:
            g = dY * (saved > 0) if ctx.relu else dY
            gd = g.double()
            red = [0, 2, 3]
            shape = (1, C, 1, 1)
            xmu = x.double() - mean.view(shape)
            sums = torch.cat([gd.sum(red), (gd * xmu).sum(red), gd.new_tensor([x.numel() // C])])
            rw = (sums[C:2 * C] * invstd).to(weight.dtype) if want_w else None
            rb = sums[:C].to(bias.dtype) if want_b else None
            dist.all_reduce(sums, group=ctx.group)
            n = sums[2 * C]
            a = invstd * (weight.double() if weight is not None else 1.0)
            dX = (a.view(shape) * (gd - (sums[:C] / n).view(shape)
                                    - xmu * (invstd * invstd * sums[C:2 * C] / n).view(shape))).to(x.dtype)
            dS = g if ctx.has_skip and ctx.needs_input_grad[3] else None
        if ctx.sink is not None and dS is not None:  # conv1's dX GEMM adds it (EPI_ADD_RES)
            ctx.sink.g, dS = dS, None
        return dX, rw, rb, dS, None, None, None, None, None, None, None


class BatchNorm2d(nn.BatchNorm2d):
    """BatchNorm2d with the activation fused in (state_dict / semantics of torch's).
    ``forward(x, skip=None, relu=None)`` computes act(BN(x) [+ skip]); ``relu`` defaults
    to the module's ``fused_relu`` (set for the stem BN, whose ReLU module is then a
    FusedReLU no-op).  bf16 channels-last inputs on the GPU run the HIP kernels
    (training: batch statistics; eval: running statistics, one elementwise pass);
    anything else (fp32 parity runs) uses PyTorch's batch_norm."""

    fused_relu = False
    MIOPEN_MIN_BATCH = 8
    sync_group = None  # a process group: training statistics over all its ranks' batches (src/dp.py)

    def forward(self, x, skip=None, relu=None, skip_sink=None, out_res=False):
        """``out_res``: this BN produces the residual stream (a Bottleneck's bn3, a downsample's
        BN): on the HIP path its output carries the 8-bit stream residue (``_mmu_res``,
        STREAM_RESIDUE), and a skip's own residue is read."""
        relu = self.fused_relu if relu is None else relu
        # (the kernels take f32 per-channel parameters / statistics: a module cast to bf16 --
        # module.to(torch.bfloat16) -- takes the torch path)
        hip = (not _TORCH_ONLY[0] and x.is_cuda and x.dtype == torch.bfloat16 and (skip is None or skip.dtype == torch.bfloat16)
               and x.shape[1] % 8 == 0 and self.weight is not None and self.weight.dtype == torch.float32
               and (self.running_mean is None or self.running_mean.dtype == torch.float32))
        skip_res = getattr(skip, "_mmu_res", None) if skip is not None else None
        res = hip and out_res and STREAM_RESIDUE and (skip is None or skip_res is not None)
        if hip:
            x = x.contiguous(memory_format=torch.channels_last)
            if skip is not None:
                skip = skip.contiguous(memory_format=torch.channels_last)
        y_res = torch.empty(x.numel(), dtype=torch.int8, device=x.device) if res else None
        if not res:
            skip_res = None
        if self.sync_group is not None and self.training and self.track_running_stats:
            y = _SyncBatchNormAct.apply(x, self.weight, self.bias, skip, self, relu, skip_sink, self.sync_group, hip,
                                        skip_res, y_res)
            return _with_res(y, y_res)
        if hip:
            if self.training and self.track_running_stats:
                # the statistics the producing conv's epilogue wrote (BN_STATS_FUSION), if any
                parts = x.__dict__.pop("_mmu_bnparts", None)
                link = _BnLink() if BN_BWD_FUSION and torch.is_grad_enabled() else None
                y = _BatchNormAct.apply(x, self.weight, self.bias, skip, self, relu, skip_sink, skip_res, y_res,
                                        parts, link)
                if link is not None:
                    y._mmu_bnb = link
                return _with_res(y, y_res)
            if not self.training and not (torch.is_grad_enabled() and (
                    x.requires_grad or self.weight.requires_grad or (skip is not None and skip.requires_grad))):
                # the one-pass running-statistics kernel has no backward: a graph through an
                # eval-mode BN (frozen statistics during training) takes the torch path below
                Y = torch.empty_like(x)
                K.batchnorm_fwd(x, Y, self.weight, self.bias, self.running_mean, self.running_var, False,
                                0.0, self.eps, relu=relu, skip=skip, skip_res=skip_res, y_res=y_res)
                return _with_res(Y, y_res)
        if self.training or not self.track_running_stats:
            # MIOpen's NHWC batch-norm crashes in host code for tiny batches on this stack
            with torch.backends.cudnn.flags(enabled=x.shape[0] >= self.MIOPEN_MIN_BATCH):
                y = super().forward(x)
        else:  # inference as one per-channel affine pass
            s = self.weight * (self.running_var + self.eps).rsqrt()
            t = self.bias - self.running_mean * s
            y = x * s.view(1, -1, 1, 1).to(x.dtype) + t.view(1, -1, 1, 1).to(x.dtype)
        if skip is not None:
            y = y + skip
        return torch.relu(y) if relu else y


def _with_res(y, res):
    if res is not None:
        y._mmu_res = res
    return y


def _is_stem(w16, stride, padding):
    """the ResNet stem conv (7x7, stride 2, pad 3, 3 -> 64): forward and filter gradient on
    mmu_stem_conv_* (its data gradient is never needed: the image is a leaf input)"""
    return (tuple(w16.shape) == (64, 3, 7, 7) and tuple(stride) == (2, 2) and tuple(padding) == (3, 3))


# downsample blocks: conv1's dX epilogue adds the downsample conv's dX (no autograd sum) -- MMU_DS_SINK=0: off
DS_SINK = os.environ.get("MMU_DS_SINK", "1") != "0"
WGRAD_PUMP = int(os.environ.get("MMU_WGRAD_PUMP", "1"))  # deferred BERT items issued per BatchNorm backward
SIDE_WGRAD_MIN_BATCH = int(os.environ.get("MMU_SIDE_WGRAD_MIN_BATCH", "128"))


def _side_wgrad(t):
    """filter gradients of this [N, C, H, W] map's conv go to the side stream (_wgrad_run)"""
    return t.is_cuda and t.shape[0] >= SIDE_WGRAD_MIN_BATCH


def _wgrad_run(fn, *tensors):
    """Run a filter-gradient product (off the backward's data-gradient chain) on the device's
    side stream, ordered after everything the main stream has enqueued so far; the tensors it
    reads are record_stream'ed for the caching allocator and the main stream joins the side
    stream when the backward ends (kernels.join_at_backward_end).  The trunk's backward is a
    chain of short, latency-bound kernels (BatchNorm passes, small-map convs), so the side
    stream's products fill the CUs the chain leaves idle.  Only from SIDE_WGRAD_MIN_BATCH
    images up (tensors[0] is the [N, C, H, W] map): the stream hop costs ~35 us of host time
    per conv, and at batch 32 the step is bound by kernel issue -- measured 167.7 -> 165.6 ms
    at batch 256, but 41.7 -> 46.7 ms at batch 32 without the gate (profiles/r3_side_wgrad_ab.txt)."""
    dev = tensors[0].device
    if not _side_wgrad(tensors[0]):
        fn()
        return
    main = torch.cuda.current_stream(dev)
    side = K.side_stream(dev)
    side.wait_stream(main)
    for t in tensors:
        t.record_stream(side)
    with torch.cuda.stream(side):
        fn()
    K.join_at_backward_end(main, side)


class _ConvBF16(torch.autograd.Function):
    """Conv2d on the bf16 filter copy kept by the parameter store (updated by the fused
    optimizer), so no per-step autocast cast of the f32 filter; the backward adds MIOpen's
    bf16 filter gradient straight into the f32 gradient view (one kernel instead of a cast
    plus an AccumulateGrad add)."""

    @staticmethod
    def forward(ctx, x, w, w16, stride, padding, flipped=None, stats=None, link=None, sink_out=None):
        ctx.save_for_backward(x, w16)
        ctx.w, ctx.conf, ctx.flipped, ctx.link, ctx.sink_out = w, (stride, padding), flipped, link, sink_out
        cout = w16.shape[0]
        if _is_stem(w16, stride, padding):  # the 7x7 / 2 stem: mmu_stem_conv_fwd
            n, _, h, wd = x.shape
            y = torch.empty((n, cout, (h - 1) // 2 + 1, (wd - 1) // 2 + 1), dtype=x.dtype, device=x.device,
                            memory_format=torch.channels_last)
            K.stem_conv_fwd(x, w16, y)
            return y
        geo = _conv_geo(w16, stride, padding)
        ctx.route = route = _mmu_conv(geo, x.shape, cout)
        if route[0]:
            ks, st = geo
            n, _, h, wd = x.shape
            ho, wo = (h + 2 * (ks // 2) - ks) // st + 1, (wd + 2 * (ks // 2) - ks) // st + 1
            y = torch.empty((n, cout, ho, wo), dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
            if stats is not None:  # + the BatchNorm statistics of y, from the epilogue
                stats.parts = K.bn_stats_table(n * ho * wo, cout, x.device)
                K.conv_implicit(x, w16, y, ks, st, stats=stats.parts[0])
            else:
                K.conv_implicit(x, w16, y, ks, st)
            return y
        return torch.ops.aten.convolution(x, w16, None, stride, padding, (1, 1), False, (0, 0), 1)

    @staticmethod
    def backward(ctx, dy):
        return _hand_dx(ctx, _ConvBF16._bwd(ctx, dy)) + (None,)

    @staticmethod
    def _bwd(ctx, dy):
        x, w16 = ctx.saved_tensors
        stride, padding = ctx.conf
        need_x, need_w = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        dy = dy.contiguous(memory_format=torch.channels_last)
        cl = torch.channels_last
        # filter gradients: one implicit-im2col MFMA GEMM straight into the f32 gradient
        # (mmu_conv_wgrad / mmu_stem_conv_wgrad) instead of MIOpen's wrw + a zero fill + an add
        stem = _is_stem(w16, stride, padding)
        geo = None if stem else _conv_geo(w16, stride, padding)
        route = (True, False, True) if stem else ctx.route
        mmu_w = need_w and route[2]
        if stem:
            wgrad = K.stem_conv_wgrad
        else:
            def wgrad(dy_, x_, dw_, accumulate):
                K.conv_wgrad(dy_, x_, dw_, geo[0], geo[1], accumulate)
        # 3x3 / stride-1 data gradient: the same implicit GEMM on dY with the flipped filter,
        # [Cin][3][3][Cout]
        mmu_x = need_x and route[1]
        dx = rw = None
        g = ctx.w.grad
        store_g = need_w and g is not None and g.dtype == torch.float32 and g.is_contiguous(memory_format=cl)
        if need_x and not mmu_x and store_g and not mmu_w and not _side_wgrad(dy):
            # both products on MIOpen, both on this stream: one call (its host cost is ~30 us)
            dx, gw, _ = torch.ops.aten.convolution_backward(dy, x, w16, None, stride, padding, (1, 1), False, (0, 0),
                                                            1, (True, True, False))
            g.add_(gw)
            return dx, None, None, None, None, None, None, None
        if need_x and not mmu_x:
            dx = torch.ops.aten.convolution_backward(dy, x, w16, None, stride, padding, (1, 1), False, (0, 0), 1,
                                                     (True, False, False))[0]
        if mmu_x:
            dx = torch.empty_like(x, memory_format=cl)
            # the store's flipped copy (refreshed with the bf16 filters), else one made here
            wf = ctx.flipped() if ctx.flipped is not None else w16.flip(2, 3).permute(1, 2, 3, 0).contiguous()
            bnb = ctx.link.operands() if ctx.link is not None else None
            if bnb is not None:  # + the backward reduction of the BatchNorm that produced x
                table = K.bn_stats_table(dx.numel() // dx.shape[1], dx.shape[1], dx.device)
                K.conv3x3_implicit(dy, wf, dx, bnb=bnb, table=table[0])
                ctx.link.parts = table
            else:
                K.conv3x3_implicit(dy, wf, dx)
        if store_g:
            # straight into the gradient store, on the side stream
            def dw_side():
                if mmu_w:
                    wgrad(dy, x, g, accumulate=True)
                else:
                    g.add_(torch.ops.aten.convolution_backward(dy, x, w16, None, stride, padding, (1, 1), False,
                                                               (0, 0), 1, (False, True, False))[1])
            _wgrad_run(dw_side, dy, x)
        elif need_w:
            if mmu_w:
                rw = torch.empty(w16.shape, dtype=torch.float32, device=x.device, memory_format=cl)
                wgrad(dy, x, rw, accumulate=False)
            else:
                rw = torch.ops.aten.convolution_backward(dy, x, w16, None, stride, padding, (1, 1), False, (0, 0), 1,
                                                         (False, True, False))[1].float()
            if g is not None:
                g.add_(rw)
                rw = None
        return dx, rw, None, None, None, None, None, None


class _SkipGrad:
    """The gradient of a Bottleneck's residual input, handed to conv1's backward, whose dX GEMM
    adds it in its epilogue (EPI_ADD_RES[_BNB]) instead of autograd summing two gradients of x:
    * identity blocks: bn3's backward hands dY3 (and its ReLU mask); autograd always runs it
      before conv1's (conv1 feeds bn3);
    * downsample blocks (ds = True): the downsample conv's backward hands its dX.  The block
      builds that branch after conv3, so autograd (later-created nodes first) runs it before
      conv1's backward; should it not, conv1 marks the sink done and the downsample conv returns
      its dX to autograd as usual (and conv1 then writes no BatchNorm reduction for x: its dX
      is not x's whole gradient)."""
    __slots__ = ("g", "ds", "done")

    def __init__(self, ds=False):
        self.g, self.ds, self.done = None, ds, False


def _hand_dx(ctx, out):
    """a downsample conv's backward: its dX goes to the block's sink (conv1 adds it) when conv1
    has not run yet"""
    so = ctx.sink_out
    if so is None or out[0] is None or so.done:
        return out
    so.g = out[0].contiguous(memory_format=torch.channels_last)
    return (None,) + tuple(out[1:])


def _mask_bits(mask, like):
    """a ReLU mask (u8, bit e of byte i = element 8i+e of the channels-last map) as a 0/1 tensor
    shaped / laid out like ``like`` ([N, C, H, W] channels-last)"""
    bits = (mask.view(-1, 1) >> torch.arange(8, device=mask.device, dtype=torch.uint8)) & 1
    return bits.view(like.shape[0], like.shape[2], like.shape[3], like.shape[1]).permute(0, 3, 1, 2).to(like.dtype)


def _rows(t):
    """[N, C, H, W] channels-last -> its [N*H*W, C] row-major view."""
    return t.permute(0, 2, 3, 1).reshape(-1, t.shape[1])


def _conv_geo(w16, stride, padding):
    """(ksize, stride) of a square 3x3 / pad 1 or 1x1 / pad 0 conv with equal strides (the
    shapes mmu_conv_implicit / mmu_conv_wgrad take), else None"""
    k = tuple(w16.shape[2:])
    if k not in ((3, 3), (1, 1)) or stride[0] != stride[1] or tuple(padding) != (k[0] // 2,) * 2:
        return None
    return k[0], stride[0]


# Routing decisions (_mmu_conv / _mmu_1x1) are taken as if every map held ROUTE_M_SCALE times its
# rows: a data-parallel rank running B / N samples sets N to route its convs exactly as the single
# device does at the global batch B (tests/test_dp_gpu.py: the sync-BN root cause)
ROUTE_M_SCALE = 1
# Route A/B switch (round 6): with the BatchNorm passes fused into the conv epilogues, an mmu
# product also saves a BatchNorm pass.  MMU_ROUTE_FUSED=1 moves every shape-eligible 1x1 forward
# and the 128-channel 3x3 forward onto mmu; 2 also the 64-channel 3x3 forward / data gradient.
ROUTE_FUSED = int(os.environ.get("MMU_ROUTE_FUSED", "0"))


def _mmu_conv(geo, xshape, cout):
    """(forward, data gradient, filter gradient) of a conv on the gathered-operand MFMA
    products (mmu_conv_implicit / mmu_conv_wgrad) instead of MIOpen, from same-box timings
    of both engines (profiles/r3_conv_census_b256.txt, r3_conv_strided.txt):
      3x3 stride 1: forward for Cout >= 256 (% 128), dX for Cin >= 128 (% 128: layer2's
        128-channel dX is 117 vs 142 us at batch 256, 36 vs 41 us at batch 32), dW for
        Cin % 256 == 0 (layer3 / layer4 conv2);
      strided 3x3 (layer3 / layer4 conv2 at >= 12544 output pixels: forward and dW) and the
        1x1 / stride-2 downsample (forward and dW at 12544..50176 output pixels: layer3 /
        layer4 at batch 256, layer2's forward at batch 32); their dX stays MIOpen's."""
    if geo is None:
        return False, False, False
    ks, st = geo
    n, cin, h, w = xshape
    pad = ks // 2
    M = ROUTE_M_SCALE * n * ((h + 2 * pad - ks) // st + 1) * ((w + 2 * pad - ks) // st + 1)
    if ks == 3 and st == 1:
        fwd = cin % 64 == 0 and cout % 128 == 0 and (cout >= 256 or ROUTE_FUSED >= 1) and M >= 256
        dx = cout % 64 == 0 and cin % 128 == 0 and M >= 256
        if ROUTE_FUSED >= 2:
            fwd = cin % 64 == 0 and cout % 64 == 0 and M >= 256
            dx = cout % 64 == 0 and cin % 64 == 0 and M >= 256
        dw = cin % 256 == 0 and cout % 128 == 0 and M >= 1024
        return fwd, dx, dw
    if st == 1:  # 1x1 stride 1: _Conv1x1
        return False, False, False
    if ks == 3:
        fwd = cin % 64 == 0 and cout % 128 == 0 and cout >= 256 and M >= 12544
    else:
        fwd = cin % 64 == 0 and cout % 128 == 0 and 12544 <= M <= 50176
    # (the 2-tile 256 -> 512 downsample filter gradient only at batch 256's 200 k pixels)
    dw = cin % 256 == 0 and cout % 128 == 0 and M >= 12544 and (ks == 3 or cin * cout >= 8 * 65536 or M >= 100352)
    return fwd, False, dw


def _mmu_1x1(cin, cout, M, H):
    """Which products of a 1x1 stride-1 conv (rows M = N*H*W) run on mmu_gemm instead of
    MIOpen, from profiles/r1_conv1x1_b256.txt / _b32.txt (same-box timings, both engines):
    dX always for the reducing convs (cin > cout) and for M >= 12544; the forward for
    25088 <= M <= 50176 (and not the widening 14x14 product at batch 256); the weight
    gradient for M <= 50176 at H <= 14 (layer3 / layer4; below M = 12544 -- the batch-32 to
    batch-128 ranks of config 4 -- since the short-K split-K of profiles/r3_wgrad_shortk_ab.txt
    brought it level with MIOpen's wrw, which also pays a bf16 -> f32 add into the store).
    mmu_gemm needs N % 128 == 0 for its output columns (and M-major A rows % 128 for dW)."""
    M = M * ROUTE_M_SCALE
    fwd = cout % 128 == 0 and cin % 64 == 0 and (ROUTE_FUSED >= 1 or (25088 <= M <= 50176 and (cin > cout or M < 50176)))
    dx = cin % 128 == 0 and cout % 64 == 0 and (cin > cout or M >= 12544)
    dw = cin % 128 == 0 and cout % 128 == 0 and M <= 50176 and H <= 14
    return fwd, dx, dw


class _Conv1x1(torch.autograd.Function):
    """1x1 stride-1 convolution of a channels-last bf16 map, as products over its [N*H*W, C]
    rows:  Y = X W^T,  dX = dY W (+ the skip gradient: EPI_ADD_RES),  dW += dY^T X (f32,
    split-K, straight into the gradient store) -- each on mmu_gemm or MIOpen per _mmu_1x1.
    The GEMMs are excluded from bench.py's BERT-layer GEMM timing (timing_paused)."""

    @staticmethod
    def forward(ctx, x, w, w16, sink, stats=None, link=None, sink_out=None):
        Nb, C, H, W = x.shape
        Co = w16.shape[0]
        M = Nb * H * W
        use_f, use_d, use_w = _mmu_1x1(C, Co, M, H)
        if use_f:
            y = torch.empty((Nb, Co, H, W), dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
            epi = None
            if stats is not None:  # + the BatchNorm statistics of y, from the epilogue
                stats.parts = K.bn_stats_table(M, Co, x.device)
                epi = K.epilogue(K.EPI_STORE_STATS, colsum=stats.parts[0])
            with K.timing_paused():
                K.gemm(_rows(x), C, 1, w16.view(Co, C), C, 1, _rows(y), Co, M, Co, C, epi=epi)
        else:
            y = torch.ops.aten.convolution(x, w16, None, (1, 1), (0, 0), (1, 1), False, (0, 0), 1)
        ctx.save_for_backward(x, w16)
        ctx.w, ctx.sink, ctx.use, ctx.link, ctx.sink_out = w, sink, (use_d, use_w), link, sink_out
        return y

    @staticmethod
    def backward(ctx, dy):
        return _hand_dx(ctx, _Conv1x1._bwd(ctx, dy)) + (None,)

    @staticmethod
    def _bwd(ctx, dy):
        x, w16 = ctx.saved_tensors
        use_d, use_w = ctx.use
        need_x, need_w = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        Nb, C, H, W = x.shape
        Co = w16.shape[0]
        M = Nb * H * W
        dy = dy.contiguous(memory_format=torch.channels_last)
        skip = rmask = None
        late_ds = False
        if ctx.sink is not None:
            skip, ctx.sink.g = ctx.sink.g, None
            ctx.sink.done = True
            late_ds = ctx.sink.ds and skip is None  # (the downsample's dX comes through autograd)
            if isinstance(skip, tuple):  # (bn3's dY, its ReLU mask): the gated skip gradient
                skip, rmask = skip
        dx = rw = None
        with K.timing_paused():
            if need_x and use_d:
                dx = torch.empty_like(x, memory_format=torch.channels_last)
                bnb = ctx.link.operands() if ctx.link is not None and not late_ds else None
                if bnb is not None:  # + the backward reduction of the BatchNorm that produced x
                    table = K.bn_stats_table(M, C, x.device)
                    epi = K.epilogue(K.EPI_ADD_RES_BNB if skip is not None else K.EPI_STORE_BNB,
                                     residual=_rows(skip) if skip is not None else None, colsum=table[0], bn=bnb,
                                     res_mask=rmask)
                    ctx.link.parts = table
                else:
                    epi = (K.epilogue(K.EPI_ADD_RES, residual=_rows(skip), res_mask=rmask)
                           if skip is not None else None)
                K.gemm(_rows(dy), Co, 1, w16.view(Co, C), C, 0, _rows(dx), C, M, C, Co, epi=epi)
                skip = None
            elif need_x:
                both = need_w and not use_w and ctx.w.grad is not None and not _side_wgrad(dy)
                gx, gw, _ = torch.ops.aten.convolution_backward(dy, x, w16, None, (1, 1), (0, 0), (1, 1), False,
                                                                (0, 0), 1, (True, both, False))
                if rmask is not None:
                    skip = skip * _mask_bits(rmask, skip)
                dx = gx if skip is None else gx + skip
                if both:  # (one MIOpen call for both products when neither goes elsewhere)
                    ctx.w.grad.add_(gw)
                    return dx, None, None, None, None, None
            if need_w:
                g = ctx.w.grad
                if g is None:
                    g = rw = torch.zeros_like(ctx.w, memory_format=torch.contiguous_format)

                def dw():  # straight into the gradient store, on the side stream
                    with K.timing_paused():
                        if use_w:
                            K.gemm(_rows(dy), Co, 0, _rows(x), C, 0, g.view(Co, C), C, Co, C, M,
                                   epi=K.epilogue(K.EPI_STORE, accumulate=True))
                        else:
                            g.add_(torch.ops.aten.convolution_backward(dy, x, w16, None, (1, 1), (0, 0), (1, 1), False,
                                                                       (0, 0), 1, (False, True, False))[1])
                if rw is None:
                    _wgrad_run(dw, dy, x)
                else:
                    dw()
        return dx, rw, None, None, None, None


class StoreConv2d(nn.Conv2d):
    """nn.Conv2d (same parameters / state_dict) that, once the model's parameter store
    holds a bf16 copy of its filter, convolves bf16 channels-last inputs with that copy.
    The copy's freshness is the store's business: MultimodalBertEncoder._prepare() runs
    check_views / maybe_sync_compute before every forward."""

    _src = None

    def attach_compute(self, store, name):
        import weakref
        self._src = (weakref.ref(store), name)

    def _compute_weight(self, x):
        src = self._src
        if (src is not None and not _TORCH_ONLY[0] and x.is_cuda and x.dtype == torch.bfloat16 and self.bias is None and self.groups == 1
                and self.dilation == (1, 1)):
            store = src[0]()
            if store is not None:
                return store.compute_of(src[1])
        return None

    def _flipped_getter(self):
        """() -> the store's flipped [Cin, 3, 3, Cout] copy of this 3x3 filter (created on the
        first data-gradient call), or None"""
        src = self._src
        if src is None or self.kernel_size != (3, 3):
            return None
        store, name = src[0](), src[1]
        if store is None or not hasattr(store, "flipped_filter"):
            return None
        return lambda: store.flipped_filter(name)

    def _is_1x1(self):
        return self.kernel_size == (1, 1) and self.stride == (1, 1) and self.padding == (0, 0)

    def takes_skip_grad(self, x):
        """True when this conv's backward will add a _SkipGrad into its dX GEMM."""
        if not (self._is_1x1() and torch.is_grad_enabled() and x.requires_grad):
            return False
        if self._compute_weight(x) is None:
            return False
        N_, C, H, W = x.shape
        return _mmu_1x1(C, self.out_channels, N_ * H * W, H)[1]

    def forward(self, x, sink=None, bnb=False, sink_out=None):
        """bnb: x is a training BatchNorm's output and this conv its only consumer (the gradient
        of x is this conv's dX alone): the dX epilogue may write that BatchNorm's backward
        reduction (BN_BWD_FUSION, _BnLink)"""
        w16 = self._compute_weight(x)
        if w16 is not None:
            link = x.__dict__.get("_mmu_bnb") if bnb else None
            x = x.contiguous(memory_format=torch.channels_last)
            # a training forward (the BatchNorm after this conv uses batch statistics): the conv's
            # epilogue writes them when it runs on the mmu products (BN_STATS_FUSION)
            st = _BnStats() if BN_STATS_FUSION and self.training and torch.is_grad_enabled() else None
            if self._is_1x1():
                y = _Conv1x1.apply(x, self.weight, w16, sink, st, link, sink_out)
            else:
                y = _ConvBF16.apply(x, self.weight, w16, self.stride, self.padding, self._flipped_getter(), st, link,
                                    sink_out)
            if st is not None and st.parts is not None:
                y._mmu_bnparts = st.parts
            return y
        if sink is not None or sink_out is not None:
            raise RuntimeError("StoreConv2d: a skip-gradient sink needs the bf16 path")
        return super().forward(x)


class _MaxPool3s2(torch.autograd.Function):
    """MaxPool2d(3, 2, 1) on a channels-last bf16 map via mmu_maxpool_fwd / _bwd (1-byte
    argmax per output element; the backward is a gather over the covering windows)."""

    @staticmethod
    def forward(ctx, x):
        B, C, H, W = x.shape
        OH, OW = (H - 1) // 2 + 1, (W - 1) // 2 + 1
        y = torch.empty((B, C, OH, OW), dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
        am = torch.empty((B, OH, OW, C), dtype=torch.uint8, device=x.device)
        K.maxpool_fwd(x, y, am)
        ctx.save_for_backward(am)
        ctx.shape = x.shape
        return y

    @staticmethod
    def backward(ctx, dy):
        (am,) = ctx.saved_tensors
        dy = dy.contiguous(memory_format=torch.channels_last)
        dx = torch.empty(ctx.shape, dtype=dy.dtype, device=dy.device, memory_format=torch.channels_last)
        K.maxpool_bwd(dy, am, dx)
        return dx


class MaxPool2d(nn.MaxPool2d):
    """nn.MaxPool2d (torchvision's stem pool, child 3) whose 3x3 / stride-2 / pad-1 case on
    channels-last bf16 maps runs the HIP kernels; anything else is PyTorch's."""

    def forward(self, x):
        if (not _TORCH_ONLY[0] and x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and x.shape[1] % 8 == 0
                and self.kernel_size in (3, (3, 3)) and self.stride in (2, (2, 2)) and self.padding in (1, (1, 1))
                and self.dilation in (1, (1, 1)) and not self.ceil_mode and not self.return_indices):
            return _MaxPool3s2.apply(x.contiguous(memory_format=torch.channels_last))
        return super().forward(x)


class FusedReLU(nn.ReLU):
    """The stem's ReLU slot (torchvision child index 2): the preceding BatchNorm2d
    already applied it, so this is the identity."""

    def forward(self, x):
        return x


class Bottleneck(nn.Module):
    def __init__(self, cin, width, stride):
        super().__init__()
        cout = width * 4
        self.conv1 = StoreConv2d(cin, width, 1, bias=False)
        self.bn1 = BatchNorm2d(width)
        self.conv2 = StoreConv2d(width, width, 3, stride=stride, padding=1, bias=False)
        self.bn2 = BatchNorm2d(width)
        self.conv3 = StoreConv2d(width, cout, 1, bias=False)
        self.bn3 = BatchNorm2d(cout)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = None
        if stride != 1 or cin != cout:
            self.downsample = nn.Sequential(StoreConv2d(cin, cout, 1, stride=stride, bias=False), BatchNorm2d(cout))

    def forward(self, x):
        sink = None
        ds_pair = (isinstance(self.downsample, nn.Sequential) and len(self.downsample) == 2
                   and isinstance(self.downsample[0], StoreConv2d) and isinstance(self.downsample[1], BatchNorm2d))
        if (self.training and self.bn3.track_running_stats and x.is_cuda and x.dtype == torch.bfloat16
                and (self.downsample is None or (DS_SINK and ds_pair and self.downsample[0]._compute_weight(x) is not None))
                and self.conv1.takes_skip_grad(x)):
            x = x.contiguous(memory_format=torch.channels_last)
            sink = _SkipGrad(ds=self.downsample is not None)
        if sink is not None and sink.ds:
            # the downsample branch after conv3: autograd (later-created nodes first) then runs its
            # backward before conv1's, and conv1's dX epilogue adds the downsample's dX (_SkipGrad)
            y = self.bn1(self.conv1(x, sink=sink, bnb=True), relu=True)
            y = self.bn2(self.conv2(y, bnb=True), relu=True)
            y = self.conv3(y, bnb=True)
            skip = self.downsample[1](self.downsample[0](x, sink_out=sink), out_res=True)
            out = self.bn3(y, skip=skip, relu=True, out_res=True)
            if getattr(skip, "_mmu_res", None) is not None:
                del skip._mmu_res
            return out
        if self.downsample is None:
            skip = x
        elif isinstance(self.downsample, nn.Sequential) and len(self.downsample) == 2 and isinstance(
                self.downsample[1], BatchNorm2d):
            skip = self.downsample[1](self.downsample[0](x), out_res=True)
        else:
            skip = self.downsample(x)
        # (x's gradient is conv1's dX alone when bn3 hands its skip gradient to the sink)
        y = self.bn1(self.conv1(x, sink=sink, bnb=sink is not None), relu=True)
        y = self.bn2(self.conv2(y, bnb=True), relu=True)
        out = self.bn3(self.conv3(y, bnb=True), skip=skip, relu=True, skip_sink=sink, out_res=True)
        if getattr(skip, "_mmu_res", None) is not None:
            del skip._mmu_res  # read by this bn3 only: free the residue with the block
        return out


def resnet152_trunk(blocks=(3, 8, 36, 3)):
    """Sequential(conv1, bn1, relu, maxpool, layer1..layer4) -> [B,2048,H/32,W/32]."""
    stem_bn = BatchNorm2d(64)
    stem_bn.fused_relu = True
    mods = [StoreConv2d(3, 64, 7, stride=2, padding=3, bias=False), stem_bn, FusedReLU(inplace=True),
            MaxPool2d(3, 2, 1)]
    cin = 64
    for i, (width, n) in enumerate(zip((64, 128, 256, 512), blocks)):
        stage = []
        for b in range(n):
            stage.append(Bottleneck(cin, width, 2 if (b == 0 and i > 0) else 1))
            cin = width * 4
        mods.append(nn.Sequential(*stage))
    trunk = nn.Sequential(*mods)
    for m in trunk.modules():
        if isinstance(m, nn.Conv2d):
            nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
        elif isinstance(m, nn.BatchNorm2d):
            nn.init.ones_(m.weight)
            nn.init.zeros_(m.bias)
    return trunk
