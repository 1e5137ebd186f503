"""Data-parallel MMBT training: one process per GPU, RCCL gradient all-reduce over xGMI.

The reference is single-device (train.py:307-310); this is the build's DP layer
(SURVEY §8e).  Gradients already live in ONE flat f32 buffer laid out in the
order backward completes them (src/params.py), so buckets are plain contiguous
slices: [classifier + pooler + layer 11 ...], ..., [layer 0 ...], [embeddings +
image projection + ResNet].  Each fused BERT layer's backward reports when its
weight gradients are enqueued, the embedding backward when the embedding tables'
are, and each ResNet residual block when the gradient of its input is formed (a
tensor hook on the block input, registered by a forward pre-hook: by then every
parameter gradient of the block is enqueued); as soon as a bucket's parts are all
done its all-reduce (torch.distributed backend "nccl" = RCCL) is issued.  The collective
runs on RCCL's own stream, ordered after the producing kernels by an event, so it
overlaps the backward of the layers below.  ``finish()`` issues what is left and
makes the compute stream wait before the optimizer step.  Mean = sum / world size
(the per-rank loss is a per-rank mean over equal per-rank batches).

``optimizer`` (a src.optim.BertAdam): ``finish()`` leaves the rank SUM in the gradient store and
sets the optimizer's ``grad_scale`` to 1/world for its next step, whose fused kernel folds the
mean into the clip coefficient -- no separate pass over the 677 MB f32 gradient buffer.
Without it ``finish()`` divides the store in place (the gradients read as the mean).

``reduce_dtype=torch.bfloat16`` all-reduces a bf16 copy of each bucket (half the xGMI
bytes; every averaged gradient rounded to 8 significant bits before BertAdam) and casts the
sum back into the f32 store at ``finish()``; the default keeps the f32 buckets
(DESIGN §6 has the measured comparison).
"""
import torch
import torch.distributed as dist

from . import kernels as K


class GradBucketer:
    def __init__(self, model, bucket_bytes=64 << 20, group=None, reduce_dtype=torch.float32, optimizer=None):
        self.model = model
        self.optimizer = optimizer
        self.reduce_dtype = reduce_dtype
        self._lowp = {}  # bucket -> low-precision copy being all-reduced
        self.enc = model.enc
        self.store = model.store
        self.group = group
        self.world = dist.get_world_size(group)
        self.bucket_bytes = bucket_bytes
        self._plan()
        self.enc._grad_ready_hook = self._on_ready
        self.pending = []
        self.launched = set()
        self.done_segs = set()
        self.enabled = True
        self._trunk_side = False
        self._hooks = [m.register_forward_pre_hook(self._block_pre_hook(k)) for k, m in self._blocks.items()]

    def _plan(self):
        st = self.store
        n_layers = len(self.enc._lw)
        # flat order: clf, pooler, layer n-1 ... layer 0, embeddings, img proj, resnet (reverse)
        layer_spans = []
        for i in reversed(range(n_layers)):
            names = [n for n in st.names if n.startswith(f"{self.enc._prefix}encoder.layer.{i}.")]
            o0 = min(st.offsets[n] for n in names)
            o1 = max(st.offsets[n] + st.params[n].numel() for n in names)
            layer_spans.append((i, o0, o1))
        head_end = layer_spans[0][1]
        buckets, cur = [], None
        for i, o0, o1 in layer_spans:
            if cur is None:
                cur = {"start": 0 if i == n_layers - 1 else o0, "end": o1, "layers": {i}}
            else:
                cur["end"] = o1
                cur["layers"].add(i)
            if 4 * (cur["end"] - cur["start"]) >= self.bucket_bytes:
                buckets.append(cur)
                cur = None
        if cur is not None:
            buckets.append(cur)
        assert head_end == 0 or buckets[0]["start"] == 0
        tail_start = buckets[-1]["end"]
        total = st.numel()
        # tail: embeddings + image projection ("emb"), then the ResNet residual blocks in
        # backward order (layer4 last block ... layer1 first block), then the stem: buckets of
        # whole segments, each issued when its segments' gradients are all enqueued (the stem's
        # at finish())
        segs = []  # (key, start, end) in flat order
        for n in st.names:
            o = st.offsets[n]
            if o < tail_start:
                continue
            key = self._segment_of(n)
            if segs and segs[-1][0] == key:
                segs[-1][2] = max(segs[-1][2], o + st.params[n].numel())
            else:
                segs.append([key, o, o + st.params[n].numel()])
        assert not segs or segs[0][1] == tail_start
        cur = None
        for key, o0, o1 in segs:
            if cur is None:
                cur = {"start": o0, "end": o1, "layers": set(), "segs": {key}}
            else:
                cur["end"] = o1
                cur["segs"].add(key)
            if 4 * (cur["end"] - cur["start"]) >= self.bucket_bytes:
                buckets.append(cur)
                cur = None
        if cur is not None:
            buckets.append(cur)
        self.buckets = buckets
        self.seg_to_buckets = {}
        for b, bk in enumerate(buckets):
            for key in bk.get("segs", ()):
                self.seg_to_buckets.setdefault(key, []).append(b)
        prefix = f"{self.enc._prefix}img_encoder."
        mods = dict(self.enc.img_encoder.named_modules(prefix=prefix[:-1]))
        self._blocks = {key: mods[key] for key, _, _ in segs if key not in ("emb", "proj", "stem") and key in mods}
        self.layer_to_bucket = {i: b for b, bk in enumerate(buckets) for i in bk["layers"]}
        self.done_layers = set()

    def _segment_of(self, name):
        """tail segment of a parameter: "emb" (text embeddings), "proj" (the image projection,
        reported by ProjectFunction.backward once its dW / db are enqueued), the ResNet residual
        block ``<prefix>img_encoder.model.<stage>.<block>`` (stages 4..7 = layer1..layer4), or
        "stem"."""
        prefix = f"{self.enc._prefix}img_encoder."
        if name.startswith(f"{self.enc._prefix}img_embeddings.img_embeddings."):
            return "proj"
        if not name.startswith(prefix):
            return "emb"
        parts = name[len(prefix):].split(".")
        if len(parts) >= 3 and parts[0] == "model" and parts[1] in ("4", "5", "6", "7"):
            return prefix + ".".join(parts[:3])
        return "stem"

    def _block_pre_hook(self, key):
        def pre(module, args):
            x = args[0] if args else None
            if (self.enabled and self.world > 1 and torch.is_grad_enabled() and isinstance(x, torch.Tensor)
                    and x.requires_grad):
                # the block's filter gradients go to the side stream at this batch (resnet._wgrad_run)
                from .resnet import _side_wgrad
                self._trunk_side = _side_wgrad(x)
                x.register_hook(lambda g: self._on_segment(key))
        return pre

    def _on_segment(self, key):
        """a tail segment's gradients are all enqueued: issue the buckets it completes"""
        if not self.enabled or self.world == 1:
            return
        self.done_segs.add(key)
        for b in self.seg_to_buckets.get(key, ()):
            segs = self.buckets[b]["segs"]
            if "stem" not in segs and segs <= self.done_segs:
                self._issue(b)

    def _issue(self, b):
        if b in self.launched:
            return
        bk = self.buckets[b]
        view = self.store.grad[bk["start"]:bk["end"]]
        side = K.side_stream_if_any(view.device) if view.is_cuda else None
        if side is not None and torch.cuda.current_stream(view.device) != side:
            # from the main stream, a bucket goes behind the side stream's work only when some
            # of its gradients are written there: the ResNet blocks' filter gradients at batches
            # that put them on the side stream (the encoder layers' buckets are issued from the
            # deferred work itself, already on the side stream); the embedding / projection
            # buckets stay on the main stream so they do not queue behind deferred work
            segs = bk.get("segs", ())
            if not (self._trunk_side and any(k not in ("emb", "proj") for k in segs)):
                side = None

        def reduce():
            buf = view
            if self.reduce_dtype != view.dtype:
                buf = self._lowp[b] = view.to(self.reduce_dtype)
            return dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        if side is not None:
            # filter gradients may still be in flight on the side stream (src/resnet.py
            # _wgrad_run): the all-reduce is issued from it, behind the main stream's work too
            side.wait_stream(torch.cuda.current_stream(view.device))
            with torch.cuda.stream(side):
                work = reduce()
        else:
            work = reduce()
        self.pending.append(work)
        self.launched.add(b)

    def _on_ready(self, lw):
        if lw in ("embeddings", "proj"):
            self._on_segment({"embeddings": "emb", "proj": "proj"}[lw])
            return
        if not self.enabled or self.world == 1 or not hasattr(lw, "module"):
            return
        i = self.enc._lw.index(lw)
        self.done_layers.add(i)
        b = self.layer_to_bucket[i]
        if self.buckets[b]["layers"] <= self.done_layers:
            self._issue(b)

    def finish(self):
        """Issue the remaining buckets, wait for all, average."""
        if self.world == 1:
            return
        for b in range(len(self.buckets)):
            self._issue(b)
        for w in self.pending:
            w.wait()
        cur = torch.cuda.current_stream(self.store.grad.device) if self.store.grad.is_cuda else None
        for b, buf in self._lowp.items():
            bk = self.buckets[b]
            self.store.grad[bk["start"]:bk["end"]].copy_(buf)
            if cur is not None:  # (allocated on the side stream, read here: keep it until this copy ran)
                buf.record_stream(cur)
        if self.optimizer is not None and hasattr(self.optimizer, "grad_scale"):
            self.optimizer.grad_scale = 1.0 / self.world
        else:
            self.store.grad.mul_(1.0 / self.world)
        self.pending, self.launched, self.done_layers, self.done_segs = [], set(), set(), set()
        self._lowp = {}


def convert_sync_batchnorm(model, group=None):
    """Normalise the image trunk over the whole data-parallel batch, as the single-device
    reference does (src/mmbt.py:19-21; SURVEY §8e "DP + BatchNorm"): every BatchNorm2d of
    ``model`` exchanges its per-channel sums with the other ranks in training
    (resnet._SyncBatchNormAct, one all-reduce of 2C+1 f64 per BN per pass: 2 x 155 small
    collectives per step).  The exchanges run on a communicator of their own (a new group over
    the same ranks), so they do not queue behind the gradient buckets' all-reduces.  Without
    it every rank normalises over its own per-rank batch (the default: no collective on the
    forward's critical path).  Returns the number of BatchNorm2d modules converted."""
    from .resnet import BatchNorm2d
    if dist.get_world_size(group) == 1:
        return 0
    ranks = dist.get_process_group_ranks(group) if group is not None else list(range(dist.get_world_size()))
    sync = dist.new_group(ranks=ranks)
    n = 0
    for m in model.modules():
        if isinstance(m, BatchNorm2d):
            m.sync_group = sync
            n += 1
    return n


def average_buffers(model, group=None):
    """Average the floating-point buffers (ResNet BatchNorm running_mean / running_var) over
    the ranks.  Each rank's BatchNorm normalises over its own batch in training, so the
    running statistics drift apart between ranks; averaging them before evaluation and
    checkpointing gives every rank (and the rank-0 checkpoint) the same statistics, the
    mean of what the ranks saw.  num_batches_tracked (integer) is equal on every rank."""
    world = dist.get_world_size(group)
    if world == 1:
        return
    bufs = [b for b in model.buffers() if b.is_floating_point()]
    if not bufs:
        return
    flat = torch._utils._flatten_dense_tensors(bufs)
    dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
    flat.mul_(1.0 / world)
    for b, f in zip(bufs, torch._utils._unflatten_dense_tensors(flat, bufs)):
        b.copy_(f)


def sync_buffers_on_eval(model, group=None):
    """Call average_buffers whenever the model leaves training mode (model.eval() /
    model.train(False), as Model_.eval_loop does before validation, test and checkpoints)."""
    train = model.train

    def train_(mode=True):
        if not mode and model.training:
            average_buffers(model, group)
        return train(mode)
    model.train = train_
    return model


def broadcast_parameters(model, src=0, group=None):
    """Start every rank from rank 0's weights (flat buffer + BN running stats)."""
    dist.broadcast(model.store.flat, src, group=group)
    for b in model.buffers():
        dist.broadcast(b, src, group=group)
    model.store.sync_compute()
