"""Flat parameter / gradient / bf16-compute storage for the MMBT module tree.

Every trainable tensor of the model is a view into ONE f32 master buffer and its
``.grad`` a view into ONE f32 gradient buffer, laid out in the order backward
finishes them (classifier, pooler, encoder layers 11..0, embeddings, ResNet
layer4..stem).  This gives:
  * the fused BertAdam one launch over all 169 M parameters (src/optim.py);
  * contiguous reverse-layer gradient buckets for the RCCL all-reduce (src/dp.py);
  * fused views (Q|K|V weight [2304,768], bias [2304]) the kernels read directly;
  * bf16 copies of every GEMM weight, written by the optimizer kernel, resynced
    only when the f32 masters were changed elsewhere (load_state_dict, .to());
  * transposed (K-major) bf16 copies of registered fused weights (the BERT layer
    matrices: the data-gradient GEMMs read them as a K-major B operand), refreshed by
    one batched transpose launch after every write of the bf16 copies.
Module names / shapes are untouched, so state_dict keys stay the reference's.
"""
import weakref

import torch

STORES = weakref.WeakSet()  # live stores, looked up by the fused optimizer


class ParamStore:
    def __init__(self, entries, compute_names):
        """entries: [(name, Parameter)] in flat order (unique params);
        compute_names: names (subset) that get a bf16 GEMM copy, in bf16 flat order."""
        self.names = [n for n, _ in entries]
        self.params = dict(entries)
        self.compute_names = list(compute_names)
        self.flat = self.grad = self.compute = None
        self.offsets, self.coffsets = {}, {}
        self._versions = None
        self._tspecs = {}  # key (tuple of names) -> shape [rows, cols] of the fused compute view
        self._tcopies = {}
        self._fcopies = {}  # conv filter name -> flipped, transposed bf16 copy [Cin, 3, 3, Cout]
        self._tjobs = None
        self._cviews = {}  # name -> compute_of view (rebuilt with the buffers)
        self.build()
        STORES.add(self)

    # ------------------------------------------------------------------ layout
    @staticmethod
    def _shaped(buf, off, p):
        """view of buf[off:off+numel] with p's shape; 4-D conv weights are laid out channels-last
        (O, kh, kw, I) so MIOpen sees NHWC activations AND NHWC filters."""
        k = p.numel()
        if p.dim() == 4:
            O, I, kh, kw = p.shape
            return buf[off:off + k].view(O, kh, kw, I).permute(0, 3, 1, 2)
        return buf[off:off + k].view(p.shape)

    def build(self):
        ps = [self.params[n] for n in self.names]
        device = ps[0].device
        total = sum(p.numel() for p in ps)
        flat = torch.empty(total, dtype=torch.float32, device=device)
        grad = torch.zeros(total, dtype=torch.float32, device=device)
        off = 0
        for n, p in zip(self.names, ps):
            k = p.numel()
            if p.device != device:
                raise RuntimeError(f"ParamStore: {n} on {p.device}, expected {device}")
            pv, gv = self._shaped(flat, off, p), self._shaped(grad, off, p)
            pv.copy_(p.detach())
            if p.grad is not None:
                gv.copy_(p.grad.detach())
            p.data = pv
            p.grad = gv
            self.offsets[n] = off
            off += k
        self.flat, self.grad = flat, grad
        self._cviews = {}
        ctot = sum(self.params[n].numel() for n in self.compute_names)
        self.compute = torch.empty(ctot, dtype=torch.bfloat16, device=device)
        off = 0
        for n in self.compute_names:
            self.coffsets[n] = off
            off += self.params[n].numel()
        # transposed and flipped copies are re-allocated on the (new) device: a job table
        # holding the old buffers' pointers would write through a foreign-device pointer
        self._tcopies, self._tjobs = {}, None
        for key, shape in self._tspecs.items():
            self._alloc_transposed(key, shape)
        for name in list(self._fcopies):
            O, I = self.params[name].shape[:2]
            self._fcopies[name] = torch.empty(I, 3, 3, O, dtype=torch.bfloat16, device=device)
        self.sync_compute()

    @property
    def device(self):
        return self.flat.device

    def numel(self):
        return self.flat.numel()

    def span(self, names):
        """(offset, numel) of a run of consecutive names in the flat buffer"""
        o0 = self.offsets[names[0]]
        tot = 0
        for n in names:
            if self.offsets[n] != o0 + tot:
                raise RuntimeError(f"ParamStore: {names} are not contiguous")
            tot += self.params[n].numel()
        return o0, tot

    def fused(self, names, shape):
        o, k = self.span(names)
        return self.flat[o:o + k].view(shape)

    def fused_grad(self, names, shape):
        o, k = self.span(names)
        return self.grad[o:o + k].view(shape)

    def fused_compute(self, names, shape):
        c0 = self.coffsets[names[0]]
        tot = 0
        for n in names:
            if self.coffsets[n] != c0 + tot:
                raise RuntimeError(f"ParamStore: compute copies of {names} are not contiguous")
            tot += self.params[n].numel()
        return self.compute[c0:c0 + tot].view(shape)

    def transposed_compute(self, names, shape):
        """bf16 [cols, rows] copy of the fused compute view ``names`` ([rows, cols]), kept in
        step with the bf16 copies (sync_compute, and sync_transposed after the optimizer)."""
        key = tuple(names)
        if key not in self._tspecs:
            self._tspecs[key] = tuple(shape)
            self._alloc_transposed(key, shape)
            self.sync_transposed()
        return self._tcopies[key]

    def _alloc_transposed(self, key, shape):
        rows, cols = shape
        self._tcopies[key] = torch.empty(cols, rows, dtype=torch.bfloat16, device=self.compute.device)
        self._tjobs = None

    def flipped_filter(self, name):
        """bf16 [Cin, 3, 3, Cout] copy of the 3x3 filter ``name`` flipped in both taps (the B
        operand of the conv data gradient as an implicit GEMM, src/resnet.py), kept in step
        with the bf16 copies like the transposed ones (9 strided jobs of the same launch)."""
        if name not in self._fcopies:
            O, I, kh, kw = self.params[name].shape
            assert (kh, kw) == (3, 3), name
            self._fcopies[name] = torch.empty(I, 3, 3, O, dtype=torch.bfloat16, device=self.compute.device)
            self._tjobs = None
            self.sync_transposed()
        return self._fcopies[name]

    def sync_transposed(self):
        """Refresh every transposed / flipped copy from the bf16 copies: ONE batched HIP launch."""
        if not self._tcopies and not self._fcopies:
            return
        if self._tjobs is None:
            rows = []
            for key, dst in self._tcopies.items():
                r, c = self._tspecs[key]
                src = self.fused_compute(list(key), (r, c))
                rows.append([src.data_ptr(), dst.data_ptr(), r, c, 0, 0])
            for name, dst in self._fcopies.items():  # src [O][t][I] -> dst[i][8 - t][o], one job per tap
                O, I = self.params[name].shape[:2]
                base = self.compute_of(name).data_ptr()
                for t in range(9):
                    rows.append([base + 2 * t * I, dst.data_ptr() + 2 * (8 - t) * O, O, I, 9 * I, 9 * O])
            self._tjobs = (torch.tensor(rows, dtype=torch.int64).to(self.compute.device), len(rows),
                           max(r[2] for r in rows), max(r[3] for r in rows))
        if self.compute.device.type != "cuda":
            for key, dst in self._tcopies.items():  # host-side stores (CPU tests): plain copy
                dst.copy_(self.fused_compute(list(key), self._tspecs[key]).t())
            for name, dst in self._fcopies.items():
                dst.copy_(self.compute_of(name).flip(2, 3).permute(1, 2, 3, 0))
            return
        from . import kernels as K
        jobs, n, mr, mc = self._tjobs
        K.transpose_bf16_batched(jobs, n, mr, mc, self.compute)

    def grad_of(self, name):
        return self._shaped(self.grad, self.offsets[name], self.params[name])

    # ------------------------------------------------------------------ grads
    def ensure_grads(self, quick=False):
        """Re-attach grad views if a caller dropped them (e.g. Module.zero_grad(set_to_none=True)).
        quick: only look at the first / last tensor (what set_to_none touches: all of them)."""
        base = self.grad.data_ptr()
        names = self.names
        if quick:
            ends = [names[0], names[-1]]
            if all(self.params[n].grad is not None and
                   self.params[n].grad.data_ptr() == base + 4 * self.offsets[n] for n in ends):
                return
        params, offsets = self.params, self.offsets
        for n in names:
            p = params[n]
            o = offsets[n]
            g = p.grad
            if g is not None and g.data_ptr() == base + 4 * o:
                continue  # (the common case: no view to build)
            view = self._shaped(self.grad, o, p)
            if g is None:
                view.zero_()
            else:
                view.copy_(g)
            p.grad = view

    def zero_grad(self):
        self.ensure_grads()
        self.grad.zero_()

    # ------------------------------------------------------------------ bf16 copies
    def _current_versions(self):
        return tuple(self.params[n]._version for n in self.compute_names)

    def sync_compute(self):
        """bf16 copy of every compute tensor in its STORAGE order (conv weights: O, kh, kw, I),
        the order the fused optimizer writes them in."""
        with torch.no_grad():
            for n in self.compute_names:
                c, o, k = self.coffsets[n], self.offsets[n], self.params[n].numel()
                self.compute[c:c + k].copy_(self.flat[o:o + k])
        self._versions = self._current_versions()
        self.sync_transposed()

    def compute_of(self, name):
        """bf16 copy of one tensor, shaped like the parameter (conv weights channels-last);
        the view is cached until the buffers are rebuilt (build())."""
        v = self._cviews.get(name)
        if v is None:
            v = self._cviews[name] = self._shaped(self.compute, self.coffsets[name], self.params[name])
        return v

    def maybe_sync_compute(self):
        """bf16 copies follow the masters; only an out-of-band write (version bump) needs a resync."""
        if self._current_versions() != self._versions:
            self.sync_compute()

    def check_views(self):
        """True if every parameter still aliases the flat buffer (Module._apply breaks this)."""
        flat = self.flat
        base, dev, params, offsets = flat.data_ptr(), flat.device, self.params, self.offsets
        # (a data pointer inside the flat buffer's allocation implies its device; the device is
        # compared for one tensor to catch a store whose buffer moved)
        return params[self.names[0]].device == dev and all(
            params[n].data_ptr() == base + 4 * offsets[n] for n in self.names)
