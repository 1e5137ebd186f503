"""BASELINE config 4 on the FULL model (ResNet-152 + 12 BERT layers, L = 513): two ranks on ONE
MI355X over gloo (RCCL needs one GPU per rank; the 8-GPU RCCL run is the driver's), per-rank
batch 2 against one device at batch 4 (reference single-device step: src/framework.py:276-304,
BertAdam at train.py:136-147).  The small-model versions are in tests/test_dp_gpu.py; these
exercise what only the real model has: 64 MB buckets cut through 12 layers and the 334 MB tail,
the per-residual-block trunk segments of all 50 Bottlenecks, the deferred side-stream BERT
weight gradients with their memory budget's early flush, and BertAdam applying the 1/world
mean itself (dp.GradBucketer(optimizer=...)).

Weights: the conditioned recipe (oracle/weights.py FULL_C) -- the round-1 recipe's trunk is
chaotic (tests/test_oracle.py::test_trunk_conditioning_of_the_fixture_recipes), which would
turn the two sides' f32 summation-order differences into trunk-sized ones."""
import os

import pytest
import torch
import torch.distributed as dist

from test_dp_gpu import _spawn

pytestmark = pytest.mark.gpu

B, T = 4, 508


def _setup(rank, world, port):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.join(os.path.dirname(here), "multi-modal-uncertainty_amd"), os.path.dirname(here)]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.backends.cudnn.deterministic = True


def _model(prec, sd):
    from src.mmbt import MultimodalBertClf
    from src.optim import BertAdam
    from src.testing import make_args
    torch.manual_seed(0)
    m = MultimodalBertClf(make_args(bert_hidden_dropout=0.0, bert_attn_dropout=0.0, dropout=0.0, img_precision=prec))
    m.load_state_dict(sd, strict=True)
    m = m.to("cuda:0")
    named = list(m.named_parameters())
    nd = ["bias", "LayerNorm.bias", "LayerNorm.weight"]
    groups = [{"params": [p for n, p in named if not any(k in n for k in nd)], "weight_decay": 0.01},
              {"params": [p for n, p in named if any(k in n for k in nd)], "weight_decay": 0.0}]
    return m, BertAdam(groups, lr=1e-3, warmup=0.1, t_total=10.0)


def _batch():
    from src.testing import synthetic_batch
    x, y = synthetic_batch(B, T, lens=[508, 300, 508, 77], seed=41)
    return tuple(t.to("cuda:0") for t in x), y.to("cuda:0")


def _exact_worker(rank, world, port, q, variant):
    """the bucketed all-reduce inside the real backward == the mean of the ranks' local
    gradients (each rank's own backward without the bucketer, all-gathered), with the product
    bf16 trunk in training mode"""
    try:
        _setup(rank, world, port)
        from oracle.weights import FULL_C, make_state_dict
        from src import encoder as E
        from src import resnet as R
        from src.dp import GradBucketer, broadcast_parameters
        if variant == "side_flush":
            R.SIDE_WGRAD_MIN_BATCH = 1   # every trunk filter gradient on the side stream
            E.DEFER_MAX_BYTES = 1        # the deferred BERT weight-gradient work issued after every piece
        m, _ = _model("bf16", make_state_dict(0, FULL_C))
        m.train()
        broadcast_parameters(m)
        x, y = _batch()
        sl = slice(rank * B // world, (rank + 1) * B // world)
        xs, ys = tuple(t[sl] for t in x), y[sl]

        def backward():
            m.store.zero_grad()
            torch.manual_seed(5)
            m.compute_loss(m(*xs), ys).backward()
            torch.cuda.synchronize()

        backward()
        local = m.store.grad.clone()
        bk = GradBucketer(m)  # the default 64 MB buckets
        issued = []
        orig = bk._issue
        bk._issue = lambda b: (issued.append(b), orig(b))
        backward()
        during = len(bk.launched)
        bk.finish()
        torch.cuda.synchronize()
        got = m.store.grad.clone()
        parts = [torch.empty_like(local) for _ in range(world)]
        dist.all_gather(parts, local)
        want = sum(parts) / world
        n_trunk = sum(1 for b in issued if any(k not in ("emb", "proj") for k in bk.buckets[b].get("segs", ())))
        q.put((rank, ((got - want).norm() / want.norm()).item(), ((local - want).norm() / want.norm()).item(),
               during, len(bk.buckets), n_trunk))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, "ERR", traceback.format_exc()))


@pytest.mark.parametrize("variant", ["default", "side_flush"])
def test_dp_full_model_bucketer_averages_real_backward(variant):
    """Bar: the averaged gradient equals the mean of the local gradients to 1e-6 (relative
    Frobenius; the two backwards are the same kernels on the same inputs, up to the float-
    atomic order of the bias column sums); the ranks' local gradients differ (different
    halves of the batch), buckets are launched from inside backward, trunk buckets among them.
    "side_flush": trunk filter gradients on the side stream and the deferred BERT weight-
    gradient work flushed after every piece (encoder.DEFER_MAX_BYTES = 1)."""
    for rank, err, spread, during, nb, n_trunk in _spawn(_exact_worker, 2, variant):
        print(f"\n[dp full {variant}] rank {rank}: averaged-gradient rel err {err:.3e} (local vs mean {spread:.3e}); "
              f"{during} of {nb} buckets launched inside backward, {n_trunk} of them trunk buckets")
        assert spread > 1e-3, "the ranks' local gradients are identical: the test would not see a mix-up"
        assert err <= 1e-6, err
        assert during >= nb // 2 and n_trunk >= 1, (during, nb, n_trunk)


def _parity_worker(rank, world, port, q):
    """one device on the global batch vs two ranks on its halves (BN on running statistics,
    dropout 0: the reference's single-device step, sample by sample), fp32 trunk, two BertAdam
    steps (the first has lr 0 under warmup_linear), the 1/world mean applied by BertAdam"""
    try:
        _setup(rank, world, port)
        from oracle.weights import FULL_C, make_state_dict
        from src.dp import GradBucketer, broadcast_parameters
        sd = make_state_dict(0, FULL_C)
        x, y = _batch()

        def run(ranks):
            m, o = _model("fp32", sd)
            m.eval()
            bk = None
            xs, ys = x, y
            if ranks:
                broadcast_parameters(m)
                bk = GradBucketer(m, optimizer=o)
                sl = slice(rank * B // world, (rank + 1) * B // world)
                xs, ys = tuple(t[sl] for t in x), y[sl]
            for it in range(2):
                p0 = m.store.flat.clone()
                o.zero_grad()
                m.compute_loss(m(*xs), ys).backward()
                if bk is not None:
                    bk.finish()
                    assert o.grad_scale == 1.0 / world  # the mean is BertAdam's
                g = m.store.grad.clone() * (o.grad_scale if bk is not None else 1.0)
                o.step()
            assert o.grad_scale == 1.0
            torch.cuda.synchronize()
            out = g, m.store.flat - p0
            del m, o
            torch.cuda.empty_cache()
            return out

        g1, d1 = run(False)
        g2, d2 = run(True)
        q.put((rank, ((g2 - g1).norm() / g1.norm()).item(), ((d2 - d1).norm() / d1.norm()).item(),
               d1.abs().max().item()))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, "ERR", traceback.format_exc()))


def test_dp_full_model_equal_single_device_global_batch():
    """SURVEY §8(e) at config 4's model: grads and the post-BertAdam parameter change of 2
    ranks x 2 samples == 1 device x 4 samples to 1e-6 relative (f32 buckets)."""
    for rank, gerr, perr, upd in _spawn(_parity_worker, 2):
        print(f"\n[dp full parity] rank {rank}: grad rel err {gerr:.3e}, post-step param-change rel err {perr:.3e}")
        assert upd > 0
        assert gerr <= 1e-6, gerr
        assert perr <= 1e-6, perr


def _sync_worker(rank, world, port, q):
    """TRAINING mode (batch statistics) with the bf16 product trunk: 2 ranks with whole-batch
    BatchNorm (dp.convert_sync_batchnorm) and 2 ranks without it, against the exact step (one
    device, fp32 trunk) and the single device's own bf16 step"""
    try:
        _setup(rank, world, port)
        from oracle.weights import FULL_C, make_state_dict
        from src.dp import GradBucketer, broadcast_parameters, convert_sync_batchnorm
        sd = make_state_dict(0, FULL_C)
        x, y = _batch()
        keep = None

        def run(prec, ranks, sync=False):
            nonlocal keep
            m, o = _model(prec, sd)
            m.train()
            xs, ys, bk = x, y, None
            if ranks:
                broadcast_parameters(m)
                if sync:
                    assert convert_sync_batchnorm(m) == 155
                bk = GradBucketer(m)
                sl = slice(rank * B // world, (rank + 1) * B // world)
                xs, ys = tuple(t[sl] for t in x), y[sl]
            o.zero_grad()
            m.compute_loss(m(*xs), ys).backward()
            if bk is not None:
                bk.finish()
            torch.cuda.synchronize()
            if keep is None:  # without the key biases: their true gradient is 0 (softmax shift invariance)
                keep = torch.ones_like(m.store.grad, dtype=torch.bool)
                trunk = torch.zeros_like(keep)
                for n in m.store.names:
                    sl_ = slice(m.store.offsets[n], m.store.offsets[n] + m.store.params[n].numel())
                    if n.endswith("attention.self.key.bias"):
                        keep[sl_] = False
                    if "img_encoder" in n:
                        trunk[sl_] = True
                keep = (keep, trunk)
            g = m.store.grad.clone()
            bufs = torch.cat([b.double().flatten() for b in m.buffers() if b.is_floating_point()])
            del m, o
            torch.cuda.empty_cache()
            return g, bufs

        gr, _ = run("fp32", False)
        g1, b1 = run("bf16", False)
        g2, b2 = run("bf16", True, sync=True)
        g3, _ = run("bf16", True, sync=False)
        rel = lambda a, b=gr, k=0: ((a - b)[keep[k]].norm() / b[keep[k]].norm()).item()  # noqa: E731
        # (the statistics show in the trunk's gradients: compared there, BERT's dominate the whole)
        q.put((rank, rel(g1), rel(g2), rel(g3, g1, 1), rel(g2, g1, 1), ((b2 - b1).norm() / b1.norm()).item(),
               rel(g1, gr, 1), rel(g2, gr, 1)))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, "ERR", traceback.format_exc()))


def test_dp_full_model_sync_batchnorm_train_mode():
    """Whole-batch BatchNorm under DP on the full trunk (155 BatchNorms exchanging their sums):
    the synchronised 2-rank bf16 step is no further from the exact step than 1.5x the single
    device's bf16 step, over all gradients and over the trunk's alone; per-rank statistics (no exchange) put the trunk's gradients >= 3x further
    from the single device's than the synchronised run does; the running statistics equal the
    single device's (1e-3: statistics of bf16 maps)."""
    for rank, e1, e2, e3, e2s, eb, e1t, e2t in _spawn(_sync_worker, 2):
        print(f"\n[dp full sync-bn] rank {rank}: grad rel err vs the exact step: single-device bf16 {e1:.3e} "
              f"(trunk {e1t:.3e}), 2-rank whole-batch BN {e2:.3e} (trunk {e2t:.3e}); trunk grads vs the single "
              f"device: whole-batch BN {e2s:.3e}, per-rank BN {e3:.3e}; running stats {eb:.3e}")
        assert e2 <= 1.5 * e1 + 1e-6, (e2, e1)
        assert e2t <= 1.5 * e1t + 1e-6, (e2t, e1t)
        assert e3 >= 3 * e2s, (e3, e2s)
        assert eb <= 1e-3, eb
