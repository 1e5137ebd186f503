"""Two ranks on ONE MI355X over gloo (RCCL needs one GPU per rank; the 8-GPU RCCL run is
the driver's): a real bf16 training backward of the small MMBT with the gradient
bucketer (src/dp.py) attached, so its buckets are launched by the hooks that fire inside
backward -- the BERT layers', the embedding backward's and the ResNet blocks' input-gradient
hooks -- and the flat gradient after finish() equals the mean of the two ranks' local
gradients (each rank's own backward without the bucketer, all-gathered)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    try:
        import sys
        here = os.path.dirname(os.path.abspath(__file__))
        sys.path[:0] = [os.path.join(os.path.dirname(here), "multi-modal-uncertainty_amd"), os.path.dirname(here)]
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.backends.cudnn.deterministic = True
        from src.dp import GradBucketer, broadcast_parameters
        from src.mmbt import MultimodalBertClf
        from src.testing import small_args, synthetic_batch
        from oracle.weights import SMALL
        dev = "cuda:0"
        torch.manual_seed(0)
        model = MultimodalBertClf(small_args(bert_hidden_dropout=0.0, bert_attn_dropout=0.0, dropout=0.0))
        model = model.to(dev).train()
        broadcast_parameters(model)
        x, y = synthetic_batch(4, 16, vocab=SMALL.vocab, seed=10 + rank)  # a different batch per rank
        x, y = tuple(t.to(dev) for t in x), y.to(dev)

        def backward():
            model.store.zero_grad()
            model.compute_loss(model(*x), y).backward()
            torch.cuda.synchronize()

        backward()  # local gradient (no bucketer yet)
        local = model.store.grad.clone()
        bk = GradBucketer(model, bucket_bytes=4 << 20)
        issued = []
        orig = bk._issue

        def spy(b):
            issued.append((b, b in bk.launched))
            orig(b)
        bk._issue = spy
        backward()
        during = len(bk.launched)
        n_tail = sum(1 for b, _ in issued if "segs" in bk.buckets[b])
        bk.finish()
        torch.cuda.synchronize()
        got = model.store.grad.clone()
        parts = [torch.empty_like(local) for _ in range(world)]
        dist.all_gather(parts, local)
        want = sum(parts) / world
        err = (got - want).abs().max().item()
        scale = want.abs().max().item()
        q.put((rank, err, scale, during, len(bk.buckets), n_tail, (local - want).abs().max().item()))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, "ERR", traceback.format_exc()))


def test_bucketer_hooks_average_real_backward():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    errs = [r for r in res if r[1] == "ERR"]
    assert not errs, errs[0][2]
    for rank, err, scale, during, nb, n_tail, spread in res:
        assert spread > 1e-6 * scale, "the ranks' local gradients are identical: the test would not see a mix-up"
        assert err <= 1e-6 * scale + 1e-9, f"rank {rank}: averaged gradient off by {err:.3e} (scale {scale:.3e})"
        assert during >= 1, "no bucket launched inside backward"
        assert n_tail >= 1, "no embedding / trunk bucket launched inside backward"
