"""CPU, world_size 2 over gloo: the DP gradient bucketer (src/dp.py) averages the flat
gradient buffer exactly, launching a bucket as soon as its layers report ready, and
broadcast_parameters makes every rank start from rank 0's weights."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


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
        from src.dp import GradBucketer, broadcast_parameters
        from src.mmbt import MultimodalBertClf
        from src.testing import small_args
        torch.manual_seed(100 + rank)  # different init per rank on purpose
        model = MultimodalBertClf(small_args())
        broadcast_parameters(model)
        w_sum = float(model.store.flat.double().sum())
        bk = GradBucketer(model, bucket_bytes=8 << 20)
        g = torch.Generator().manual_seed(rank)
        model.store.grad.copy_(torch.randn(model.store.numel(), generator=g))
        launched = []
        for lw in reversed(model.enc._lw):  # backward order: top layer first
            bk._on_ready(lw)
            launched.append(len(bk.launched))
        bk.finish()
        q.put((rank, w_sum, model.store.grad.double().sum().item(), model.store.grad[:1000].tolist(), launched,
               len(bk.buckets)))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, "ERR", traceback.format_exc()))


def test_bucketed_allreduce_matches_mean():
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
    res.sort()
    # expected mean of the two ranks' random gradients
    sizes = None
    gens = [torch.Generator().manual_seed(r) for r in range(world)]
    from src.mmbt import MultimodalBertClf
    from src.testing import small_args
    n = MultimodalBertClf(small_args()).store.numel()
    mean = sum(torch.randn(n, generator=g).double() for g in gens) / world
    for rank, w_sum, gsum, head, launched, nb in res:
        assert abs(gsum - float(mean.sum())) < 1e-3 * abs(float(mean.sum())) + 1e-2
        torch.testing.assert_close(torch.tensor(head, dtype=torch.float64), mean[:1000], rtol=1e-5, atol=1e-6)
        assert launched[-1] >= 1, "no bucket launched during backward"
    assert res[0][1] == res[1][1], "ranks start from different weights"
