"""Diagnose the 2-rank sync-BN parity: single device on the global batch vs two ranks on its
halves (gloo, one GPU), with and without the gradient bucketer; prints the worst tensors."""
import os
import socket
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))


def worker(rank, world, port, q, prec, use_bucketer, sync):
    sys.path[:0] = [os.path.join(HERE, "..", "multi-modal-uncertainty_amd"), os.path.join(HERE, "..")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.backends.cudnn.deterministic = True
    from src.dp import GradBucketer, broadcast_parameters, convert_sync_batchnorm
    from src.mmbt import MultimodalBertClf
    from src.testing import small_args, synthetic_batch
    from oracle.weights import SMALL
    dev, B = "cuda:0", 8

    def make():
        torch.manual_seed(0)
        m = MultimodalBertClf(small_args(bert_hidden_dropout=0.0, bert_attn_dropout=0.0, dropout=0.0,
                                         img_precision=prec)).to(dev)
        return m.train()
    x, y = synthetic_batch(B, 16, lens=[16, 9, 12, 16, 5, 16, 11, 14], vocab=SMALL.vocab, seed=31)
    x, y = tuple(t.to(dev) for t in x), y.to(dev)
    m1 = make()
    m1.store.zero_grad()
    m1.compute_loss(m1(*x), y).backward()
    g1 = m1.store.grad.clone()
    m2 = make()
    broadcast_parameters(m2)
    if sync:
        convert_sync_batchnorm(m2)
    bk = GradBucketer(m2, bucket_bytes=1 << 20) if use_bucketer else None
    sl = slice(rank * B // world, (rank + 1) * B // world)
    m2.store.zero_grad()
    m2.compute_loss(m2(*(t[sl] for t in x)), y[sl]).backward()
    if bk is not None:
        bk.finish()
    else:
        dist.all_reduce(m2.store.grad)
        m2.store.grad.mul_(0.5)
    g2 = m2.store.grad.clone()
    torch.cuda.synchronize()
    rows = []
    for n in m2.store.names:
        o, k = m2.store.offsets[n], m2.store.params[n].numel()
        a, b = g1[o:o + k], g2[o:o + k]
        rows.append(((a - b).norm() / (a.norm() + 1e-30)).item())
    worst = sorted(zip(rows, m2.store.names), reverse=True)[:12]
    q.put((rank, ((g2 - g1).norm() / g1.norm()).item(), worst))
    dist.destroy_process_group()


def main():
    for prec in ("fp32",):
        for use_bk in (False, True):
            for sync in (True, False):
                s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
                ctx = mp.get_context("spawn")
                q = ctx.Queue()
                ps = [ctx.Process(target=worker, args=(r, 2, port, q, prec, use_bk, sync)) for r in range(2)]
                for p in ps:
                    p.start()
                res = sorted([q.get(timeout=300) for _ in range(2)])
                for p in ps:
                    p.join(timeout=60)
                r0 = res[0]
                print(f"== {prec} bucketer={use_bk} sync={sync}: grad rel err {r0[1]:.3e}", flush=True)
                for e, n in r0[2][:8]:
                    print(f"   {e:.3e}  {n}", flush=True)


if __name__ == "__main__":
    main()
