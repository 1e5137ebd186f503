"""Is the train step host-bound at a given per-rank batch?  Times bench.py's step three ways on one
GPU: (a) wall per step with the roofline instrumentation on (GEMM / block HIP events, as the timed
region of bench.py), (b) wall per step without it, (c) host time to enqueue one step while the GPU
is still busy with the previous ones (the step's Python / launch cost).

  python tools/host_time.py [--batch 32] [--steps 20]
"""
import argparse
import os
import sys
import time

import torch

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "multi-modal-uncertainty_amd"))
os.environ.setdefault("MIOPEN_USER_DB_PATH", os.path.join(REPO, "multi-modal-uncertainty_amd", "miopen_db"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    from src.mmbt import MultimodalBertClf
    from src.optim import BertAdam
    from src.testing import make_args, synthetic_batch
    from src import kernels as K
    from src import encoder
    torch.backends.cudnn.benchmark = True
    dev = torch.device("cuda", 0)
    torch.manual_seed(1234)
    model = MultimodalBertClf(make_args()).to(dev)
    opt = BertAdam([{"params": list(model.parameters()), "weight_decay": 0.01}], lr=5e-5, warmup=0.1,
                   t_total=10000.0)
    x, y = synthetic_batch(a.batch, 508, seed=100, device=dev)
    model.train()

    def step():
        opt.zero_grad()
        loss = model.compute_loss(model(*x), y)
        loss.backward()
        opt.step()
        return loss

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    for inst in (True, False, True, False):
        K.timing_enable(inst)
        encoder.block_timing(inst)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        host = []
        for _ in range(a.steps):
            h0 = time.perf_counter()
            step()
            host.append(time.perf_counter() - h0)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.steps
        if inst:
            K.timing_read()
            encoder.block_timing_read()
        K.timing_enable(False)
        encoder.block_timing(False)
        host.sort()
        print(f"batch {a.batch} instrumentation {'on ' if inst else 'off'}: wall {dt * 1e3:6.2f} ms per step, "
              f"host enqueue median {host[len(host) // 2] * 1e3:6.2f} ms (min {host[0] * 1e3:6.2f})", flush=True)


if __name__ == "__main__":
    main()
