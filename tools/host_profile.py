"""cProfile of the train step's host side (bench.py's step at a per-rank batch): where the Python /
launch time of one step goes.

  python tools/host_profile.py [--batch 32] [--steps 5]
"""
import argparse
import cProfile
import os
import pstats
import sys

import torch

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "multi-modal-uncertainty_amd"))
os.environ.setdefault("MIOPEN_USER_DB_PATH", os.path.join(REPO, "multi-modal-uncertainty_amd", "miopen_db"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    from src.mmbt import MultimodalBertClf
    from src.optim import BertAdam
    from src.testing import make_args, synthetic_batch
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

    # the backward's Python (autograd Functions) on this thread, so the profile sees it
    torch.autograd.set_multithreading_enabled(False)
    for _ in range(5):
        step()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(a.steps):
        step()
    pr.disable()
    torch.cuda.synchronize()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(45)
    st.sort_stats("cumulative").print_stats(35)


if __name__ == "__main__":
    main()
