"""Where a ViLT classification step's time goes (bench.py --workload vilt's step): cProfile of the
host side over a few synchronised steps, plus each stage timed alone with a synchronize around it.

  python tools/vilt_profile.py [--batch 128] [--steps 5]
"""
import argparse
import cProfile
import os
import pstats
import sys
import time

import torch

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "multi-modal-uncertainty_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    from transformers import ViltConfig, ViltForImagesAndTextClassification
    from src.vilt import ViltHIP
    from src import vilt as V
    dev = torch.device("cuda", 0)
    torch.manual_seed(1234)
    g = torch.Generator().manual_seed(300)
    cfg = ViltConfig(num_images=1, num_labels=2)
    hip = ViltHIP(ViltForImagesAndTextClassification(cfg).eval(), dev)
    B, Lt = a.batch, cfg.max_position_embeddings
    ids = torch.randint(1000, cfg.vocab_size, (B, Lt), generator=g).to(dev)
    pix = torch.randn(B, 1, 3, cfg.image_size, cfg.image_size, generator=g).to(dev)
    mask = torch.ones(B, Lt, dtype=torch.long, device=dev)
    run = lambda: hip(ids, mask, None, pix, None)  # noqa: E731
    for _ in range(3):
        run()
    torch.cuda.synchronize()

    def timed(f, n=a.steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            f()
        torch.cuda.synchronize()
        return 1e3 * (time.perf_counter() - t0) / n

    print(f"step {timed(run):.2f} ms")
    p1 = pix[:, 0]
    pm = torch.ones(B, cfg.image_size, cfg.image_size, device=dev)
    print(f"  text embed {timed(lambda: hip._text(ids, None)):.2f} ms")
    print(f"  visual embed {timed(lambda: hip._visual(p1, pm, 1)):.2f} ms")
    xm = V.patch_mask(pm, 12, 12)
    print(f"    patch_mask {timed(lambda: V.patch_mask(pm, 12, 12)):.2f} ms")
    print(f"    select_patches {timed(lambda: V.select_patches(xm.flatten(1), 144)):.2f} ms")
    txt = hip._text(ids, None)
    img, img_mask = hip._visual(p1, pm, 1)
    X = torch.cat([txt, img], 1)
    L, H = X.shape[1], X.shape[2]
    km = ((1.0 - torch.cat([mask.to(img_mask.dtype), img_mask], 1).float()) * V.MASK_NEG).contiguous()
    X2 = X.reshape(B * L, H).contiguous()
    print(f"  encoder layers {timed(lambda: V._encoder_layers(X2, km, hip.layers, B, L)):.2f} ms")
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(a.steps):
        run()
    torch.cuda.synchronize()
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
