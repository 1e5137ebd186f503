#!/usr/bin/env python3
"""Robustness / uncertainty evaluation entry point (reference eval_robustness.py CLI, :20-34).

MMBT mode (the build's uncertainty pass, BASELINE config 3):
  --mmbt --checkpoint_paths ck1.pt ... ckK.pt [--mc_samples 30] --phase val
runs the K-member deep ensemble x T-pass MC-dropout as one batched encoder launch
per op (src/uncertainty.py) and writes
  <save_path>/uncertainty_<phase>_logits.npy   [S, K, T, n_classes]
  <save_path>/uncertainty_<phase>_labels.npy   [S]
  <save_path>/uncertainty_<phase>_metrics.json {nll, ece, acc, n, K, T}
Without --mmbt: the reference's FashionMNIST MIMO robustness pass (eval_robustness.py:42-121,
BASELINE config 1's model family): each of the 4 quarter-crop views zeroed in turn (the
weight-sharing model sees the other 3), predictions [4, S, heads, 10] and labels written as
<checkpoint>_predictions_robustness.npy / <checkpoint>_labels.npy.  --data_dir / --sample_size
/ --synthetic_images as in train_fashionmnist.py (without image files the run fails unless
--synthetic_images is given).
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import numpy as np  # noqa: E402
import torch  # noqa: E402

FLAGS = [
    ("--checkpoint_path", dict(type=str, default=None, help="Path to load the model")),
    ("--model_type", dict(type=str, default="Vanilla",
                          choices=["Vanilla", "MIMO-shuffle-instance", "MIMO-shuffle-view", "MultiHead",
                                   "MIMO-shuffle-all", "single-model-weight-sharing"])),
    ("--use_gpu", dict(action="store_true")), ("--device", dict(default=0, type=int)),
    ("--save_path", dict(type=str, required=True, help="Path to save the model")),
    ("--seed", dict(type=int, default=42)), ("--verbose", dict(action="store_true")),
    ("--batch_size", dict(type=int, default=64)), ("--transformer", dict(action="store_true")),
    ("--multimodal_num_attention_heads", dict(type=int, default=3)),
    ("--multimodal_num_hidden_layers", dict(type=int, default=3)), ("--dropout", dict(type=float, default=0)),
    # MMBT uncertainty mode
    ("--mmbt", dict(action="store_true")), ("--checkpoint_paths", dict(nargs="*", default=[])),
    ("--mc_samples", dict(type=int, default=1)), ("--n_bins", dict(type=int, default=15)),
    ("--phase", dict(type=str, default="val")), ("--synthetic", dict(type=int, default=0)),
    ("--datapath", dict(type=str, default=None)), ("--max_seq_len", dict(type=int, default=512)),
    ("--num_image_embeds", dict(type=int, default=3)), ("--n_workers", dict(type=int, default=0)),
    ("--bert_model", dict(type=str, default="bert-base-uncased")),
    ("--gin_file", dict(nargs="*", default=[])), ("--gin_param", dict(nargs="*", default=[])),
    ("--data_dir", dict(type=str, default=None)), ("--sample_size", dict(type=int, default=None)),
    ("--synthetic_images", dict(action="store_true")),
]


def get_args(parser):
    for flag, kw in FLAGS:
        parser.add_argument(flag, **kw)


def run_mmbt(args):
    from src import gin
    from src.mmbt import MultimodalBertClf
    from src.testing import make_args
    from src.training_loop import _load_pretrained_model
    from src.uncertainty import EnsembleMMBT, UncertaintyMeter
    from src.utils import set_seed
    from eval_mmbt_robustness import load_data
    set_seed(args.seed)
    args.drop_img_percent = 0.0
    data, n_classes, vocab = load_data(args)
    paths = args.checkpoint_paths or ([args.checkpoint_path] if args.checkpoint_path else [])
    if not torch.cuda.is_available():
        raise RuntimeError("the MMBT uncertainty pass runs on MI355X HIP kernels: no GPU visible")
    dev = torch.device("cuda:{}".format(args.device))
    members = []
    for i, p in enumerate(paths or [None]):
        margs = make_args(n_classes=n_classes, vocab=vocab, num_image_embeds=args.num_image_embeds,
                          bert_model=args.bert_model)
        torch.manual_seed(args.seed + i)
        m = MultimodalBertClf(margs)
        if p:
            _load_pretrained_model(m, p)
        members.append(m.to(dev))
    ens = EnsembleMMBT(members)
    meter = UncertaintyMeter(args.n_bins)
    all_logits, labels = [], []
    with torch.no_grad():
        for x, y in data[args.phase]:
            txt, segment, mask, img = (t.to(dev) for t in x)
            lo = ens.logits(txt, segment, mask, img, mc_samples=args.mc_samples)   # [K, T, B, C]
            flat = lo.permute(2, 0, 1, 3).reshape(lo.shape[2], -1, lo.shape[3])  # [B, K*T, C]
            meter.update(flat, y.to(dev))
            all_logits.append(lo.permute(2, 0, 1, 3).cpu())
            labels.append(y)
    res = dict(meter.result(), K=len(members), T=args.mc_samples)
    os.makedirs(args.save_path, exist_ok=True)
    np.save(os.path.join(args.save_path, f"uncertainty_{args.phase}_logits.npy"), torch.cat(all_logits).numpy())
    np.save(os.path.join(args.save_path, f"uncertainty_{args.phase}_labels.npy"), torch.cat(labels).numpy())
    with open(os.path.join(args.save_path, f"uncertainty_{args.phase}_metrics.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))
    return res


def run_fmnist(args):
    """eval_robustness.py:42-121: view i zeroed (or dropped for the weight-sharing model) for
    i = 0..3 over the test loader, in the reference's loop order."""
    from src import dataset
    from src.training_loop import _load_pretrained_model
    from train_fashionmnist import build_model
    if args.checkpoint_path is None:
        raise ValueError("--checkpoint_path is required without --mmbt")
    model = build_model(args)
    _, valid, _ = dataset.get_fmnist(datapath=args.data_dir, batch_size=args.batch_size, download=True,
                                     shuffle=True, sample_size=args.sample_size, seed=args.seed,
                                     synthetic_images=args.synthetic_images)
    if getattr(valid.dataset, "synthetic", False):
        print("WARNING: FashionMNIST images are SYNTHETIC (seeded noise, real labels)")
    print("Loading Checkpoint from {}".format(args.checkpoint_path))
    _load_pretrained_model(model, args.checkpoint_path)
    dev = torch.device("cuda:{}".format(args.device)) if args.use_gpu and torch.cuda.is_available() \
        else torch.device("cpu")
    model.to(dev).eval()
    outputs, labels, m = [], [], 4
    with torch.no_grad():
        for i in range(m):
            y_hat = []
            for x, y in valid:
                if args.model_type != "single-model-weight-sharing":
                    x, y = dataset.data_forming_func(x, y, "eval", model_type=args.model_type)
                    x_ = x.to(dev).clone()
                    x_[:, i] = 0  # view i zeroed, the others kept
                    y_ = model(x_)
                else:
                    b, mm, c, h, w = x.shape
                    keep = [j for j in range(mm) if j != i]
                    x_, y = dataset.data_forming_func(x[:, keep].contiguous(), y, "eval", model_type=args.model_type)
                    y_ = model(x_.to(dev)).view(b, mm - 1, -1)
                y_hat.append(y_.float().cpu().numpy())
                if i == 0:
                    labels.append(y.cpu().numpy())
            outputs.append(np.concatenate(y_hat, axis=0))
    outputs = np.stack(outputs, axis=0)
    M_, S, M, C = outputs.shape
    print("Gathered predictions of {} samples, {} views, {} dups, {} classes".format(S, M_, M, C))
    labels = np.concatenate(labels, axis=0)
    os.makedirs(args.save_path, exist_ok=True)
    name = args.checkpoint_path.split("/")[-1].split(".")[0]
    np.save(os.path.join(args.save_path, f"{name}_predictions_robustness.npy"), outputs)
    np.save(os.path.join(args.save_path, f"{name}_labels.npy"), labels)
    return outputs, labels


def main(argv=None):
    parser = argparse.ArgumentParser(description="Train Models")
    get_args(parser)
    args, remaining = parser.parse_known_args(argv)
    assert remaining == [], remaining
    from src import gin
    gin.load(args, args.gin_file, args.gin_param)
    return run_mmbt(args) if args.mmbt else run_fmnist(args)


if __name__ == "__main__":
    main()
