#!/usr/bin/env python3
"""FashionMNIST MIMO training entry point -- BASELINE config 1 ("single-modality classifier
on CPU, plumbing").  Same command line as the reference train_fashionmnist.py (flags
:22-42, models :60-81, optimizers :89-124, resume :129-145, callbacks :147-166,
Model_.train_loop :173-191).

Differences from the reference, each a fix of a crash against its own framework or an
offline necessity:
  * ``acc`` takes the 4th ``dummy_dim`` argument Model_ passes (src/framework.py:112 calls
    metrics with 4 arguments; the reference's 3-argument acc raises TypeError);
  * ``scheduler_metric`` is passed to train_loop (the reference sets args.scheduler_metric
    but never passes it, and train_loop reads kwargs["scheduler_metric"]);
  * images: only the label files ship (reference fashionMNIST/FashionMNIST/*-labels-*);
    without image files the loader raises unless --synthetic_images is given, which serves
    seeded synthetic 28x28 images with the REAL labels (src/dataset.FashionMNISTQuarters;
    recorded as ``synthetic_images`` in <save_path>/run_meta.json).  --sample_size caps the
    set for smoke runs;
  * gin front end: --gin_file / --gin_param bindings (configs/training.gin's ``train.*``
    scope) map onto the flags (src/gin.py).
The ResNet runs on the CPU by default (the config is CPU plumbing); ``--transformer``
selects MIMOTransfomer, whose fusion blocks are the HIP kernels (needs --use_gpu).
"""
import argparse
import json
import logging
import os
import sys
from functools import partial

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import pandas as pd  # noqa: E402
import torch  # noqa: E402

from src import dataset, gin  # noqa: E402
from src.framework import Model_  # noqa: E402
from src.model import MIMOResNet, MIMOTransfomer, model_configure  # noqa: E402
from src.training_loop import _construct_default_callbacks  # noqa: E402

logger = logging.getLogger(__name__)

MODEL_TYPES = ["Vanilla", "MIMO-shuffle-instance", "MIMO-shuffle-view", "MultiHead", "MIMO-shuffle-all",
               "single-model-weight-sharing"]


def get_args(parser):
    parser.add_argument("--batch_size", type=int, default=32)
    parser.add_argument("--lr", type=float, default=0.1)
    parser.add_argument("--wd", type=int, default=0.001)
    parser.add_argument("--momentum", type=int, default=0.9)
    parser.add_argument("--n_epochs", type=int, default=100)
    parser.add_argument("--model_type", type=str, default="Vanilla", choices=MODEL_TYPES)
    parser.add_argument("--use_gpu", action="store_true")
    parser.add_argument("--device", default=0, type=int)
    parser.add_argument("--save_path", type=str, required=True, help="Path to save the model")
    parser.add_argument("--seed", type=int, default=42)
    parser.add_argument("--verbose", action="store_true")
    parser.add_argument("--patience", type=int, default=10)
    parser.add_argument("--resume", action="store_true")
    parser.add_argument("--multimodal_num_attention_heads", type=int, default=3)
    parser.add_argument("--multimodal_num_hidden_layers", type=int, default=3)
    parser.add_argument("--transformer", action="store_true")
    parser.add_argument("--warmup", type=float, default=0.1)
    parser.add_argument("--dropout", type=float, default=0)
    # additions
    parser.add_argument("--data_dir", type=str, default=None, help="FashionMNIST root (default $DATA_DIR)")
    parser.add_argument("--sample_size", type=int, default=None)
    parser.add_argument("--synthetic_images", action="store_true",
                        help="serve seeded noise images when the FashionMNIST image files are missing")
    parser.add_argument("--gin_file", nargs="*", default=[])
    parser.add_argument("--gin_param", nargs="*", default=[])


def acc(y_pred, y_true, eval, dummy_dim=None):
    """Accuracy in % over every head (train) or of the head mean (eval)
    (reference train_fashionmnist.py:44-55, plus Model_'s 4th argument)."""
    if not eval:
        y_pred = y_pred.reshape(-1, y_pred.shape[2])
        y_true = y_true.reshape(-1)
    else:
        y_pred = y_pred.mean(1)
    _, y_pred = y_pred.max(1)
    return (y_pred == y_true).float().mean() * 100


def build_model(args):
    emb_dim, out_dim = model_configure[args.model_type]
    if args.transformer:
        assert args.model_type in ("MultiHead", "MIMO-shuffle-instance")
        return MIMOTransfomer(out_dim=out_dim, num_classes=10, image_dim=14 * 14, hidden_size=768,
                              multimodal_num_attention_heads=args.multimodal_num_attention_heads,
                              multimodal_num_hidden_layers=args.multimodal_num_hidden_layers, drop=args.dropout)
    return MIMOResNet(num_channels=1, emb_dim=emb_dim, out_dim=out_dim, num_classes=10)


def build_optimizer(args, model, n_train_batches):
    if args.transformer:
        from src.optim import BertAdam
        no_decay = ["bias", "LayerNorm.bias", "LayerNorm.weight"]
        named = list(model.named_parameters())
        groups = [
            {"params": [p for n, p in named if not any(nd in n for nd in no_decay)], "weight_decay": 0.01},
            {"params": [p for n, p in named if any(nd in n for nd in no_decay)], "weight_decay": 0.0},
        ]
        optimizer = BertAdam(groups, lr=args.lr, warmup=args.warmup, t_total=n_train_batches * args.n_epochs)
        scheduler = torch.optim.lr_scheduler.ReduceLROnPlateau(optimizer, "max", patience=10, factor=0.5)
        args.scheduler_metric = "val_acc"
    else:
        optimizer = torch.optim.SGD(model.parameters(), lr=args.lr, weight_decay=args.wd, momentum=args.momentum)
        scheduler = torch.optim.lr_scheduler.ReduceLROnPlateau(
            optimizer, mode="min", factor=0.1, patience=10, threshold=0.0001, threshold_mode="rel", cooldown=0,
            min_lr=0, eps=1e-08)
        args.scheduler_metric = "val_loss"
    return optimizer, scheduler


def main(argv=None):
    parser = argparse.ArgumentParser(description="Train Models")
    get_args(parser)
    args, remaining = parser.parse_known_args(argv)
    assert remaining == [], remaining
    unused = gin.load(args, args.gin_file, args.gin_param)
    if unused:
        logger.warning("gin bindings not mapped to train_fashionmnist.py flags: %s", sorted(unused))
    model = build_model(args)
    train, valid, _ = dataset.get_fmnist(datapath=args.data_dir, batch_size=args.batch_size, download=True,
                                         shuffle=True, sample_size=args.sample_size, seed=args.seed,
                                         synthetic_images=args.synthetic_images)
    optimizer, scheduler = build_optimizer(args, model, len(train))
    os.makedirs(args.save_path, exist_ok=True)
    synthetic = bool(getattr(train.dataset, "synthetic", False))
    if synthetic:
        print("WARNING: FashionMNIST images are SYNTHETIC (seeded noise, real labels)")
    with open(os.path.join(args.save_path, "run_meta.json"), "w") as f:
        json.dump({"synthetic_images": synthetic, "model_type": args.model_type, "seed": args.seed}, f)
    history_csv_path = os.path.join(args.save_path, "history.csv")
    if args.resume:
        ck = torch.load(os.path.join(args.save_path, "model_last_epoch.pt"), map_location="cpu", weights_only=True)
        model.load_state_dict(ck["model"])
        H = pd.read_csv(history_csv_path)
        H = {c: list(H[c].values) for c in H.columns if c != "Unnamed: 0"}
        epoch_start = len(H["epoch"]) + 1
    else:
        H = {}
        if os.path.exists(history_csv_path):
            logger.info("Removing %s", history_csv_path)
            os.remove(history_csv_path)
        epoch_start = 1
    callbacks = _construct_default_callbacks(model, optimizer, H, args.save_path, checkpoint_monitor="val_acc")
    for c in callbacks:
        c.set_save_path(args.save_path)
        c.set_model(model, ignore=False)
        c.set_optimizer(optimizer)
    m = Model_(model=model, optimizer=optimizer, scheduler=scheduler,
               data_forming_func=partial(dataset.data_forming_func, model_type=args.model_type),
               metrics=[acc], verbose=args.verbose)
    for c in callbacks:
        c.set_model_pytoune(m)
    if args.use_gpu and torch.cuda.is_available():
        m.to(torch.device("cuda:{}".format(args.device)))
    elif args.transformer:
        raise RuntimeError("--transformer: the fusion blocks run on the MI355X HIP kernels (--use_gpu, GPU visible)")
    m.train_loop(train, valid_generator=valid, test_generator=valid, steps_per_epoch=len(train),
                 validation_steps=len(valid), test_steps=len(valid), epochs=args.n_epochs - 1, callbacks=callbacks,
                 patience=args.patience, epoch_start=epoch_start, scheduler_step_on="epoch", auc=False,
                 scheduler_metric=args.scheduler_metric)
    return H


if __name__ == "__main__":
    main()
