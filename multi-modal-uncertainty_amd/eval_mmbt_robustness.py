#!/usr/bin/env python3
"""Modality-robustness predictions of an MMBT checkpoint -- the reference
eval_mmbt_robustness.py command line and output files (:20-44, :94-110) on the
batched MI355X pass (src/robustness.py: image trunk once per batch, the 43
encoder passes grouped into 3 launches by sequence length).

Writes robustness_<ckpt>_predictions_<phase>.npy  [S, 3 + 2*n_repeats, n_classes]
       robustness_<ckpt>_labels_<phase>.npy       [S]
"""
import argparse
import logging
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from src import dataset  # noqa: E402
from src.mmbt import MultimodalBertClf  # noqa: E402
from src.robustness import robustness_logits  # noqa: E402
from src.training_loop import _load_pretrained_model  # noqa: E402
from src.utils import set_seed, torch_to  # noqa: E402

logger = logging.getLogger(__name__)

FLAGS = [
    ("--save_path", dict(type=str, required=True, help="Path to save the model")),
    ("--phase", dict(type=str, required=True)), ("--batch_size", dict(type=int, required=True)),
    ("--checkpoint_path", dict(type=str, required=True, help="Path to load the model")),
    ("--use_gpu", dict(action="store_true")), ("--device", dict(default=0, type=int)),
    ("--seed", dict(type=int, default=42)), ("--verbose", dict(action="store_true")),
    ("--n_repeats", dict(type=int, default=20, help="Number of times to repeat the random sampling")),
    ("--dataset", dict(type=str, choices=["food101", "hateful-meme-dataset"], default="hateful-meme-dataset")),
    ("--num_image_embeds", dict(type=int, default=3)), ("--drop_img_percent", dict(type=float, default=0.0)),
    ("--dropout", dict(type=float, default=0.1)), ("--datapath", dict(type=str)),
    ("--bert_model", dict(type=str, default="bert-base-uncased", choices=["bert-base-uncased", "bert-large-uncased"])),
    ("--max_seq_len", dict(type=int, default=512)), ("--n_workers", dict(type=int, default=0)),
    ("--hidden", dict(nargs="*", type=int, default=[])), ("--hidden_sz", dict(type=int, default=768)),
    ("--img_embed_pool_type", dict(type=str, default="avg", choices=["max", "avg"])),
    ("--img_hidden_sz", dict(type=int, default=2048)), ("--include_bn", dict(type=int, default=True)),
    ("--synthetic", dict(type=int, default=0, help="N synthetic samples instead of the dataset")),
]


def get_args(parser):
    for flag, kw in FLAGS:
        parser.add_argument(flag, **kw)


def load_data(args):
    if args.synthetic:
        from src.testing import _Vocab
        T = args.max_seq_len - args.num_image_embeds - 1
        ds = dataset.SyntheticFood101(args.synthetic, max_text=T, min_text=T // 2, seed=2)
        ld = torch.utils.data.DataLoader(ds, batch_size=args.batch_size, shuffle=False,
                                         num_workers=args.n_workers, collate_fn=dataset.collate_fn)
        return {"train": ld, "val": ld, "test": ld}, 101, _Vocab()
    tr, va, te, n_classes, vocab = dataset.get_food101(datapath=args.datapath, batch_size=args.batch_size,
                                                       drop_img_percent=args.drop_img_percent,
                                                       max_seq_len=args.max_seq_len,
                                                       num_image_embeds=args.num_image_embeds,
                                                       n_workers=args.n_workers)
    return {"train": tr, "val": va, "test": te}, n_classes, vocab


def main(argv=None):
    parser = argparse.ArgumentParser(description="Eval Models")
    get_args(parser)
    args, remaining = parser.parse_known_args(argv)
    assert remaining == [], remaining
    set_seed(args.seed)
    data, args.n_classes, args.vocab = load_data(args)
    model = MultimodalBertClf(args)
    _load_pretrained_model(model, args.checkpoint_path)
    if not torch.cuda.is_available():
        raise RuntimeError("the MMBT robustness pass runs on MI355X HIP kernels: no GPU visible")
    dev = torch.device("cuda:{}".format(args.device))
    model.to(dev)
    model.eval()
    preds, labels = [], []
    with torch.no_grad():
        for x, y in data[args.phase]:
            x, y = torch_to(x, dev), torch_to(y, dev)
            txt, segment, mask, img = x  # collate order; model(*x) binds mask<-segment, segment<-mask
            preds.append(robustness_logits(model, txt, segment, mask, img, args.n_repeats).float().cpu())
            labels.append(y.cpu())
    preds = torch.cat(preds).numpy()
    labels = torch.cat(labels).numpy()
    name = args.checkpoint_path.split("/")[-1].split(".")[0]
    os.makedirs(args.save_path, exist_ok=True)
    np.save(os.path.join(args.save_path, f"robustness_{name}_predictions_{args.phase}.npy"), preds)
    np.save(os.path.join(args.save_path, f"robustness_{name}_labels_{args.phase}.npy"), labels)
    S, M, C = preds.shape
    print("Gathered predictions of {} samples, {} variants, {} classes".format(S, M, C))
    print("Gathered labels of {} samples".format(len(labels)))


if __name__ == "__main__":
    main()
