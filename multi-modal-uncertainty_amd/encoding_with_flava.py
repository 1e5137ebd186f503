#!/usr/bin/env python3
"""Precompute FLAVA image / text embeddings -- the reference data/encoding_with_flava.py
(:11-41 encoding loop, :43-74 Hateful Memes / Food-101 drivers) on the MI355X HIP encoders
(src/flava_encoders.py), writing the per-sample files the FLAVA fusion transformer's dataset
reads (src/dataset.py FlavaEncodedDataset):

  <data_path>/flava_embeds_<max_length>/<name>.img   [197, 768]  image_embeddings
  <data_path>/flava_embeds_<max_length>/<name>.text  [T, 768]    text_embeddings
  <data_path>/flava_embeds_<max_length>/<phase>_unseen_error_cases.txt

Differences, all offline necessities or speed:
  * weights: the reference loads facebook/flava-full (network).  Here ``--weights`` takes a
    local FlavaModel state_dict (safetensors / a weights_only torch file); without it the
    model is transformers' FlavaModel(FlavaConfig()) with seeded random weights;
  * processor: FlavaImageProcessor (PIL backend) + a BertTokenizer on a local vocab
    ($BERT_VOCAB, src/dataset.py) instead of FlavaProcessor.from_pretrained;
  * samples are encoded ``--batch_size`` at a time (texts padded to the batch's longest; each
    sample's embeddings are cut to its own length, so they equal the one-at-a-time result);
  * tensors are saved on the CPU (the reference saves CUDA tensors).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

from src.flava_encoders import FlavaEncodersHIP  # noqa: E402


def build_model(weights=None, seed=0):
    from transformers import FlavaConfig, FlavaModel
    torch.manual_seed(seed)
    model = FlavaModel(FlavaConfig()).eval()
    if weights:
        if weights.endswith(".safetensors"):
            from safetensors.torch import load_file
            sd = load_file(weights)
        else:
            sd = torch.load(weights, map_location="cpu", weights_only=True)
        model.load_state_dict(sd, strict=False)
    return model


def build_processor(max_length):
    from transformers import FlavaImageProcessorPil
    from src.dataset import bert_tokenizer
    image_proc = FlavaImageProcessorPil()
    tok = bert_tokenizer("bert-base-uncased")

    def processor(texts, images):
        px = image_proc(images=images, return_tensors="pt")["pixel_values"]
        t = tok(texts, return_tensors="pt", padding=True, max_length=max_length, truncation=True)
        return px, t["input_ids"], t["attention_mask"], t.get("token_type_ids")
    return processor


def encoding_with_flava(data_path, meta_data, image_path_renaming, encoders, processor, max_length=512,
                        phases=("train", "dev", "test"), batch_size=16):
    from PIL import Image
    dev = encoders.device
    out_root = f"{data_path}/flava_embeds_{max_length}"
    for phase in phases:
        error_cases = []
        rows = list(meta_data[phase].index)
        for s in range(0, len(rows), batch_size):
            idx = rows[s:s + batch_size]
            names, images, texts = [], [], []
            for ind in idx:
                image_path, text = meta_data[phase].loc[ind][["img", "text"]]
                names.append(image_path_renaming(image_path))
                images.append(Image.open(os.path.join(data_path, image_path)).convert("RGB"))
                texts.append(text)
            px, ids, am, tt = processor(texts, images)
            img, txt = encoders(px.to(dev), ids.to(dev), am.to(dev), None if tt is None else tt.to(dev))
            lens = am.sum(1).tolist()
            for k, name in enumerate(names):
                path = f"{out_root}/{'/'.join(name.split('/')[:-1])}"
                os.makedirs(path, exist_ok=True)
                torch.save(img[k].cpu().clone(), f"{out_root}/{name}.img")
                torch.save(txt[k, :int(lens[k])].cpu().clone(), f"{out_root}/{name}.text")
        print(phase, len(error_cases))
        with open(f"{out_root}/{phase}_unseen_error_cases.txt", "w") as f:
            for ind in error_cases:
                f.write(f"{ind}\n")


def _meta(data_path, files):
    import pandas as pd
    return {ph: pd.read_json(path_or_buf=os.path.join(data_path, fn), lines=True) for ph, fn in files.items()}


def generation_for_hatefulmeme(data_path, encoders, processor, max_length=512, batch_size=16):
    meta = _meta(data_path, {"train": "train.jsonl", "dev": "dev_unseen.jsonl", "test": "test_unseen.jsonl"})
    encoding_with_flava(data_path, meta, lambda p: p.split("/")[-1].split(".")[0], encoders, processor, max_length,
                        batch_size=batch_size)


def generation_for_food101(data_path, encoders, processor, max_length, batch_size=16):
    meta = _meta(data_path, {"train": "train.jsonl", "dev": "dev.jsonl", "test": "test.jsonl"})
    encoding_with_flava(data_path, meta, lambda p: p.split(".")[0], encoders, processor, max_length,
                        batch_size=batch_size)


def main(argv=None):
    ap = argparse.ArgumentParser(description="FLAVA embeddings on the MI355X HIP encoders")
    ap.add_argument("max_length", type=int, nargs="?", default=512)
    ap.add_argument("--dataset", choices=["food101", "hateful-meme-dataset"], default="food101")
    ap.add_argument("--data_path", required=True)
    ap.add_argument("--weights", default=None)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--batch_size", type=int, default=16)
    a = ap.parse_args(argv)
    if not torch.cuda.is_available():
        raise RuntimeError("the FLAVA encoders run on the MI355X HIP kernels: no GPU visible")
    encoders = FlavaEncodersHIP(build_model(a.weights, a.seed), "cuda")
    processor = build_processor(a.max_length)
    if a.dataset == "food101":
        generation_for_food101(a.data_path, encoders, processor, a.max_length, a.batch_size)
    else:
        generation_for_hatefulmeme(a.data_path, encoders, processor, a.max_length, a.batch_size)


if __name__ == "__main__":
    main()
