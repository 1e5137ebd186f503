"""Food-101 input contract on CPU and the GPU input tail.

Reference behaviour restated in the expectations below (the reference module itself does
not import here: torchvision / pytorch_pretrained_bert are absent):
  * text = ([SEP] + wordpieces[:max_seq_len - num_image_embeds - 1])[1:]  (src/dataset.py:372-376,400-401)
  * segment = 1 on every text token (zeros, sliced, += 1: :377,400-403)
  * label = index of the row's label in `labels` (:386-388)
  * missing image -> a gray 128 256x256 RGB image through the same transform (:393-396)
  * Resize(256) / CenterCrop(224) / ToTensor / Normalize(mean, std) (:488-498)
  * collate_fn pads to the longest text; mask 1 on real tokens (:420-438)
GPU: mmu_image_normalize (uint8 HWC crops -> normalised channels-last image) against the
same normalisation in numpy; DevicePrefetcher yields the CPU path's batches on the device.
"""
import json
import os

import numpy as np
import pytest
import torch


def _vocab():
    from src.dataset import Vocab
    v = Vocab()
    v.add([f"w{i}" for i in range(50)])
    return v


def _write_rows(tmp_path, n_words):
    from PIL import Image
    rng = np.random.default_rng(0)
    Image.fromarray(rng.integers(0, 256, (300, 400, 3), dtype=np.uint8)).save(tmp_path / "a.png")
    Image.fromarray(rng.integers(0, 256, (260, 240, 3), dtype=np.uint8)).save(tmp_path / "b.png")
    rows = [{"text": " ".join(f"w{i % 50}" for i in range(n_words)), "img": "a.png", "label": "pizza"},
            {"text": "w1 w2 zzz w3", "img": None, "label": "ramen"},
            {"text": "w7", "img": "b.png", "label": "pizza"}]
    with open(tmp_path / "train.jsonl", "w") as f:
        for r in rows:
            f.write(json.dumps(r) + "\n")
    return rows


def _dataset(tmp_path, transform, max_seq_len=16, n_img=3):
    from src.dataset import JsonlDataset
    return JsonlDataset(str(tmp_path / "train.jsonl"), str.split, transform, _vocab(), 2, 0.0, max_seq_len, n_img,
                        ["pizza", "ramen"])


def test_crop_u8_then_normalize_equals_transform():
    from PIL import Image
    from src.dataset import MEAN, STD, food101_crop_u8, food101_transform
    img = Image.fromarray(np.random.default_rng(3).integers(0, 256, (333, 250, 3), dtype=np.uint8))
    u8 = food101_crop_u8(img)
    assert u8.dtype == torch.uint8 and tuple(u8.shape) == (224, 224, 3)
    a = (u8.numpy().astype(np.float32) / 255.0 - np.array(MEAN, np.float32)) / np.array(STD, np.float32)
    assert np.array_equal(food101_transform(img).numpy(), a.transpose(2, 0, 1))


def test_jsonl_item_contract(tmp_path):
    from PIL import Image
    from src.dataset import food101_transform
    rows = _write_rows(tmp_path, 40)
    ds = _dataset(tmp_path, food101_transform, max_seq_len=16, n_img=3)
    v = _vocab()
    ids, seg, img, label = ds[0]
    keep = 16 - 3 - 1                                   # wordpieces kept after the leading [SEP]
    assert ids.tolist() == [v.stoi[w] for w in rows[0]["text"].split()[:keep]]
    assert seg.tolist() == [1.0] * keep and label.tolist() == [0]
    ids, seg, img, label = ds[1]                       # unknown word -> [UNK]; missing image -> gray
    assert ids.tolist() == [v.stoi["w1"], v.stoi["w2"], v.stoi["[UNK]"], v.stoi["w3"]] and label.tolist() == [1]
    gray = food101_transform(Image.fromarray(128 * np.ones((256, 256, 3), dtype=np.uint8)))
    assert torch.equal(img, gray)
    assert tuple(ds[2][2].shape) == (3, 224, 224)


def test_collate_pads_and_masks(tmp_path):
    from src.dataset import collate_fn, food101_crop_u8
    _write_rows(tmp_path, 40)
    ds = _dataset(tmp_path, food101_crop_u8)
    (txt, seg, mask, img), tgt = collate_fn([ds[i] for i in range(3)])
    assert txt.shape == (3, 12) and mask.sum(1).tolist() == [12, 4, 1]
    assert torch.equal(seg, mask) and (txt * (1 - mask)).abs().sum() == 0
    assert img.dtype == torch.uint8 and tuple(img.shape) == (3, 224, 224, 3) and tgt.tolist() == [0, 1, 0]


@pytest.mark.gpu
def test_image_normalize_kernel(dev):
    from src import kernels as K
    from src.dataset import MEAN, STD
    for shape in ((4, 224, 224, 3), (1, 5, 7, 3)):       # full 16-B vectors and a ragged tail
        u8 = torch.randint(0, 256, shape, dtype=torch.uint8)
        ref = (u8.numpy().astype(np.float32) / 255.0 - np.array(MEAN, np.float32)) / np.array(STD, np.float32)
        ref = torch.from_numpy(ref).permute(0, 3, 1, 2)
        B, H, W, _ = shape
        for dt, tol in ((torch.float32, 1e-5), (torch.bfloat16, 3e-2)):
            out = torch.empty((B, 3, H, W), dtype=dt, device=dev, memory_format=torch.channels_last)
            K.image_normalize(u8.to(dev), MEAN, STD, out)
            err = (out.float().cpu() - ref).abs().max().item()
            assert err <= tol * max(1.0, ref.abs().max().item()), (shape, dt, err)
    with pytest.raises(Exception):
        K.image_normalize(u8.to(dev).float(), MEAN, STD, out)


@pytest.mark.gpu
def test_device_prefetcher_matches_cpu_path(dev, tmp_path):
    from src.dataset import DevicePrefetcher, collate_fn, food101_crop_u8, food101_transform
    _write_rows(tmp_path, 40)
    mk = lambda tf: torch.utils.data.DataLoader(_dataset(tmp_path, tf), batch_size=2, collate_fn=collate_fn,  # noqa
                                                pin_memory=True)
    got = list(DevicePrefetcher(mk(food101_crop_u8), dev))
    ref = list(mk(food101_transform))
    assert len(got) == len(ref) == 2
    for ((gt, gs, gm, gi), gy), ((rt, rs, rm, ri), ry) in zip(got, ref):
        assert gi.is_cuda and gi.is_contiguous(memory_format=torch.channels_last)
        for a, b in ((gt, rt), (gs, rs), (gm, rm), (gy, ry)):
            assert torch.equal(a.cpu(), b)
        assert (gi.cpu() - ri).abs().max().item() < 1e-5


@pytest.mark.parametrize("tag,drop,msl", [("d0_m12", 0.0, 12), ("d50_m12", 0.5, 12), ("d50_m512", 0.5, 512)])
def test_jsonl_collate_match_reference_golden(tag, drop, msl):
    """Bit-exact A0 pin: tests/golden/a0_contract.npz was written by oracle/gen_golden.py
    --what a0 running the reference's OWN JsonlDataset / get_labels_and_frequencies /
    collate_fn / numpy_seed (src/dataset.py:348-438, src/utils.py:167-181) over the committed
    tests/golden/a0/train.jsonl (empty, 1-token, truncated and 600-word texts, OOV words,
    missing and dropped images).  Same tokenizer (str.split), vocab and PIL transform here."""
    import types
    from oracle.gen_golden import a0_transform, a0_vocab_stoi
    from src.dataset import JsonlDataset, collate_fn, get_labels_and_frequencies
    here = os.path.dirname(os.path.abspath(__file__))
    g = np.load(os.path.join(here, "golden", "a0_contract.npz"))
    path = os.path.join(here, "golden", "a0", "train.jsonl")
    labels, freqs = get_labels_and_frequencies(path)
    assert labels == g["labels"].tolist() and [freqs[k] for k in labels] == g["label_counts"].tolist()
    vocab = types.SimpleNamespace(stoi=a0_vocab_stoi())
    ds = JsonlDataset(path, str.split, a0_transform, vocab, len(labels), drop, msl, 3, labels)
    assert [r["img"] is None for r in ds.data] == g[f"{tag}_img_dropped"].tolist()
    items = [ds[i] for i in range(len(ds))]
    assert [len(it[0]) for it in items] == g[f"{tag}_item_lens"].tolist()
    for lo, hi in ((0, 4), (4, 10)):
        (txt, seg, mask, img), tgt = collate_fn(items[lo:hi])
        for k, v in (("text", txt), ("segment", seg), ("mask", mask), ("img", img), ("tgt", tgt)):
            want = torch.from_numpy(g[f"{tag}_b{lo}_{k}"])
            assert str(v.dtype) == str(g[f"{tag}_b{lo}_{k}_dtype"]), (tag, lo, k, v.dtype)
            assert torch.equal(v, want), (tag, lo, k)
