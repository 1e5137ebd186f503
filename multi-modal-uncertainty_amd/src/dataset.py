"""MMBT input contract: Food-101 jsonl dataset, vocab, collate.

Same public names / signatures as the reference src/dataset.py MMBT part
(JsonlDataset :348-405, get_labels_and_frequencies :408-417, collate_fn :420-438,
Vocab/get_vocab :440-472, get_food101 :474-545).  Differences forced by the image:
  * torchvision is absent: Resize(256) -> CenterCrop(224) -> ToTensor -> Normalize is
    restated on PIL + numpy (`food101_transform`);
  * BertTokenizer.from_pretrained needs the network: the vocab is read from a local
    file (`<DATA_DIR>/<bert_model>-vocab.txt` or $BERT_VOCAB) via transformers' BertTokenizer.
``SyntheticFood101`` produces batches of the same contract for benchmarks and tests.

GPU input tail: with ``gpu_normalize=True`` the workers stop after
decode / resize / center-crop (``food101_crop_u8``: uint8 HWC, 150 KB per image instead of
602 KB of f32), and ``DevicePrefetcher`` copies the next pinned batch to the GPU on a side
stream and runs ToTensor + Normalize there (mmu_image_normalize), one batch ahead of the
training step.
"""
import json
import os
from collections import Counter

import numpy as np
import torch
from torch.utils.data import Dataset

from .utils import numpy_seed

MEAN = (0.46777044, 0.44531429, 0.40661017)
STD = (0.12221994, 0.12145835, 0.14380469)


def _resize_crop(img, size, crop):
    from PIL import Image
    w, h = img.size
    if w <= h:
        nw, nh = size, int(size * h / w)
    else:
        nw, nh = int(size * w / h), size
    img = img.resize((nw, nh), Image.BILINEAR)
    left, top = int(round((nw - crop) / 2.0)), int(round((nh - crop) / 2.0))
    return np.asarray(img.crop((left, top, left + crop, top + crop)), dtype=np.uint8)


def food101_transform(img, size=256, crop=224):
    """Resize shorter side to `size` (bilinear), center-crop `crop`, to [0,1] CHW, normalise
    (Resize(256) / CenterCrop(224) / ToTensor / Normalize, reference src/dataset.py:488-498)."""
    a = _resize_crop(img, size, crop).astype(np.float32) / 255.0
    a = (a - np.array(MEAN, dtype=np.float32)) / np.array(STD, dtype=np.float32)
    return torch.from_numpy(a.transpose(2, 0, 1).copy())


def food101_crop_u8(img, size=256, crop=224):
    """The worker half of food101_transform: resize + center-crop only -> uint8 [crop, crop, 3]
    (HWC); ToTensor + Normalize run on the GPU (DevicePrefetcher / mmu_image_normalize)."""
    return torch.from_numpy(_resize_crop(img, size, crop).copy())


class DevicePrefetcher:
    """Wraps a DataLoader of ``collate_fn`` batches: copies batch i+1 to ``device`` on a side
    stream (non-blocking from pinned memory) while batch i trains, and turns uint8 HWC crops
    into the normalised channels-last image there (mmu_image_normalize; f32 images, e.g.
    from food101_transform or SyntheticFood101, are only copied).  Yields the same
    ((text, segment, mask, img), tgt) tuples, already on the device."""

    def __init__(self, loader, device, mean=MEAN, std=STD, dtype=torch.float32):
        self.loader, self.device, self.mean, self.std, self.dtype = loader, torch.device(device), mean, std, dtype
        self.dataset = getattr(loader, "dataset", None)
        self.sampler = getattr(loader, "sampler", None)  # Model_.train_loop sets a DistributedSampler's epoch

    def __len__(self):
        return len(self.loader)

    def _stage(self, batch, stream):
        from . import kernels as K
        (txt, seg, mask, img), tgt = batch
        with torch.cuda.stream(stream):
            txt, seg, mask, tgt = (t.to(self.device, non_blocking=True) for t in (txt, seg, mask, tgt))
            if img.dtype == torch.uint8:
                raw = img.to(self.device, non_blocking=True)
                B, H, W, _ = raw.shape
                img = torch.empty((B, 3, H, W), dtype=self.dtype, device=self.device,
                                  memory_format=torch.channels_last)
                K.image_normalize(raw, self.mean, self.std, img)
                raw.record_stream(stream)
            else:
                img = img.to(self.device, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(stream)
        return ((txt, seg, mask, img), tgt), ev

    def __iter__(self):
        stream = torch.cuda.Stream(device=self.device)
        it = iter(self.loader)
        nxt = None
        try:
            nxt = self._stage(next(it), stream)
        except StopIteration:
            return
        while nxt is not None:
            batch, ev = nxt
            try:
                nxt = self._stage(next(it), stream)
            except StopIteration:
                nxt = None
            cur = torch.cuda.current_stream(self.device)
            cur.wait_event(ev)
            for t in (*batch[0], batch[1]):
                t.record_stream(cur)
            yield batch


class Vocab(object):
    def __init__(self, emptyInit=False):
        if emptyInit:
            self.stoi, self.itos, self.vocab_sz = {}, [], 0
        else:
            self.itos = ["[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]"]
            self.stoi = {w: i for i, w in enumerate(self.itos)}
            self.vocab_sz = len(self.itos)

    def add(self, words):
        for w in words:
            if w not in self.stoi:
                self.stoi[w] = len(self.itos)
                self.itos.append(w)
        self.vocab_sz = len(self.itos)


def _vocab_file(bert_model):
    cands = [os.environ.get("BERT_VOCAB", ""),
             os.path.join(os.environ.get("DATA_DIR", ""), f"{bert_model}-vocab.txt"),
             os.path.join(os.environ.get("DATA_DIR", ""), bert_model, "vocab.txt")]
    for c in cands:
        if c and os.path.exists(c):
            return c
    raise FileNotFoundError(f"no local vocab for {bert_model}: set $BERT_VOCAB or put {bert_model}-vocab.txt in "
                            f"$DATA_DIR (BertTokenizer.from_pretrained needs the network)")


def bert_tokenizer(bert_model):
    from transformers import BertTokenizer
    return BertTokenizer(vocab_file=_vocab_file(bert_model), do_lower_case=True)


def get_vocab(bert_model):
    tok = bert_tokenizer(bert_model)
    vocab = Vocab()
    vocab.stoi = dict(tok.get_vocab())  # (transformers 5 has no .ids_to_tokens: invert the map)
    vocab.itos = {i: w for w, i in vocab.stoi.items()}
    vocab.vocab_sz = len(vocab.itos)
    return vocab


class JsonlDataset(Dataset):
    """One Food-101 row -> (text ids, segment, image, label); text = wordpieces truncated to
    max_seq_len - num_image_embeds - 1 after a leading [SEP] that is then dropped
    (the first [SEP] belongs to the image tokens)."""

    def __init__(self, data_path, tokenizer, transforms, vocab, n_classes, drop_img_percent, max_seq_len,
                 num_image_embeds, labels):
        with open(data_path) as f:
            self.data = [json.loads(line) for line in f]
        self.data_dir = os.path.dirname(data_path)
        self.tokenizer, self.vocab, self.n_classes, self.labels = tokenizer, vocab, n_classes, labels
        self.text_start_token = ["[SEP]"]
        with numpy_seed(0):
            for row in self.data:
                if np.random.random() < drop_img_percent:
                    row["img"] = None
        self.max_seq_len = max_seq_len - num_image_embeds
        self.transforms = transforms

    def __len__(self):
        return len(self.data)

    def __getitem__(self, index):
        row = self.data[index]
        words = self.text_start_token + self.tokenizer(row["text"])[:(self.max_seq_len - 1)]
        unk = self.vocab.stoi["[UNK]"]
        ids = torch.LongTensor([self.vocab.stoi.get(w, unk) for w in words])[1:]
        segment = torch.ones(len(ids))
        label = torch.LongTensor([self.labels.index(row["label"])])
        from PIL import Image
        if row["img"]:
            image = Image.open(os.path.join(self.data_dir, row["img"])).convert("RGB")
        else:
            image = Image.fromarray(128 * np.ones((256, 256, 3), dtype=np.uint8))
        return ids, segment, self.transforms(image), label


def get_labels_and_frequencies(path):
    with open(path) as f:
        labels = [json.loads(line)["label"] for line in f]
    freqs = Counter()
    if labels and isinstance(labels[0], list):
        for row in labels:
            freqs.update(row)
    else:
        freqs.update(labels)
    return list(freqs.keys()), freqs


def collate_fn(batch):
    """Pad to the longest text in the batch -> ((text, segment, mask, img), tgt)."""
    lens = [len(r[0]) for r in batch]
    B, T = len(batch), max(lens)
    text = torch.zeros(B, T, dtype=torch.long)
    segment = torch.zeros(B, T, dtype=torch.long)
    mask = torch.zeros(B, T, dtype=torch.long)
    for i, (r, n) in enumerate(zip(batch, lens)):
        text[i, :n] = r[0]
        segment[i, :n] = r[1]
        mask[i, :n] = 1
    img = torch.stack([r[2] for r in batch])
    tgt = torch.cat([r[3] for r in batch]).long()
    return (text, segment, mask, img), tgt


def get_food101(bert_model="bert-base-uncased", datapath=None, drop_img_percent=0.0, max_seq_len=512,
                num_image_embeds=3, batch_size=128, n_workers=20, gpu_normalize=False, device=None, sampler=None):
    """``sampler``: optional factory ds -> Sampler for the TRAIN split (data parallel:
    a DistributedSampler, so every rank draws a disjoint shard; dev/test stay whole)."""
    datapath = datapath or os.environ["DATA_DIR"]
    tokenizer = bert_tokenizer(bert_model).tokenize
    labels, _ = get_labels_and_frequencies(os.path.join(datapath, "train.jsonl"))
    vocab = get_vocab(bert_model)
    n_classes = len(labels)

    def make(split):
        tf = food101_crop_u8 if gpu_normalize else food101_transform
        return JsonlDataset(os.path.join(datapath, f"{split}.jsonl"), tokenizer, tf, vocab, n_classes,
                            drop_img_percent, max_seq_len, num_image_embeds, labels)

    def loader(ds, shuffle, smp=None):
        dl = torch.utils.data.DataLoader(ds, batch_size=batch_size, shuffle=shuffle and smp is None, sampler=smp,
                                         num_workers=n_workers, collate_fn=collate_fn,
                                         pin_memory=torch.cuda.is_available())
        return DevicePrefetcher(dl, device) if gpu_normalize else dl

    train_ds = make("train")
    train = loader(train_ds, True, sampler(train_ds) if sampler is not None else None)
    return train, loader(make("dev"), False), loader(make("test"), False), n_classes, vocab


class SyntheticFood101(Dataset):
    """Seeded stand-in with the JsonlDataset item contract (texts of random length up to
    max_text, image already normalised) -- no dataset is available offline."""

    def __init__(self, n, max_text=508, n_classes=101, vocab_size=30522, min_text=None, seed=0):
        self.n, self.max_text, self.n_classes, self.vocab_size = n, max_text, n_classes, vocab_size
        self.min_text = max_text if min_text is None else min_text
        self.seed = seed

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        g = torch.Generator().manual_seed(self.seed * 1000003 + i)
        T = int(torch.randint(self.min_text, self.max_text + 1, (1,), generator=g))
        ids = torch.randint(1000, self.vocab_size, (T,), generator=g)
        img = torch.randn(3, 224, 224, generator=g)
        y = torch.randint(0, self.n_classes, (1,), generator=g)
        return ids, torch.ones(T), img, y


# ------------------------------------------------------------------------------ FLAVA
# Precomputed FLAVA embeddings of Hateful Memes (src/dataset.py:177-226, 287-336 of the
# reference; BASELINE config 5).  The embeddings are written by data/encoding_with_flava.py
# (needs the remote facebook/flava-full weights: not reproducible offline), one
# `<name>.img` [L_img, 768] and `<name>.text` [L_txt, 768] tensor file per meme.
def data_forming_func_transformer(x, y, phase, model_type):
    """Labels per member / MIMO instance shuffles (reference src/dataset.py:30-54)."""
    img, txt = x
    if model_type == "Vanilla" and phase == "train":
        y = y.unsqueeze(1).repeat(1, 1)
    elif model_type == "MultiHead" and phase == "train":
        y = y.unsqueeze(1).repeat(1, 2)
    elif model_type == "MIMO-shuffle-instance" and phase == "train":
        idx = torch.randperm(img.size(0))
        img = img[idx]
        y_img = y[idx]
        idx = torch.randperm(img.size(0))
        txt = txt[idx]
        y_txt = y[idx]
        y = torch.stack([y_img, y_txt], dim=1)
    return (img, txt), y


class BaseDataset(Dataset):
    """`<predix_dir>/<phase>.jsonl` metadata minus the listed encoder failures
    (reference src/dataset.py:177-193)."""

    def __init__(self, predix_dir, phase, label_dict=None, error_cases_remover=True, **kwargs):
        import pandas as pd
        self.meta_data = pd.read_json(os.path.join(predix_dir, f"{phase}.jsonl"), lines=True)
        self.label_dict = label_dict
        print(f"Loaded {len(self.meta_data)} samples from {phase} set.")
        if error_cases_remover:
            with open(os.path.join(predix_dir, "flava_embeds", f"{phase}_error_cases.txt"), "r") as f:
                error_cases = [int(x) for x in f.read().split("\n")[:-1]]
            self.meta_data = self.meta_data.drop(labels=error_cases, axis=0)
            print(f"Loaded {len(self.meta_data)} samples from {phase} set after removing {len(error_cases)} "
                  f"error cases.")

    def __len__(self):
        return len(self.meta_data)


class FlavaEncodedDataset(BaseDataset):
    """(image embeddings, text embeddings, label) per meme (reference src/dataset.py:196-213).
    The tensor files are read with torch.load(weights_only=True): they hold plain tensors."""

    def __init__(self, predix_dir, phase, label_dict, error_cases_remover=True, **kwargs):
        super().__init__(predix_dir, phase, label_dict, error_cases_remover, **kwargs)
        assert "name_extractor" in kwargs
        self.name_extractor = kwargs["name_extractor"]
        self.emb_dir = os.path.join(predix_dir, "flava_embeds")

    def __getitem__(self, idx):
        save_name = self.name_extractor(self.meta_data.iloc[idx]["img"])
        img = torch.load(os.path.join(self.emb_dir, save_name + ".img"), weights_only=True)
        txt = torch.load(os.path.join(self.emb_dir, save_name + ".text"), weights_only=True)
        label = torch.LongTensor([self.label_dict.index(self.meta_data.iloc[idx]["label"])])
        return img, txt, label


def collate_fn_flava(batch):
    """Zero-pad image / text embedding sequences to the batch maximum (reference :216-226)."""
    from torch.nn.utils.rnn import pad_sequence
    imgs, txts, labels = [], [], []
    for i, t, lab in batch:
        imgs.append(i)
        txts.append(t)
        labels.append(lab)
    imgs = pad_sequence(imgs, batch_first=True, padding_value=0.)
    txts = pad_sequence(txts, batch_first=True, padding_value=0.)
    return (imgs, txts), torch.tensor(labels)


def get_dataset(training, dev, testing, collate_func, args, sampler=None):
    """Loaders over the (optionally sub-sampled) training set (reference :287-321)."""
    torch.manual_seed(args.seed)
    n = len(training) if args.sample_size is None else args.sample_size
    training_sub = torch.utils.data.Subset(training, list(range(len(training)))[:n])
    mk = lambda ds, shuffle, smp=None: torch.utils.data.DataLoader(  # noqa: E731
        ds, batch_size=args.batch_size, shuffle=shuffle and smp is None, sampler=smp, collate_fn=collate_func,
        pin_memory=torch.cuda.is_available())
    if sampler is not None:
        sampler = sampler(training_sub)
    train = mk(training_sub, True, sampler)
    print("training_loader LENGTH:", len(train))
    return train, mk(dev, False), mk(testing, False)


def get_dataset_flava(args, datapath, sampler=None):
    kw = dict(name_extractor=args.name_extractor)
    return get_dataset(FlavaEncodedDataset(datapath, "train", args.labels, args.error_cases_remover, **kw),
                       FlavaEncodedDataset(datapath, "dev", args.labels, args.error_cases_remover, **kw),
                       FlavaEncodedDataset(datapath, "test", args.labels, args.error_cases_remover, **kw),
                       collate_fn_flava, args, sampler)


class SyntheticFlava(Dataset):
    """Seeded stand-in for FlavaEncodedDataset items: 197 image-patch embeddings (FLAVA
    ViT-B/16 at 224^2 + CLS) and a text embedding sequence of random length <= max_text."""

    def __init__(self, n, l_img=197, max_text=77, min_text=None, n_classes=2, width=768, seed=0):
        self.n, self.l_img, self.max_text, self.n_classes, self.width = n, l_img, max_text, n_classes, width
        self.min_text = max_text if min_text is None else min_text
        self.seed = seed

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        g = torch.Generator().manual_seed(self.seed * 1000003 + i)
        T = int(torch.randint(self.min_text, self.max_text + 1, (1,), generator=g))
        img = torch.randn(self.l_img, self.width, generator=g)
        txt = torch.randn(T, self.width, generator=g)
        return img, txt, torch.randint(0, self.n_classes, (1,), generator=g)


# ------------------------------------------------------------------------------ FashionMNIST
# BASELINE config 1 (train_fashionmnist.py on CPU).  Reference src/dataset.py:56-182.
def data_forming_func(x, y, phase, model_type):
    """Targets per head / view shuffles of a quarter-crop batch x [B, m, C, H, W]
    (reference src/dataset.py:56-100; the same global-RNG draws in the same order)."""
    b, m, c, h, w = x.shape
    if model_type == "Vanilla" and phase == "train":
        y = y.unsqueeze(1).repeat(1, 1)
    elif model_type == "single-model-weight-sharing":
        y = y.unsqueeze(1).repeat(1, m).view(-1)  # [B*m]
        x = x.view(-1, c, h, w)                   # [B*m, C, H, W]
    elif model_type == "MultiHead" and phase == "train":
        y = y.unsqueeze(1).repeat(1, m)
    elif model_type == "MIMO-shuffle-instance" and phase == "train":
        # 4 independent instance permutations, one per view (the reference hard-codes 4)
        xs, ys = [], []
        for i in range(4):
            idx = torch.randperm(x.size(0))
            xs.append(x[idx, i])
            ys.append(y[idx])
        x, y = torch.stack(xs, dim=1), torch.stack(ys, dim=1)
    elif model_type == "MIMO-shuffle-view" and phase == "train":
        x = x[:, torch.randperm(x.size(1))]
        y = y.unsqueeze(1).repeat(1, m)
    elif model_type == "MIMO-shuffle-all" and phase == "train":
        xs, ys = [], []
        for i in range(m):
            idx = torch.randperm(x.size(0))
            xs.append(x[idx, i])
            ys.append(y[idx])
        x, y = torch.stack(xs, dim=1), torch.stack(ys, dim=1)
        ind = torch.randperm(x.size(1))
        x, y = x[:, ind], y[:, ind]
    return x, y


class QuarterCrop(object):
    """28x28 image -> its 4 quarters [upper-left, upper-right, lower-left, lower-right]
    (reference src/dataset.py:103-127).  Works on an [H, W] array / tensor."""

    def __init__(self, expected_size):
        self.expected_size = expected_size
        self.crop_size_w = int(expected_size[0] / 2)
        self.crop_size_h = int(expected_size[1] / 2)

    def __call__(self, img):
        h, w = img.shape[-2:]
        assert w == self.expected_size[0] and h == self.expected_size[1]
        ch, cw = self.crop_size_h, self.crop_size_w
        tops, lefts = [0, 0, cw, ch], [0, ch, 0, ch]  # the reference's (starts_x, starts_y) as (top, left)
        return [img[..., t:t + ch, l:l + cw] for t, l in zip(tops, lefts)]


def read_idx(path):
    """IDX file (optionally .gz) -> numpy array (the FashionMNIST / MNIST container format)."""
    import gzip
    op = gzip.open if path.endswith(".gz") else open
    with op(path, "rb") as f:
        data = f.read()
    magic = int.from_bytes(data[0:4], "big")
    if magic >> 8 != 0x08:
        raise ValueError(f"{path}: not a uint8 IDX file (magic {magic:#x})")
    nd = magic & 0xFF
    dims = [int.from_bytes(data[4 + 4 * i:8 + 4 * i], "big") for i in range(nd)]
    arr = np.frombuffer(data, dtype=np.uint8, offset=4 + 4 * nd)
    if arr.size != int(np.prod(dims)):
        raise ValueError(f"{path}: {arr.size} bytes for dims {dims}")
    return arr.reshape(dims)


def _find_idx(root, stem):
    for d in (os.path.join(root, "FashionMNIST", "raw"), os.path.join(root, "FashionMNIST"), root):
        for name in (stem, stem + ".gz"):
            p = os.path.join(d, name)
            if os.path.exists(p):
                return p
    return None


class FashionMNISTQuarters(Dataset):
    """FashionMNIST as the reference serves it (torchvision FashionMNIST + QuarterCrop +
    ToTensor: [4, 1, 14, 14] float in [0, 1], int64 label; reference src/dataset.py:148-162).

    Labels come from the IDX label file under ``datapath``.  The image files are absent
    from this offline checkout (only the label files ship).  A missing image
    file raises FileNotFoundError (the reference downloads or fails) unless the caller
    opts in with ``synthetic_images=True``: the images are then SYNTHETIC -- seeded uint8
    28x28 noise per index, paired with the real labels -- ``self.synthetic`` is True and a
    warning is logged."""

    def __init__(self, datapath, train=True, seed=777, sample_size=None, synthetic_images=False):
        pre = "train" if train else "t10k"
        lab = _find_idx(datapath, f"{pre}-labels-idx1-ubyte")
        if lab is None:
            raise FileNotFoundError(f"no FashionMNIST {pre} label file under {datapath}")
        self.labels = torch.from_numpy(read_idx(lab).astype(np.int64))
        img = _find_idx(datapath, f"{pre}-images-idx3-ubyte")
        self.synthetic = img is None
        if self.synthetic:
            if not synthetic_images:
                raise FileNotFoundError(
                    f"no FashionMNIST {pre}-images-idx3-ubyte[.gz] under {datapath} (there is no network to "
                    f"download it); pass synthetic_images=True / --synthetic_images to train on seeded noise")
            import logging
            logging.getLogger(__name__).warning(
                "FashionMNIST %s images missing under %s: serving SYNTHETIC seeded noise images with the real "
                "labels (synthetic_images=True)", pre, datapath)
            g = torch.Generator().manual_seed(seed + (0 if train else 1))
            self.images = torch.randint(0, 256, (len(self.labels), 28, 28), generator=g, dtype=torch.uint8)
        else:
            self.images = torch.from_numpy(read_idx(img).copy())
        if sample_size is not None:
            self.labels, self.images = self.labels[:sample_size], self.images[:sample_size]
        self.crop = QuarterCrop((28, 28))

    def __len__(self):
        return len(self.labels)

    def __getitem__(self, i):
        quarters = self.crop(self.images[i].float().div(255.0))  # ToTensor: /255
        return torch.stack([q.unsqueeze(0) for q in quarters]), self.labels[i]


def get_fmnist(datapath=None, batch_size=128, download=False, shuffle=True, sample_size=None, seed=777,
               synthetic_images=False):
    """(train_loader, test_loader, None) of [B, 4, 1, 14, 14] quarter crops (reference
    src/dataset.py:130-175; ``download`` is accepted and ignored: there is no network;
    ``synthetic_images``: see FashionMNISTQuarters)."""
    if datapath is None:
        from . import DATA_DIR as datapath
    torch.manual_seed(seed)
    training = FashionMNISTQuarters(datapath, True, seed, sample_size, synthetic_images)
    testing = FashionMNISTQuarters(datapath, False, seed, sample_size, synthetic_images)
    train_loader = torch.utils.data.DataLoader(training, batch_size=batch_size, shuffle=shuffle)
    test_loader = torch.utils.data.DataLoader(testing, batch_size=batch_size, shuffle=False)
    print("training_loader LENGTH:", len(train_loader))
    return train_loader, test_loader, None
