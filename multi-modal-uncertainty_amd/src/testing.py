"""Helpers shared by tests / smoke / bench: reference-shaped ``args`` and synthetic batches.

``make_args`` builds the namespace train.py / eval_mmbt_robustness.py hand to
MultimodalBertClf (train.py:31-90 defaults); ``synthetic_batch`` draws a batch in
collate_fn order (src/dataset.py:420-438): (text, segment, mask, img), tgt.
"""
import types

import torch


class _Vocab:
    def __init__(self, size=30522):
        self.stoi = {"[PAD]": 0, "[UNK]": 100, "[CLS]": 101, "[SEP]": 102, "[MASK]": 103}
        self.vocab_sz = size


def make_args(**over):
    a = types.SimpleNamespace(
        img_embed_pool_type="avg", num_image_embeds=3, img_hidden_sz=2048, hidden_sz=768, dropout=0.0,
        bert_model="bert-base-uncased", n_classes=101, vocab=_Vocab(), max_seq_len=512,
        lr=5e-5, warmup=0.1, gradient_accumulation_steps=1, freeze_img=3, freeze_txt=5)
    for k, v in over.items():
        setattr(a, k, v)
    return a


def small_args(**over):
    """2 BERT layers, 4096-word vocab, one bottleneck per ResNet stage (fast parity cases)."""
    base = dict(bert_layers=2, vocab_size=4096, resnet_blocks=(1, 1, 1, 1))
    base.update(over)
    return make_args(**base)


def synthetic_batch(B, T, n_classes=101, vocab=30522, lens=None, seed=0, device="cpu"):
    g = torch.Generator().manual_seed(seed)
    txt = torch.randint(1000, vocab, (B, T), generator=g)
    if lens is None:
        lens = [T] * B
    mask = (torch.arange(T)[None, :] < torch.as_tensor(lens)[:, None]).long()
    txt = txt * mask
    img = torch.randn(B, 3, 224, 224, generator=g)
    y = torch.randint(0, n_classes, (B,), generator=g)
    x = (txt, mask.clone(), mask, img)
    return tuple(t.to(device) for t in x), y.to(device)
