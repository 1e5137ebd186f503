"""Tiny deterministic MMBT-shaped module for framework-loop parity (test infra only).

It exposes the attributes src/framework.py:282-285 toggles (``enc.img_encoder``,
``enc.encoder``) and the ``forward(txt, mask, segment, img)`` / ``compute_loss``
contract of src/mmbt.py:245,261, so the reference ``Model_.train_loop`` and the
build's ``Model_`` can drive the same object and their history dicts compared.
"""
import torch
import torch.nn as nn


class _Enc(nn.Module):
    def __init__(self, vocab, hid, img_feat):
        super().__init__()
        self.emb = nn.Embedding(vocab, hid)
        self.img_encoder = nn.Linear(img_feat, hid)
        self.encoder = nn.Linear(hid, hid)

    def forward(self, txt, mask, segment, img):
        t = (self.emb(txt) * mask.unsqueeze(-1).float()).sum(1) / mask.float().sum(1, keepdim=True)
        i = self.img_encoder(img.flatten(1))
        return torch.tanh(self.encoder(t + i))


class TinyMMBT(nn.Module):
    def __init__(self, vocab=50, hid=16, img_feat=12, n_classes=5, seed=0):
        super().__init__()
        g = torch.Generator().manual_seed(seed)
        self.enc = _Enc(vocab, hid, img_feat)
        self.clf = nn.Linear(hid, n_classes)
        self.loss = nn.CrossEntropyLoss()
        with torch.no_grad():
            for p in self.parameters():
                p.copy_(torch.randn(p.shape, generator=g) * 0.5)

    def forward(self, txt, mask, segment, img):
        return self.clf(self.enc(txt, mask, segment, img))

    def compute_loss(self, y_hat, y, eval=False):
        return self.loss(y_hat, y)


def tiny_batches(n_batches, bsz=4, T=6, vocab=50, n_classes=5, seed=0):
    """List of ((text, segment, mask, img), y) in collate_fn order (src/dataset.py:420-438)."""
    g = torch.Generator().manual_seed(seed)
    out = []
    for _ in range(n_batches):
        lens = torch.randint(2, T + 1, (bsz,), generator=g)
        txt = torch.randint(1, vocab, (bsz, T), generator=g)
        mask = (torch.arange(T)[None, :] < lens[:, None]).long()
        txt = txt * mask
        img = torch.randn(bsz, 3, 2, 2, generator=g)
        y = torch.randint(0, n_classes, (bsz,), generator=g)
        out.append(((txt, mask.clone(), mask, img), y))
    return out


def acc(y_pred, y_true, eval, dummy_dim=False):
    """The metric train.py:119-130 passes to Model_ (restated; train.py is not importable)."""
    if dummy_dim:
        if not eval:
            y_pred = y_pred.view(-1, y_pred.shape[2])
            y_true = y_true.view(-1)
        else:
            y_pred = y_pred.mean(1)
    _, y_pred = y_pred.max(1)
    return (y_pred == y_true).float().mean() * 100
