"""Batched modality-robustness pass (eval_mmbt_robustness.py:76-103 semantics).

Per batch the reference runs 3 + 2*n_repeats full pipelines (full, image-only,
text-only, n image-control and n text-control forwards), recomputing ResNet-152
and both embeddings every time.  Here the image features / projection are
computed ONCE per batch and the 43 encoder passes are batched by sequence length:
  L = 5+T : full                                    1 variant
  L = 5   : image-only + n image controls           1+n variants, one embed + one encoder pass
  L = 1+T : text-only + n text controls             1+n variants, one embed + one encoder pass
The control index sets are drawn from the global torch RNG in exactly the
reference's order (all image draws, then all text draws; src/mmbt.py:198-201),
so the same seed gives the same variants.  Output: [B, 3 + 2n, n_classes] logits
in the reference's stacking order.
"""
import torch

from .mmbt import control_indices


@torch.no_grad()
def robustness_logits(model, txt, mask, segment, img, n_repeats=20):
    """model(*x) order: (txt, mask, segment, img) as forward(txt, mask, segment, img) sees them."""
    enc = model.enc
    enc._prepare()
    B, T = txt.shape
    n_img = enc.n_img
    S = n_img + 2 + T
    dev = img.device
    proj = enc.img_embeddings.project(enc._image_feats(img))
    img_idx = [control_indices(S, n_img + 1) for _ in range(n_repeats)]
    txt_idx = [control_indices(S, T) for _ in range(n_repeats)]

    def run(idx_list, Lout):
        V = len(idx_list)
        idx = torch.stack(idx_list).to(dev) if idx_list[0] is not None else None
        X, km, L = enc._embed(txt, mask, segment, proj, idx=idx, Lout=Lout, V=V)
        h = enc._encode(X, km, V * B, L)
        return model.clf(enc._pool(h, V * B, L)).view(V, B, -1)

    full = run([None], S)
    img_only = torch.arange(n_img + 2)
    txt_only = torch.cat([torch.zeros(1, dtype=torch.long), torch.arange(T) + n_img + 2])
    short = run([img_only] + img_idx, n_img + 2)
    long_ = run([txt_only] + txt_idx, T + 1)
    out = torch.cat([full, short[:1], long_[:1], short[1:], long_[1:]], dim=0)  # [3+2n, B, C]
    return out.transpose(0, 1).contiguous()
