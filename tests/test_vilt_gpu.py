"""ViLT on the HIP kernels (src/vilt.py) against transformers' own ViLT classes -- the model the
reference's train.py:164-182 setup_vilt builds (ViltForImagesAndTextClassification,
num_images=1) -- with a seeded random init (dandelin/vilt-b32-mlm is not available offline;
parity therefore rests on the module's arithmetic, not on pretrained weights).

The reference model runs in fp32 on the CPU, the HIP path in bf16 (f32 accumulation and f32
residual stream).  Bar: 1e-2 * max|reference| (north star, bf16) on the classifier logits,
the pooled output and every token of the last hidden state.  Both sides draw the image-patch
selection of ViltEmbeddings.visual_embed (torch.multinomial on the CPU generator) from the
same seeded RNG state, so the token order is the reference's.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return (a - b).abs().max().item() / b.abs().max().item()


def _model(layers=12, labels=2):
    from transformers import ViltConfig, ViltForImagesAndTextClassification
    torch.manual_seed(0)
    cfg = ViltConfig(num_images=1, num_labels=labels, num_hidden_layers=layers)
    return ViltForImagesAndTextClassification(cfg).eval()


def _inputs(B, Lt, hw, seed, pad_text=True, partial_image=False):
    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(1000, 30522, (B, Lt), generator=g)
    mask = torch.ones(B, Lt, dtype=torch.long)
    if pad_text:
        mask[1, Lt // 2:] = 0  # padded text of the second sample (collate_fn_vilt pads to max_length)
        ids[1, Lt // 2:] = 0
    pix = torch.randn(B, 1, 3, hw[0], hw[1], generator=g)
    pmask = torch.ones(B, 1, hw[0], hw[1], dtype=torch.long)
    if partial_image:  # a smaller image padded into the batch (ViltProcessor pad_and_create_pixel_mask)
        pmask[0, :, :, hw[1] * 5 // 8:] = 0
        pix[0, :, :, :, hw[1] * 5 // 8:] = 0
    return ids, mask, pix, pmask


@pytest.mark.parametrize("hw,partial", [((384, 384), False), ((384, 512), True)])
def test_vilt_classifier_matches_transformers(dev, hw, partial):
    from src.vilt import ViltHIP
    model = _model()
    ids, mask, pix, pmask = _inputs(2, 40, hw, seed=7, partial_image=partial)
    torch.manual_seed(123)
    with torch.no_grad():
        ref = model(input_ids=ids, attention_mask=mask, pixel_values=pix, pixel_mask=pmask).logits
        torch.manual_seed(123)
        ref_seq, ref_pool = model.vilt(input_ids=ids, attention_mask=mask, pixel_values=pix[:, 0],
                                       pixel_mask=pmask[:, 0], return_dict=False)[:2]
    hip = ViltHIP(model, dev)
    torch.manual_seed(123)
    got = hip(ids.to(dev), mask.to(dev), None, pix.to(dev), pmask.to(dev))
    torch.manual_seed(123)
    seq, pool = hip.vilt(ids.to(dev), mask.to(dev), None, pix[:, 0].to(dev), pmask[:, 0].to(dev))
    assert got.shape == ref.shape and seq.shape == ref_seq.shape
    errs = {"logits": _rel(got, ref), "pooled": _rel(pool, ref_pool), "last_hidden": _rel(seq, ref_seq)}
    print(f"\n[vilt {hw} partial={partial}] rel err " + ", ".join(f"{k} {v:.2e}" for k, v in errs.items()))
    for k, v in errs.items():
        assert v <= 1e-2, f"{k}: {v:.3e}"


def test_vilt_bare_model_and_two_images(dev):
    """A bare ViltModel (last hidden state + pooled output) and the two-image NLVR2 form of the
    classifier (image i takes modality type i + 1; pooled outputs concatenated)."""
    from transformers import ViltConfig, ViltForImagesAndTextClassification
    from src.vilt import ViltHIP
    torch.manual_seed(1)
    cfg = ViltConfig(num_images=2, num_labels=3, num_hidden_layers=4, modality_type_vocab_size=3)
    model = ViltForImagesAndTextClassification(cfg).eval()
    g = torch.Generator().manual_seed(3)
    ids = torch.randint(1000, 30522, (3, 24), generator=g)
    pix = torch.randn(3, 2, 3, 384, 384, generator=g)
    torch.manual_seed(9)
    with torch.no_grad():
        ref = model(input_ids=ids, pixel_values=pix).logits
    torch.manual_seed(9)
    got = ViltHIP(model, dev)(ids.to(dev), None, None, pix.to(dev))
    assert _rel(got, ref) <= 1e-2
    torch.manual_seed(9)
    with torch.no_grad():
        rs, rp = model.vilt(input_ids=ids, pixel_values=pix[:, 0], return_dict=False)[:2]
    torch.manual_seed(9)
    s, p = ViltHIP(model.vilt, dev)(ids.to(dev), None, None, pix[:, 0].to(dev))
    assert _rel(s, rs) <= 1e-2 and _rel(p, rp) <= 1e-2
