"""FLAVA image / text encoders on the HIP kernels (src/flava_encoders.py; reference
data/encoding_with_flava.py:11-41) against transformers' FlavaModel itself -- the module the
reference calls -- with a seeded random init (facebook/flava-full is not available offline):
image_embeddings [B, 197, 768] and text_embeddings [B, T, 768] (padded batch), within the
north star's bf16 bar of 1e-2 of max |ref|.  Plus CPU checks of the patch im2col."""
import os
import sys

import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "multi-modal-uncertainty_amd"))

from src.flava_encoders import patchify  # noqa: E402


def test_patchify_is_the_patch_conv():
    g = torch.Generator().manual_seed(0)
    x = torch.randn(2, 3, 64, 48, generator=g)
    w = torch.randn(20, 3, 16, 16, generator=g)
    ref = torch.nn.functional.conv2d(x, w, stride=16).flatten(2).transpose(1, 2)  # [B, P, 20]
    got = (patchify(x, 16) @ w.reshape(20, -1).t()).view(2, -1, 20)
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-4)


@pytest.fixture(scope="module")
def flava():
    from transformers import FlavaConfig, FlavaModel
    torch.manual_seed(11)
    return FlavaModel(FlavaConfig()).eval()


@pytest.mark.gpu
def test_flava_encoders_match_transformers(flava):
    from src.flava_encoders import FlavaEncodersHIP
    g = torch.Generator().manual_seed(3)
    B, T = 3, 21
    px = torch.randn(B, 3, 224, 224, generator=g)
    ids = torch.randint(1000, 30000, (B, T), generator=g)
    am = torch.ones(B, T, dtype=torch.long)
    am[1, 15:] = 0
    am[2, 7:] = 0
    ids = ids * am
    with torch.no_grad():
        ref_img = flava.image_model(pixel_values=px)[0]
        ref_txt = flava.text_model(input_ids=ids, attention_mask=am)[0]
    enc = FlavaEncodersHIP(flava, "cuda")
    img, txt = enc(px.cuda(), ids.cuda(), am.cuda())
    assert img.shape == ref_img.shape and txt.shape == ref_txt.shape
    err_i = (img.cpu() - ref_img).abs().max().item()
    assert err_i <= 1e-2 * ref_img.abs().max().item(), (err_i, ref_img.abs().max().item())
    keep = am.bool()  # padded positions are not saved (encoding_with_flava cuts each text to its length)
    err_t = (txt.cpu() - ref_txt)[keep].abs().max().item()
    assert err_t <= 1e-2 * ref_txt[keep].abs().max().item(), (err_t, ref_txt[keep].abs().max().item())
    # a sample encoded alone equals its row of the padded batch (what the batched script relies on)
    _, t1 = enc(None, ids[2:3, :7].cuda(), am[2:3, :7].cuda())
    assert (t1[0].cpu() - txt[2, :7].cpu()).abs().max().item() <= 1e-2 * ref_txt[keep].abs().max().item()
