"""CPU: ViLT's patch selection (src/vilt.py select_patches / image_length / patch_mask, the
host half of the HIP ViLT path) against transformers' own ViltEmbeddings.visual_embed -- the
model the reference's train.py:164-182 builds -- run on the CPU with the same global RNG
state: the chosen patches (visual_embed's patch_index) and their mask values must be
identical, for full-size images (a random order of every patch), padded images (every valid
patch, then valid-mask-0 padding drawn with replacement) and a max_image_length below the
valid extent (a random subset)."""
import pytest
import torch


def _emb(max_image_length):
    from transformers import ViltConfig
    from transformers.models.vilt.modeling_vilt import ViltEmbeddings
    torch.manual_seed(0)
    cfg = ViltConfig(image_size=128, patch_size=32, hidden_size=64, num_attention_heads=2, intermediate_size=64,
                     num_hidden_layers=1, max_image_length=max_image_length)
    return ViltEmbeddings(cfg).eval(), cfg


@pytest.mark.parametrize("max_image_length,partial", [(-1, False), (-1, True), (7, False), (7, True)])
def test_patch_selection_matches_visual_embed(max_image_length, partial):
    from src.vilt import image_length, patch_mask, select_patches
    emb, cfg = _emb(max_image_length)
    B, Hh, Ww = 3, 128, 160
    g = torch.Generator().manual_seed(1)
    pix = torch.randn(B, 3, Hh, Ww, generator=g)
    pmask = torch.ones(B, Hh, Ww, dtype=torch.long)
    if partial:  # smaller images padded into the batch (ViltProcessor pad_and_create_pixel_mask)
        pmask[0, :, 96:] = 0
        pmask[2, 64:, :] = 0
    torch.manual_seed(123)
    with torch.no_grad():
        _, ref_mask, (ref_idx, _) = emb.visual_embed(pix, pmask, max_image_length=max_image_length)
    gh, gw = Hh // cfg.patch_size, Ww // cfg.patch_size
    torch.manual_seed(123)
    xm = patch_mask(pmask, gh, gw)
    L = image_length(xm, max_image_length)
    flat, mask = select_patches(xm.flatten(1), L)
    p = flat % (gh * gw)
    got_idx = torch.stack([p // gw, p % gw], -1).view(B, -1, 2)
    assert torch.equal(got_idx, ref_idx[:, 1:] if ref_idx.shape[1] == L + 1 else ref_idx)
    assert torch.equal(mask, ref_mask[:, 1:])
    after = torch.rand(4)  # the generator after our draws ...
    torch.manual_seed(123)
    with torch.no_grad():
        emb.visual_embed(pix, pmask, max_image_length=max_image_length)
    assert torch.equal(after, torch.rand(4))  # ... is where the reference leaves it


@pytest.mark.parametrize("max_image_length", [-1, 100])
def test_batched_draws_match_visual_embed_at_bench_shape(max_image_length):
    """bench.py --workload vilt's shape (64 full 384 x 384 images, 144 patches each): every
    sample keeps max_len of an equal number of valid patches, which select_patches draws with
    ONE [B, 144] multinomial call -- the same patches, and the generator left in the same state,
    as visual_embed's 64 per-sample calls"""
    from transformers import ViltConfig
    from transformers.models.vilt.modeling_vilt import ViltEmbeddings
    from src.vilt import image_length, patch_mask, select_patches
    torch.manual_seed(0)
    cfg = ViltConfig(image_size=384, patch_size=32, hidden_size=32, num_attention_heads=2, intermediate_size=32,
                     num_hidden_layers=1, max_image_length=max_image_length)
    emb = ViltEmbeddings(cfg).eval()
    B = 64
    pix = torch.randn(B, 3, 384, 384, generator=torch.Generator().manual_seed(2))
    pmask = torch.ones(B, 384, 384, dtype=torch.long)
    torch.manual_seed(7)
    with torch.no_grad():
        _, ref_mask, (ref_idx, _) = emb.visual_embed(pix, pmask, max_image_length=max_image_length)
    ref_after = torch.rand(4)
    torch.manual_seed(7)
    xm = patch_mask(pmask, 12, 12)
    L = image_length(xm, max_image_length)
    flat, mask = select_patches(xm.flatten(1), L)
    after = torch.rand(4)
    p = flat % 144
    got_idx = torch.stack([p // 12, p % 12], -1).view(B, -1, 2)
    assert torch.equal(got_idx, ref_idx[:, 1:] if ref_idx.shape[1] == L + 1 else ref_idx)
    assert torch.equal(mask, ref_mask[:, 1:])
    assert torch.equal(after, ref_after)


def test_vilt_train_refuses_cpu_tensors():
    """No CPU path: ViltTrainHIP on host tensors raises instead of falling back to torch."""
    from transformers import ViltConfig, ViltForImagesAndTextClassification
    from src._native import NativeError
    from src.vilt import ViltTrainHIP
    torch.manual_seed(0)
    cfg = ViltConfig(num_hidden_layers=1, image_size=64, patch_size=32, max_position_embeddings=8, vocab_size=50,
                     num_images=1, num_labels=2)
    hip = ViltTrainHIP(ViltForImagesAndTextClassification(cfg))
    with pytest.raises(NativeError, match="HIP"):
        hip(input_ids=torch.randint(5, 50, (2, 8)), pixel_values=torch.randn(2, 1, 3, 64, 64),
            labels=torch.tensor([0, 1]))


@pytest.mark.parametrize("cls", ["ViltHIP", "ViltTrainHIP"])
def test_vilt_refuses_head_dim_other_than_64(cls):
    """the attention kernels assume head_dim 64: 768 / 6 heads is refused, not run"""
    from transformers import ViltConfig, ViltForImagesAndTextClassification
    from src import vilt
    cfg = ViltConfig(num_hidden_layers=1, image_size=64, patch_size=32, max_position_embeddings=16, vocab_size=300,
                     num_images=1, num_attention_heads=6)
    with pytest.raises(NotImplementedError, match="head_dim 64"):
        if cls == "ViltHIP":
            vilt.ViltHIP(ViltForImagesAndTextClassification(cfg), "cpu")
        else:
            vilt.ViltTrainHIP(ViltForImagesAndTextClassification(cfg))
