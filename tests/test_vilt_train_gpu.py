"""ViLT TRAINING on the HIP kernels (src/vilt.py ViltTrainHIP) against transformers'
ViltForImagesAndTextClassification itself -- the model the reference trains (train.py:164-182
setup_vilt, src/framework.py:262-300: outputs = model(**batch); outputs.loss.backward()) -- run
in fp32 autograd on the same GPU from the same weights, with the same patch draws (the global CPU
generator, seeded identically before each forward).  Random-init weights of the reference's
architecture (dandelin/vilt-b32-mlm is not offline), 2 layers, 64 x 64 images (4 patches).

Bars, written before the first run: loss within 1e-2 relative; logits within 1e-2 of max|logit|;
per-parameter-tensor gradient error ||g_hip - g_ref|| / ||g_ref|| with median <= 1e-2 and 90th
percentile <= 5e-2.  One AdamW step on each is printed as a diagnostic only (Adam's first step
is lr * sign(g) per element, so near-zero gradients flip their element's update on noise)."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def _setup(dev, partial):
    from transformers import ViltConfig, ViltForImagesAndTextClassification
    from src.vilt import ViltTrainHIP
    torch.manual_seed(0)
    cfg = ViltConfig(num_hidden_layers=2, image_size=64, patch_size=32, max_position_embeddings=16, vocab_size=300,
                     num_images=1, num_labels=3)
    ref = ViltForImagesAndTextClassification(cfg).to(dev).train()
    hip_model = copy.deepcopy(ref)
    hip = ViltTrainHIP(hip_model)
    g = torch.Generator().manual_seed(3)
    B, Lt = 4, 16
    ids = torch.randint(5, 300, (B, Lt), generator=g).to(dev)
    am = torch.ones(B, Lt, dtype=torch.long)
    am[1, 10:] = 0
    am[3, 5:] = 0
    pix = torch.randn(B, 3, 64, 64, generator=g).to(dev)
    pm = torch.ones(B, 64, 64, dtype=torch.long)
    if partial:  # a smaller image padded into the batch: 2 of its 4 patches valid
        pm[2, :, 32:] = 0
    y = torch.tensor([0, 2, 1, 2], device=dev)
    # [B, num_images, ...] (the model indexes pixel_mask per image)
    batch = dict(input_ids=ids, attention_mask=am.to(dev), pixel_values=pix[:, None], pixel_mask=pm[:, None].to(dev),
                 labels=y)
    return ref, hip_model, hip, batch


@pytest.mark.parametrize("partial", [False, True])
def test_vilt_train_step_matches_transformers(dev, partial):
    from src.vilt import ViltTrainHIP
    ref, hip_model, hip, batch = _setup(dev, partial)
    assert isinstance(hip, ViltTrainHIP)
    torch.manual_seed(7)
    out_r = ref(**batch)
    out_r.loss.backward()
    torch.manual_seed(7)
    out_h = hip(**batch)
    out_h.loss.backward()
    torch.cuda.synchronize()
    lr, lh = out_r.loss.item(), out_h.loss.item()
    lg_err = (out_h.logits.float() - out_r.logits.float()).abs().max().item()
    lg_scale = out_r.logits.abs().max().item()
    errs, held = [], []
    gmax = max(p.grad.norm().item() for p in ref.parameters() if p.grad is not None)
    for (n, pr), (n2, ph) in zip(ref.named_parameters(), hip_model.named_parameters()):
        assert n == n2
        if pr.grad is None or pr.grad.norm().item() == 0.0:
            assert ph.grad is None or ph.grad.abs().max().item() == 0.0, n
            continue
        assert ph.grad is not None, n
        errs.append(((ph.grad - pr.grad).norm() / pr.grad.norm()).item())
        # every tensor is held, except the ones whose true gradient is noise: under
        # 1e-4 x the largest gradient norm, and the key biases (softmax shift invariance: exactly 0)
        if pr.grad.norm().item() > 1e-4 * gmax and "attention.key.bias" not in n:
            held.append((n, errs[-1]))
        if errs[-1] > 5e-2:
            print(f"  {n}: grad rel err {errs[-1]:.3e} (norm {pr.grad.norm().item():.3e})")
    e = torch.tensor(errs)
    med, p90 = e.median().item(), e.quantile(0.9).item()
    worst = max(held, key=lambda r: r[1])
    print(f"\n[vilt train{' partial' if partial else ''}] loss ref {lr:.6f} hip {lh:.6f}; logits err {lg_err:.2e} "
          f"(scale {lg_scale:.2e}); {len(errs)} grads: median {med:.2e} p90 {p90:.2e} max {e.max().item():.2e}; "
          f"{len(held)} held: worst {worst[1]:.2e} ({worst[0]})")
    assert abs(lh - lr) <= 1e-2 * abs(lr)
    assert lg_err <= 1e-2 * lg_scale
    assert med <= 1e-2 and p90 <= 5e-2
    assert worst[1] <= 5e-2, worst
    # one AdamW step on each (the reference's optimizer, train.py:168)
    p0 = [p.detach().clone() for p in ref.parameters()]
    for m in (ref, hip_model):
        opt = torch.optim.AdamW(m.parameters(), lr=1e-4)
        opt.step()
    du = torch.cat([(a.detach() - b).flatten() for a, b in zip(ref.parameters(), p0)])
    dh = torch.cat([(a.detach() - b).flatten() for a, b in zip(hip_model.parameters(), p0)])
    upd = ((dh - du).norm() / du.norm()).item()
    print(f"  AdamW first-step update rel err {upd:.2e} (diagnostic)")


def test_vilt_train_refuses_dropout(dev):
    from transformers import ViltConfig, ViltForImagesAndTextClassification
    from src.vilt import ViltTrainHIP
    cfg = ViltConfig(num_hidden_layers=1, image_size=64, patch_size=32, max_position_embeddings=16, vocab_size=300,
                     num_images=1, hidden_dropout_prob=0.1)
    with pytest.raises(NotImplementedError):
        ViltTrainHIP(ViltForImagesAndTextClassification(cfg))


def test_vilt_train_through_the_framework_loop(dev, tmp_path):
    """ViltTrainHIP as the model of the reference's training loop (Model_.train_loop with
    vilt=True: batches are dicts with "labels", outputs.loss / outputs.logits), AdamW as
    setup_vilt builds it: two epochs of two steps run, the history has the loop's keys, the
    loss is finite and the parameters moved."""
    from oracle.tiny_model import acc
    from src import framework, training_loop
    ref, hip_model, hip, batch = _setup(dev, False)
    del ref
    opt = torch.optim.AdamW(hip.parameters(), lr=1e-4)
    sched = torch.optim.lr_scheduler.ReduceLROnPlateau(opt, "max", patience=0, factor=0.5)
    batches = [{k: v for k, v in batch.items()} for _ in range(2)]
    H = {}
    d = str(tmp_path)
    cbs = training_loop._construct_default_callbacks(hip, opt, H, d, checkpoint_monitor="val_acc")
    for c in cbs:
        c.set_save_path(d)
        c.set_model(hip, ignore=False)
        c.set_optimizer(opt)
    m = framework.Model_(model=hip, optimizer=opt, scheduler=sched, data_forming_func=None, metrics=[acc])
    m.device = dev
    for c in cbs:
        c.set_model_pytoune(m)
    w0 = hip_model.classifier[0].weight.detach().clone()
    torch.manual_seed(11)
    m.train_loop(batches, valid_generator=batches, test_generator=batches, steps_per_epoch=2, validation_steps=2,
                 test_steps=2, epochs=2, callbacks=cbs, patience=10, epoch_start=1, scheduler_step_on="epoch",
                 auc=False, vilt=True, mmbt=False, gradient_accumulation_steps=1, scheduler_metric="val_acc")
    print(f"\n[vilt loop] history keys {list(H.keys())}, loss {H.get('loss')}")
    assert H["epoch"] == [1, 2]
    assert all(torch.isfinite(torch.tensor(H["loss"])))
    assert not torch.equal(w0, hip_model.classifier[0].weight.detach())
