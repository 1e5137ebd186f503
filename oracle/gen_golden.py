"""Generate tests/golden/* by running the REFERENCE's own code in this container.

Run:  python -m oracle.gen_golden          (needs /root/reference; CPU only)

* MMBT fixtures: the reference ``src/mmbt.py`` MultimodalBertClf with the
  golden_stubs/ third-party stand-ins, weights loaded from oracle/weights.py
  (strict), inputs synthetic (seeded).  Every forward variant
  (src/mmbt.py:245-259) is recorded with the control indices the reference drew
  from the global RNG (src/mmbt.py:199), plus image features, embeddings, pooled
  output, CE loss (eval) and a train-mode (BN batch stats, dropout 0) loss with
  per-tensor grad norms.
* FLAVA fixtures: the reference ``src/model.py`` FlavaFusionTransfomer /
  FlavaFusionTransfomerwithCLSToken with weights from
  oracle/flava_ref.make_state_dict (strict), synthetic embeddings (seeded):
  eval logits + losses, a train-mode loss (dropout 0) with per-tensor grad norms,
  and the MIMO permutations of data_forming_func_transformer (src/dataset.py:30-54).
* robustness fixtures (A11): the eval_mmbt_robustness.py:77-93 per-batch loop over the
  reference model, [B, 3 + 2n, C] with the drawn control index sets.
* A0 fixture: the reference's own JsonlDataset / collate_fn / numpy_seed over a committed
  jsonl (tests/golden/a0/) -> text / segment / mask / image / label batches.
* framework fixture: the reference ``Model_.train_loop`` (src/framework.py:213)
  with ``_construct_default_callbacks`` (src/training_loop.py:23-47) driving
  oracle/tiny_model.TinyMMBT for 2 epochs x 3 steps; history + checkpoint keys.

Only arrays (inputs / outputs) are written -- no reference source.
"""
import argparse
import json
import os
import sys
import tempfile
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REF = "/root/reference"
OUT = os.path.join(REPO, "tests", "golden")


def _import_reference(cfg, dropout):
    # transformers must resolve the real (absent) torchvision before the stub is visible
    import transformers.models.bert.modeling_bert  # noqa: F401
    sys.path[:0] = [os.path.join(HERE, "golden_stubs"), REF]
    os.environ.setdefault("DATA_DIR", tempfile.gettempdir())
    if not hasattr(np, "Inf"):
        np.Inf = np.inf  # numpy 2 removed the alias src/callbacks.py:205-215 uses
    import torchvision.models as tvm
    from pytorch_pretrained_bert import modeling as ppb
    tvm.BLOCKS = tuple(cfg.resnet_blocks)
    ppb.CONFIG.update(num_hidden_layers=cfg.n_layers, vocab_size=cfg.vocab,
                      hidden_dropout_prob=dropout, attention_probs_dropout_prob=dropout)
    from src import mmbt, framework, training_loop  # the reference's own modules
    return mmbt, framework, training_loop


def _args(cfg):
    a = types.SimpleNamespace()
    a.img_embed_pool_type, a.num_image_embeds = "avg", cfg.num_image_embeds
    a.img_hidden_sz, a.hidden_sz, a.dropout = cfg.img_hidden, cfg.hidden, 0.0
    a.bert_model, a.n_classes = "bert-base-uncased", cfg.n_classes
    a.vocab = types.SimpleNamespace(stoi={"[CLS]": cfg.cls_id, "[SEP]": cfg.sep_id})
    return a


def make_inputs(cfg, B, T, lens, seed):
    """Synthetic batch in collate_fn order (src/dataset.py:420-438)."""
    g = torch.Generator().manual_seed(seed)
    txt = torch.randint(1000, cfg.vocab, (B, T), generator=g)
    mask = (torch.arange(T)[None, :] < torch.as_tensor(lens)[:, None]).long()
    txt = txt * mask
    segment = mask.clone()  # segment = 1 on real tokens (src/dataset.py:403)
    img = torch.randn(B, 3, 224, 224, generator=g)
    y = torch.randint(0, cfg.n_classes, (B,), generator=g)
    return (txt, segment, mask, img), y


def gen_mmbt(tag, cfg, B, T, lens, seed=0, wseed=0):
    from oracle.weights import make_state_dict, checksum
    mmbt, _, _ = _import_reference(cfg, 0.0)
    torch.manual_seed(1234)
    model = mmbt.MultimodalBertClf(_args(cfg))
    sd = make_state_dict(wseed, cfg)
    ref_keys = list(model.state_dict().keys())
    model.load_state_dict(sd, strict=True)
    x, y = make_inputs(cfg, B, T, lens, seed)
    rec = {}
    hooks = [model.enc.img_encoder.register_forward_hook(lambda m, i, o: rec.__setitem__("feats", o.detach())),
             model.enc.img_embeddings.register_forward_hook(lambda m, i, o: rec.__setitem__("img_emb", o.detach())),
             model.enc.txt_embeddings.register_forward_hook(lambda m, i, o: rec.__setitem__("txt_emb", o.detach())),
             model.enc.pooler.register_forward_hook(lambda m, i, o: rec.__setitem__("pooled", o.detach()))]
    out = {"text": x[0].numpy(), "segment": x[1].numpy(), "mask": x[2].numpy(), "y": y.numpy(),
           "img_sum": np.float64(x[3].double().sum()), "weight_checksum": np.float64(checksum(sd)),
           "seed": np.int64(seed), "wseed": np.int64(wseed), "bn_last_gamma": np.float64(cfg.bn_last_gamma)}
    model.eval()
    with torch.no_grad():
        logits = model(*x)
        out["logits_full"] = logits.numpy()
        out["pooled_full"] = rec["pooled"].numpy()
        out["feats"] = rec["feats"].numpy()
        out["img_emb"] = rec["img_emb"].numpy()
        te = rec["txt_emb"]
        out["txt_emb_head"], out["txt_emb_tail"] = te[:, :4].numpy(), te[:, -4:].numpy()
        out["txt_emb_sum"] = te.double().sum((1, 2)).numpy()
        out["loss_eval"] = np.float64(model.compute_loss(logits, y, eval=True))
        out["logits_img_only"] = model.forward_img_only(*x).numpy()
        out["logits_txt_only"] = model.forward_txt_only(*x).numpy()
        real_randperm = torch.randperm
        for modal in ("image", "text"):
            drawn = []

            def rp(n, *a, **k):
                r = real_randperm(n, *a, **k)
                drawn.append(r.clone())
                return r
            torch.randperm = rp
            try:
                torch.manual_seed(77 if modal == "image" else 78)
                out[f"logits_control_{modal}"] = model.forward_control(*x, modal).numpy()
            finally:
                torch.randperm = real_randperm
            n = cfg.num_image_embeds + 1 if modal == "image" else T
            idx = np.zeros(n + 1, dtype=np.int64)
            idx[1:] = np.sort(drawn[0][:n].numpy() + 1)
            out[f"indices_control_{modal}"] = idx
    for h in hooks:
        h.remove()
    # train-mode step: BN batch statistics, dropout 0 (deterministic) -> loss + grad norms
    model.train()
    model.zero_grad()
    loss = model.compute_loss(model(*x), y)
    loss.backward()
    names = [n for n, p in model.named_parameters()]
    out["loss_train"] = np.float64(loss.detach())
    out["grad_norms"] = np.array([float(p.grad.double().norm()) if p.grad is not None else 0.0
                                  for _, p in model.named_parameters()])
    out["clf_weight_grad"] = model.clf.weight.grad.numpy()
    out["img_proj_bias_grad"] = model.enc.img_embeddings.img_embeddings.bias.grad.numpy()
    # eval mode on BatchNorm running statistics fitted to this batch: momentum 1 makes one
    # train-mode pass copy the batch mean / unbiased variance into running_mean / running_var,
    # so the eval trunk sees normalised activations (the random-init running stats of the
    # seeded recipe do not normalise them) and a bf16 trunk is comparable at 1e-2
    for mod in model.modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            mod.momentum = 1.0
    model.train()
    with torch.no_grad():
        model(*x)
    out["bnfit_running_mean_sum"] = np.float64(sum(float(m.running_mean.double().sum()) for m in model.modules()
                                                   if isinstance(m, torch.nn.BatchNorm2d)))
    model.eval()
    with torch.no_grad():
        lf = model(*x)
        out["bnfit_logits_full"] = lf.numpy()
        out["bnfit_loss_eval"] = np.float64(model.compute_loss(lf, y, eval=True))
        out["bnfit_logits_img_only"] = model.forward_img_only(*x).numpy()
        out["bnfit_logits_txt_only"] = model.forward_txt_only(*x).numpy()
        for modal in ("image", "text"):
            torch.manual_seed(77 if modal == "image" else 78)  # the same index sets as above
            out[f"bnfit_logits_control_{modal}"] = model.forward_control(*x, modal).numpy()
    os.makedirs(OUT, exist_ok=True)
    np.savez_compressed(os.path.join(OUT, f"mmbt_{tag}.npz"), **out)
    with open(os.path.join(OUT, f"mmbt_{tag}_keys.json"), "w") as f:
        json.dump({"state_dict_keys": ref_keys, "named_parameters": names}, f)
    print(f"wrote mmbt_{tag}: loss_eval={out['loss_eval']:.6f} loss_train={out['loss_train']:.6f}")


def gen_robustness(tag, cfg, B, T, lens, n_repeats, seed=0, wseed=0, rng_seed=2024):
    """A11: the per-batch loop of eval_mmbt_robustness.py:77-93 on the reference's own
    MultimodalBertClf (eval mode): full, image-only, text-only, then n_repeats image-control
    and n_repeats text-control forwards, stacked along dim 1 -> [B, 3 + 2n, C].  The control
    index sets come from the global torch RNG (src/mmbt.py:199), seeded once before the
    batch; the drawn index sets are recorded too."""
    from oracle.weights import make_state_dict, checksum
    mmbt, _, _ = _import_reference(cfg, 0.0)
    torch.manual_seed(1234)
    model = mmbt.MultimodalBertClf(_args(cfg))
    sd = make_state_dict(wseed, cfg)
    model.load_state_dict(sd, strict=True)
    x, y = make_inputs(cfg, B, T, lens, seed)
    model.eval()
    real_randperm = torch.randperm
    drawn = []

    def rp(n, *a, **k):
        r = real_randperm(n, *a, **k)
        drawn.append(r.clone())
        return r
    torch.randperm = rp
    try:
        torch.manual_seed(rng_seed)
        with torch.no_grad():
            outputs = [model(*x), model.forward_img_only(*x), model.forward_txt_only(*x)]
            for modal in ("image", "text"):
                for _ in range(n_repeats):
                    outputs.append(model.forward_control(*x, modal))
    finally:
        torch.randperm = real_randperm
    stack = torch.stack(outputs, dim=1)
    idx = []
    for j, r in enumerate(drawn):
        n = cfg.num_image_embeds + 1 if j < n_repeats else T
        idx.append(np.concatenate([[0], np.sort(r[:n].numpy() + 1)]))
    out = {"text": x[0].numpy(), "segment": x[1].numpy(), "mask": x[2].numpy(), "y": y.numpy(),
           "img_sum": np.float64(x[3].double().sum()), "weight_checksum": np.float64(checksum(sd)),
           "seed": np.int64(seed), "wseed": np.int64(wseed), "rng_seed": np.int64(rng_seed),
           "n_repeats": np.int64(n_repeats), "preds": stack.numpy(),
           "indices_image": np.stack(idx[:n_repeats]), "indices_text": np.stack(idx[n_repeats:])}
    os.makedirs(OUT, exist_ok=True)
    np.savez_compressed(os.path.join(OUT, f"robustness_{tag}.npz"), **out)
    print(f"wrote robustness_{tag}: preds {tuple(stack.shape)}")


def _reference_function(relpath, name, ns=None):
    """One top-level function (or class) of a reference module whose other imports are
    absent here (src/dataset.py needs torchvision transforms, a tokenizer, ViltProcessor):
    the definition is compiled from the reference file and run in a namespace holding
    torch (+ ``ns``).  Used to record golden outputs only."""
    import ast
    src_path = os.path.join(REF, relpath)
    tree = ast.parse(open(src_path).read(), filename=src_path)
    node = next(n for n in tree.body if isinstance(n, (ast.FunctionDef, ast.ClassDef)) and n.name == name)
    ns = dict({"torch": torch}, **(ns or {}))
    exec(compile(ast.Module(body=[node], type_ignores=[]), src_path, "exec"), ns)
    return ns[name]


A0_WORDS = [f"w{i}" for i in range(40)]


def a0_vocab_stoi():
    """The A0 fixture's vocabulary (Vocab() specials then the words, src/dataset.py:440-460)."""
    itos = ["[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]"] + A0_WORDS
    return {w: i for i, w in enumerate(itos)}


def a0_transform(image):
    """The fixture's image transform: PIL bilinear resize to 8x8, uint8 CHW tensor (the
    same PIL call on both sides; torchvision's Resize/CenterCrop/Normalize are absent here)."""
    from PIL import Image
    return torch.from_numpy(np.asarray(image.resize((8, 8), Image.BILINEAR), dtype=np.uint8).copy()).permute(2, 0, 1)


def gen_a0():
    """A0 input contract: the reference's own JsonlDataset (src/dataset.py:348-405),
    get_labels_and_frequencies (:408-417), collate_fn (:420-438) and numpy_seed
    (src/utils.py:167-181) over a committed jsonl (tests/golden/a0/), a str.split tokenizer,
    a fixed vocab and a PIL resize transform; drop_img_percent 0 and 0.5; max_seq_len 12 and
    512 with num_image_embeds 3."""
    from contextlib import contextmanager
    from collections import Counter
    from PIL import Image
    from torch.utils.data import Dataset
    d = os.path.join(OUT, "a0")
    os.makedirs(d, exist_ok=True)
    rng = np.random.default_rng(7)
    for name, hw in (("a.png", (30, 41)), ("b.png", (25, 19)), ("c.png", (16, 16))):
        Image.fromarray(rng.integers(0, 256, hw + (3,), dtype=np.uint8)).save(os.path.join(d, name))
    labels_pool = ["pizza", "ramen", "sushi", "tacos"]
    rows = []
    for i in range(10):
        n = [0, 1, 3, 8, 9, 10, 25, 600, 5, 2][i]
        words = [A0_WORDS[int(k)] if k < len(A0_WORDS) else "oov%d" % k for k in rng.integers(0, 46, n)]
        rows.append({"text": " ".join(words), "img": [None, "a.png", "b.png", "c.png"][i % 4] if i != 3 else "a.png",
                     "label": labels_pool[int(rng.integers(0, 4))]})
    with open(os.path.join(d, "train.jsonl"), "w") as f:
        for r in rows:
            f.write(json.dumps(r) + "\n")
    numpy_seed = _reference_function("src/utils.py", "numpy_seed", {"np": np, "contextmanager": contextmanager})
    ns = {"np": np, "json": json, "os": os, "Image": Image, "Dataset": Dataset, "numpy_seed": numpy_seed,
          "Counter": Counter}
    JsonlDataset = _reference_function("src/dataset.py", "JsonlDataset", ns)
    collate_fn = _reference_function("src/dataset.py", "collate_fn", ns)
    get_labels = _reference_function("src/dataset.py", "get_labels_and_frequencies", ns)
    path = os.path.join(d, "train.jsonl")
    labels, freqs = get_labels(path)
    vocab = types.SimpleNamespace(stoi=a0_vocab_stoi())
    out = {"labels": np.array(labels), "label_counts": np.array([freqs[k] for k in labels])}
    for tag, drop, msl in (("d0_m12", 0.0, 12), ("d50_m12", 0.5, 12), ("d50_m512", 0.5, 512)):
        ds = JsonlDataset(path, str.split, a0_transform, vocab, len(labels), drop, msl, 3, labels)
        out[f"{tag}_img_dropped"] = np.array([r["img"] is None for r in ds.data])
        items = [ds[i] for i in range(len(ds))]
        out[f"{tag}_item_lens"] = np.array([len(it[0]) for it in items])
        for lo, hi in ((0, 4), (4, 10)):
            (txt, seg, mask, img), tgt = collate_fn(items[lo:hi])
            for k, v in (("text", txt), ("segment", seg), ("mask", mask), ("img", img), ("tgt", tgt)):
                out[f"{tag}_b{lo}_{k}"] = v.numpy()
                out[f"{tag}_b{lo}_{k}_dtype"] = np.array(str(v.dtype))
    np.savez_compressed(os.path.join(OUT, "a0_contract.npz"), **out)
    print("wrote a0_contract.npz", {k: v.shape for k, v in out.items() if k.endswith("_text")})


def gen_flava(tag, cfg, B, L_img, L_txt, seed):
    from oracle import flava_ref as FR
    _import_reference(__import__("oracle.weights", fromlist=["SMALL"]).SMALL, 0.0)
    from src import model as ref_model  # the reference's own module
    forming = _reference_function("src/dataset.py", "data_forming_func_transformer")
    cls = ref_model.FlavaFusionTransfomerwithCLSToken if cfg.clstoken else ref_model.FlavaFusionTransfomer
    torch.manual_seed(4321)
    model = cls(out_dim=cfg.out_dim, num_classes=cfg.n_classes, multimodal_num_attention_heads=cfg.heads,
                multimodal_num_hidden_layers=cfg.layers, drop=cfg.drop, avg_pool=cfg.avg_pool)
    sd = FR.make_state_dict(seed, cfg)
    ref_keys = list(model.state_dict().keys())
    model.load_state_dict(sd, strict=True)
    img, txt, y = FR.make_inputs(B, L_img, L_txt, cfg.n_classes, cfg.out_dim, seed + 1)
    out = {"img_sum": np.float64(img.double().sum()), "txt_sum": np.float64(txt.double().sum()),
           "y": y.numpy(), "B": np.int64(B), "L_img": np.int64(L_img), "L_txt": np.int64(L_txt),
           "seed": np.int64(seed)}
    model.eval()
    with torch.no_grad():
        logits = model((img, txt))
        out["logits"] = logits.numpy()
        out["loss_eval"] = np.float64(model.compute_loss(logits, y, eval=True))
    model.train()
    model.zero_grad()
    x2, y2 = forming((img, txt), y, phase="train",
                                                       model_type="Vanilla" if cfg.out_dim == 1 else "MultiHead")
    logits = model(x2)
    loss = model.compute_loss(logits, y2)
    loss.backward()
    out["logits_train"] = logits.detach().numpy()
    out["loss_train"] = np.float64(loss.detach())
    names = [n for n, _ in model.named_parameters()]
    out["grad_norms"] = np.array([float(p.grad.double().norm()) for _, p in model.named_parameters()])
    out["proj_bias_grad"] = model.image_to_mm_projection.bias.grad.numpy()
    # MIMO-shuffle-instance: the permutations the reference draws from the global RNG
    torch.manual_seed(99)
    (pi, pt), py = forming((img, txt), y, phase="train",
                                                             model_type="MIMO-shuffle-instance")
    out["mimo_y"] = py.numpy()
    out["mimo_img_rowsum"] = pi.double().sum((1, 2)).numpy()
    out["mimo_txt_rowsum"] = pt.double().sum((1, 2)).numpy()
    os.makedirs(OUT, exist_ok=True)
    np.savez_compressed(os.path.join(OUT, f"flava_{tag}.npz"), **out)
    with open(os.path.join(OUT, f"flava_{tag}_keys.json"), "w") as f:
        json.dump({"state_dict_keys": ref_keys, "named_parameters": names}, f)
    print(f"wrote flava_{tag}: loss_eval={out['loss_eval']:.6f} loss_train={out['loss_train']:.6f}")


FLAVA_CASES = {  # tag: (cfg kwargs, B, L_img, L_txt, seed)
    "vanilla": (dict(out_dim=1), 6, 9, 7, 10),
    "multihead_avgpool": (dict(out_dim=2, avg_pool=True), 5, 11, 6, 11),
    "cls_multihead": (dict(out_dim=2, clstoken=True), 4, 8, 5, 12),
    "full_b32": (dict(out_dim=2), 32, 197, 77, 13),
}


FMNIST_TYPES = ["Vanilla", "MIMO-shuffle-instance", "MIMO-shuffle-view", "MultiHead", "MIMO-shuffle-all",
                "single-model-weight-sharing"]


def gen_fmnist():
    """BASELINE config 1: the reference src/model.py MIMOResNet / MIMOTransfomer and
    src/dataset.py data_forming_func on a seeded [B, 4, 1, 14, 14] quarter-crop batch, the
    reference train_fashionmnist.py acc, and one SGD step (train_fashionmnist.py:115-118)."""
    from oracle.weights import SMALL
    _import_reference(SMALL, 0.0)
    from src import model as ref_model  # the reference's own module
    forming = _reference_function("src/dataset.py", "data_forming_func")
    ref_acc = _reference_function("train_fashionmnist.py", "acc")
    B = 6
    g = torch.Generator().manual_seed(31)
    x = torch.rand(B, 4, 1, 14, 14, generator=g)
    y = torch.randint(0, 10, (B,), generator=g)
    out = {"x": x.numpy(), "y": y.numpy()}
    for mt in FMNIST_TYPES:
        torch.manual_seed(500)
        xf, yf = forming(x, y, "train", model_type=mt)
        out[f"form_{mt}_x"], out[f"form_{mt}_y"] = xf.numpy(), yf.numpy()
        emb, od = ref_model.model_configure[mt]
        torch.manual_seed(600)
        model = ref_model.MIMOResNet(num_channels=1, emb_dim=emb, out_dim=od, num_classes=10)
        sd = model.state_dict()
        # weights: the reference's own seeded init; the build's module tree must draw the same
        # numbers in the same order (checked per tensor by these sums)
        out[f"init_{mt}_sums"] = np.array([float(v.double().sum()) for v in sd.values()])
        opt = torch.optim.SGD(model.parameters(), lr=0.1, weight_decay=0.001, momentum=0.9)
        model.train()
        yh = model(xf)
        loss = model.compute_loss(yh, yf)
        opt.zero_grad()
        loss.backward()
        out[f"train_{mt}_logits"] = yh.detach().numpy()
        out[f"train_{mt}_loss"] = np.float64(loss.detach())
        out[f"train_{mt}_acc"] = np.float64(ref_acc(yh.detach(), yf, False))
        out[f"train_{mt}_grad_norms"] = np.array([float(p.grad.double().norm()) for p in model.parameters()])
        opt.step()
        out[f"train_{mt}_param_sums"] = np.array([float(p.detach().double().sum()) for p in model.parameters()])
        model.eval()
        with torch.no_grad():
            xe, ye = forming(x, y, "eval", model_type=mt)
            ye_hat = model(xe)
            out[f"eval_{mt}_logits"] = ye_hat.numpy()
            out[f"eval_{mt}_loss"] = np.float64(model.compute_loss(ye_hat, ye, eval=True))
            out[f"eval_{mt}_acc"] = np.float64(ref_acc(ye_hat, ye, True))
        out[f"keys_{mt}"] = np.array(list(model.state_dict().keys()))
    # MIMOTransfomer (eval, dropout 0): logits the HIP fusion blocks must reproduce
    for mt in ("MultiHead", "MIMO-shuffle-instance"):
        torch.manual_seed(700)
        model = ref_model.MIMOTransfomer(out_dim=4, num_classes=10, hidden_size=768, image_dim=196,
                                         multimodal_num_hidden_layers=3, multimodal_num_attention_heads=3, drop=0)
        model.eval()
        out[f"tf_{mt}_init_sums"] = np.array([float(v.double().sum()) for v in model.state_dict().values()])
        out[f"tf_{mt}_keys"] = np.array(list(model.state_dict().keys()))
        with torch.no_grad():
            out[f"tf_{mt}_logits"] = model(x).numpy()
            out[f"tf_{mt}_loss_eval"] = np.float64(model.compute_loss(model(x), y, eval=True))
    np.savez_compressed(os.path.join(OUT, "fmnist.npz"), **out)
    print("wrote fmnist.npz")


def gen_framework():
    from oracle.weights import SMALL
    from oracle.tiny_model import TinyMMBT, tiny_batches, acc
    _, framework, training_loop = _import_reference(SMALL, 0.0)
    model = TinyMMBT()
    opt = torch.optim.SGD(model.parameters(), lr=0.05, momentum=0.9)
    sched = torch.optim.lr_scheduler.ReduceLROnPlateau(opt, "max", patience=0, factor=0.5)
    train, val, test = tiny_batches(3, seed=1), tiny_batches(2, seed=2), tiny_batches(2, seed=3)
    H = {}
    with tempfile.TemporaryDirectory() as d:
        cbs = training_loop._construct_default_callbacks(model, opt, H, d, checkpoint_monitor="val_acc")
        for c in cbs:
            c.set_save_path(d)
            c.set_model(model, ignore=False)
            c.set_optimizer(opt)
        m = framework.Model_(model=model, optimizer=opt, scheduler=sched,
                             data_forming_func=lambda x, y, phase="train": (x, y), metrics=[acc])
        for c in cbs:
            c.set_model_pytoune(m)
        m.train_loop(train, valid_generator=val, test_generator=test, steps_per_epoch=len(train),
                     validation_steps=len(val), test_steps=len(test), epochs=2, callbacks=cbs, patience=10,
                     epoch_start=1, scheduler_step_on="epoch", auc=False, vilt=False, mmbt=True,
                     freeze_img=2, freeze_txt=3, gradient_accumulation_steps=2, scheduler_metric="val_acc")
        files = sorted(os.listdir(d))
        ck = torch.load(os.path.join(d, "model_last_epoch.pt"), weights_only=True)
        import pandas as pd
        csv_cols = list(pd.read_csv(os.path.join(d, "history.csv")).columns)
    hist = {k: [float(v) if not isinstance(v, str) else v for v in vals] for k, vals in H.items()}
    res = {"history": hist, "files": files, "ckpt_keys": sorted(ck.keys()),
           "model_keys": list(ck["model"].keys()), "optimizer_state_keys": sorted(ck["optimizer"].keys()),
           "csv_columns": csv_cols,
           "final_params": {k: v.tolist() for k, v in model.state_dict().items()}}
    with open(os.path.join(OUT, "framework_tiny.json"), "w") as f:
        json.dump(res, f, indent=1)
    print("wrote framework_tiny.json", files)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--what", default="all", choices=["all", "small", "small_b8", "full", "full_c", "full_c4", "framework", "flava",
                                                       "robustness", "fmnist", "a0"])
    a = ap.parse_args()
    sys.path.insert(0, REPO)
    from oracle.weights import SMALL, FULL, FULL_C
    # each generator imports the reference fresh with its own stub config -> run each in a subprocess
    if a.what == "all":
        import subprocess
        for w in ("small", "small_b8", "full", "full_c", "full_c4", "framework", "flava", "robustness", "fmnist", "a0"):
            subprocess.check_call([sys.executable, "-m", "oracle.gen_golden", "--what", w], cwd=REPO)
    elif a.what == "small":
        gen_mmbt("small_t16", SMALL, B=2, T=16, lens=[16, 9], seed=0)
    elif a.what == "small_b8":  # batch 8: BatchNorm statistics over 4x the values of the B = 2 fixtures
        gen_mmbt("small_b8", SMALL, B=8, T=16, lens=[16, 9, 16, 12, 5, 16, 14, 16], seed=2)
    elif a.what == "full":
        gen_mmbt("full_t508", FULL, B=2, T=508, lens=[508, 300], seed=1)
    elif a.what == "full_c":  # the conditioned trunk recipe (oracle/weights.py FULL_C)
        gen_mmbt("full_t508c", FULL_C, B=2, T=508, lens=[508, 300], seed=1)
    elif a.what == "full_c4":  # the same recipe at batch 4: another BatchNorm draw
        gen_mmbt("full_t508c_b4", FULL_C, B=4, T=508, lens=[508, 300, 451, 117], seed=3)
    elif a.what == "flava":
        from oracle.flava_ref import FlavaConfig
        for tag, (kw, B, Li, Lt, seed) in FLAVA_CASES.items():
            gen_flava(tag, FlavaConfig(**kw), B, Li, Lt, seed)
    elif a.what == "robustness":
        gen_robustness("small_t16", SMALL, B=3, T=16, lens=[16, 9, 12], n_repeats=3, seed=5)
        gen_robustness("full_t508", FULL, B=2, T=508, lens=[508, 301], n_repeats=2, seed=6)
    elif a.what == "fmnist":
        gen_fmnist()
    elif a.what == "a0":
        gen_a0()
    else:
        gen_framework()
