#!/usr/bin/env python3
"""MMBT / FLAVA training entry point -- same command line as the reference train.py
(flags train.py:31-90, MMBT setup :132-162, FLAVA setup :184-216, resume :269-285,
callbacks :287-305, Model_.train_loop :312-330) on the MI355X HIP path.

Additions (all optional):
  --gin_file F [F ...] / --gin_param 'train.lr=5e-5'   gin-style bindings onto the flags (src/gin.py)
  --synthetic N      train on N seeded synthetic Food-101 samples (no dataset offline)
  data parallel      launch with torch.distributed.run: one rank per GPU, RCCL all-reduce,
                     train set sharded per rank, val/test sharded per rank (ShardSampler,
                     loss / metric sums combined over the ranks in Model_.eval_loop),
                     rank 0 writes history / checkpoints.
  --synthetic with --framework flava: seeded FLAVA embeddings (197 image + <= 77 text tokens)
--framework vilt is refused: the reference's setup_vilt needs the remote dandelin/vilt-b32-mlm
weights and ViltProcessor; the ViLT training step itself is src.vilt.ViltTrainHIP.
"""
import argparse
import logging
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import pandas as pd  # noqa: E402
import torch  # noqa: E402
import torch.optim as optim  # noqa: E402

from src import dataset  # noqa: E402
from src import gin  # noqa: E402
from src.framework import Model_, shard_eval_loader  # noqa: E402
from src.training_loop import _construct_default_callbacks  # noqa: E402
from src.utils import set_seed  # noqa: E402

logger = logging.getLogger(__name__)

# (flag, kwargs) -- the reference's flags, names and defaults unchanged
FLAGS = [
    ("--use_gpu", dict(action="store_true")), ("--device", dict(default=0, type=int)),
    ("--save_path", dict(type=str, required=True, help="Path to save the model")),
    ("--seed", dict(type=int, default=42)), ("--verbose", dict(action="store_true")),
    ("--resume", dict(action="store_true")),
    ("--batch_size", dict(type=int, default=128)), ("--lr", dict(type=float, default=0.1)),
    ("--n_epochs", dict(type=int, default=100)), ("--patience", dict(type=int, default=10)),
    ("--dataset", dict(type=str, choices=["food101", "hateful-meme-dataset"], default="hateful-meme-dataset")),
    ("--sample_size", dict(type=int, default=None)),
    ("--framework", dict(type=str, choices=["vilt", "flava", "mmbt"])),
    ("--model_type", dict(type=str, default="Vanilla", choices=["Vanilla", "MIMO-shuffle-instance", "MultiHead"])),
    ("--multimodal_num_attention_heads", dict(type=int, default=3)),
    ("--multimodal_num_hidden_layers", dict(type=int, default=3)),
    ("--clstoken", dict(action="store_true")), ("--dropout", dict(type=float, default=0)),
    ("--avg_pool", dict(action="store_true")), ("--wd", dict(type=int, default=0.001)),
    ("--lr_patience", dict(type=int, default=2)), ("--lr_factor", dict(type=float, default=0.5)),
    ("--gradient_accumulation_steps", dict(type=int, default=40)),
    ("--bert_model", dict(type=str, default="bert-base-uncased", choices=["bert-base-uncased", "bert-large-uncased"])),
    ("--drop_img_percent", dict(type=float, default=0.0)), ("--embed_sz", dict(type=int, default=300)),
    ("--freeze_img", dict(type=int, default=3)), ("--freeze_txt", dict(type=int, default=5)),
    ("--hidden", dict(nargs="*", type=int, default=[])), ("--hidden_sz", dict(type=int, default=768)),
    ("--img_embed_pool_type", dict(type=str, default="avg", choices=["max", "avg"])),
    ("--img_hidden_sz", dict(type=int, default=2048)), ("--include_bn", dict(type=int, default=True)),
    ("--max_seq_len", dict(type=int, default=512)), ("--n_workers", dict(type=int, default=0)),
    ("--sync_bn", dict(type=int, default=0, help="data parallel: the image trunk's BatchNorms normalise over the "
                                                 "whole batch of all ranks (the single-device reference's "
                                                 "statistics; src/dp.convert_sync_batchnorm)")),
    ("--gpu_normalize", dict(type=int, default=1, help="Food-101: workers ship uint8 crops, ToTensor + Normalize "
                                                      "run on the GPU one batch ahead (src/dataset.py)")),
    ("--num_image_embeds", dict(type=int, default=3)), ("--warmup", dict(type=float, default=0.1)),
    # build additions
    ("--gin_file", dict(nargs="*", default=[])), ("--gin_param", dict(nargs="*", default=[])),
    ("--synthetic", dict(type=int, default=0, help="N synthetic samples instead of $DATA_DIR/<dataset>")),
]


def get_args(parser):
    for flag, kw in FLAGS:
        parser.add_argument(flag, **kw)


def add_conditional_args(args):
    if args.synthetic:
        args.datapath = None
        args.labels = list(range(101))
    else:
        args.datapath = os.path.join(os.environ["DATA_DIR"], args.dataset)
    if args.dataset == "food101":
        if not args.synthetic:
            args.labels, _ = dataset.get_labels_and_frequencies(os.path.join(args.datapath, "train.jsonl"))
        args.n_classes, args.auc, args.error_cases_remover = len(args.labels), False, False
        args.name_extractor = lambda x: x.split(".")[0]
    else:
        args.labels, args.n_classes, args.auc, args.error_cases_remover = list(range(2)), 2, True, True
        args.name_extractor = lambda x: x.split("/")[-1].split(".")[0]
    if args.avg_pool:
        assert args.model_type != "Vanilla", "avg_pool is NOT supported for Vanilla model"
    return args


def acc(y_pred, y_true, eval, dummy_dim=False):
    """top-1 accuracy in percent (the metric train.py:119-130 hands to Model_)"""
    if dummy_dim:
        if not eval:
            y_pred, y_true = y_pred.view(-1, y_pred.shape[2]), y_true.view(-1)
        else:
            y_pred = y_pred.mean(1)
    return (y_pred.max(1)[1] == y_true).float().mean() * 100


def setup_mmbt(args):
    from src.mmbt import MultimodalBertClf
    from src.optim import BertAdam
    assert args.model_type == "Vanilla", "MMBT supports only Vanilla mode"
    model = MultimodalBertClf(args)
    named = list(model.named_parameters())
    no_decay = ["bias", "LayerNorm.bias", "LayerNorm.weight"]
    groups = [{"params": [p for n, p in named if not any(nd in n for nd in no_decay)], "weight_decay": 0.01},
              {"params": [p for n, p in named if any(nd in n for nd in no_decay)], "weight_decay": 0.0}]
    optimizer = BertAdam(groups, lr=args.lr, warmup=args.warmup, t_total=args.total_steps)
    scheduler = optim.lr_scheduler.ReduceLROnPlateau(optimizer, "max", patience=args.lr_patience,
                                                     factor=args.lr_factor)
    args.scheduler_metric, args.scheduler_step_on = "val_acc", "epoch"
    args.data_forming_func = lambda x, y, phase="train": (x, y)
    args.metrics = [acc]
    return args, model, optimizer, scheduler


def setup_flava(args, steps_per_epoch):
    """reference train.py:184-216: fusion transformer, AdamW, cosine schedule with warmup."""
    from functools import partial
    from transformers.optimization import get_cosine_schedule_with_warmup
    from src.model import FlavaFusionTransfomer, FlavaFusionTransfomerwithCLSToken
    model_cls = FlavaFusionTransfomerwithCLSToken if args.clstoken else FlavaFusionTransfomer
    model = model_cls(out_dim=1 if args.model_type == "Vanilla" else 2, num_classes=args.n_classes,
                      multimodal_num_attention_heads=args.multimodal_num_attention_heads,
                      multimodal_num_hidden_layers=args.multimodal_num_hidden_layers,
                      drop=args.dropout, avg_pool=args.avg_pool)
    optimizer = torch.optim.AdamW(model.parameters(), lr=args.lr, betas=(0.9, 0.98), eps=1.0e-9,
                                  weight_decay=args.wd)
    scheduler = get_cosine_schedule_with_warmup(optimizer, num_warmup_steps=steps_per_epoch * 3,
                                                num_training_steps=steps_per_epoch * args.n_epochs)
    args.scheduler_step_on, args.scheduler_metric = "batch", None
    args.data_forming_func = partial(dataset.data_forming_func_transformer, model_type=args.model_type)
    args.metrics = [acc]
    return args, model, optimizer, scheduler


def flava_data(args, rank=0, world=1):
    sampler = (lambda ds: torch.utils.data.DistributedSampler(ds, world, rank, shuffle=True, seed=args.seed)) \
        if world > 1 else None
    if args.synthetic:
        n = args.synthetic
        tr = dataset.SyntheticFlava(n, min_text=8, n_classes=args.n_classes, seed=1)
        va = dataset.SyntheticFlava(max(n // 8, args.batch_size), min_text=8, n_classes=args.n_classes, seed=2)
        te = dataset.SyntheticFlava(max(n // 8, args.batch_size), min_text=8, n_classes=args.n_classes, seed=3)
        return dataset.get_dataset(tr, va, te, dataset.collate_fn_flava, args, sampler)
    return dataset.get_dataset_flava(args, args.datapath, sampler)


def _dp_wrap_flat(model, optimizer):
    """DP for a model without the MMBT parameter store (FLAVA): one flat RCCL all-reduce
    (average) of every gradient before each optimizer step."""
    import torch.distributed as dist
    for p in model.parameters():
        dist.broadcast(p.data, 0)
    step = optimizer.step

    def dp_step(*a, **k):
        grads = [p.grad for p in model.parameters() if p.grad is not None]
        flat = torch._utils._flatten_dense_tensors(grads)
        dist.all_reduce(flat)
        flat.mul_(1.0 / dist.get_world_size())
        for g, f in zip(grads, torch._utils._unflatten_dense_tensors(flat, grads)):
            g.copy_(f)
        return step(*a, **k)
    optimizer.step = dp_step


def food101_data(args, rank=0, world=1):
    if args.synthetic:
        from src.testing import _Vocab
        T = args.max_seq_len - args.num_image_embeds - 1
        n = args.synthetic
        tr = dataset.SyntheticFood101(n, max_text=T, min_text=T // 2, seed=1)
        va = dataset.SyntheticFood101(max(n // 8, args.batch_size), max_text=T, min_text=T // 2, seed=2)
        te = dataset.SyntheticFood101(max(n // 8, args.batch_size), max_text=T, min_text=T // 2, seed=3)
        sampler = torch.utils.data.DistributedSampler(tr, world, rank, shuffle=True, seed=args.seed) \
            if world > 1 else None
        mk = lambda ds, shuf, smp=None: torch.utils.data.DataLoader(  # noqa: E731
            ds, batch_size=args.batch_size, shuffle=shuf and smp is None, sampler=smp, num_workers=args.n_workers,
            collate_fn=dataset.collate_fn, pin_memory=True)
        return mk(tr, True, sampler), mk(va, False), mk(te, False), 101, _Vocab()
    gpu = bool(args.gpu_normalize) and torch.cuda.is_available()
    # data parallel: every rank draws a disjoint shard of the train split (reshuffled per
    # epoch by Model_.train_loop); dev / test shards are cut in main() (shard_eval_loader)
    sampler = (lambda ds: torch.utils.data.DistributedSampler(ds, world, rank, shuffle=True, seed=args.seed)) \
        if world > 1 else None
    return dataset.get_food101(datapath=args.datapath, batch_size=args.batch_size,
                               drop_img_percent=args.drop_img_percent, max_seq_len=args.max_seq_len,
                               num_image_embeds=args.num_image_embeds, n_workers=args.n_workers,
                               gpu_normalize=gpu, device=torch.device("cuda", args.device) if gpu else None,
                               sampler=sampler)


def _dp_wrap(model, optimizer, accum, sync_bn=False):
    """Hook the RCCL bucketer between backward and BertAdam; all-reduce only on update micro-batches."""
    from src.dp import GradBucketer, broadcast_parameters, convert_sync_batchnorm, sync_buffers_on_eval
    broadcast_parameters(model)
    if sync_bn:
        convert_sync_batchnorm(model)
    sync_buffers_on_eval(model)  # BatchNorm running stats averaged over ranks before eval / checkpoints
    bucketer = GradBucketer(model, optimizer=optimizer)  # 1/world folded into BertAdam's step
    state = {"micro": 0}

    def count(mod, inp):
        if mod.training and torch.is_grad_enabled():
            bucketer.enabled = state["micro"] % accum == accum - 1
            state["micro"] += 1
    model.register_forward_pre_hook(count)
    step = optimizer.step

    def dp_step(*a, **k):
        bucketer.finish()
        return step(*a, **k)
    optimizer.step = dp_step
    return bucketer


def main(argv=None):
    parser = argparse.ArgumentParser(description="Train Models")
    get_args(parser)
    args, remaining = parser.parse_known_args(argv)
    assert remaining == [], remaining
    unused = gin.load(args, args.gin_file, args.gin_param)
    if unused:
        logger.warning("gin bindings not mapped to train.py flags: %s", sorted(unused))
    args = add_conditional_args(args)
    set_seed(args.seed)
    world, rank = int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        args.device = local
    print(args)
    if args.framework == "vilt":
        raise NotImplementedError("--framework vilt: the reference's setup_vilt loads dandelin/vilt-b32-mlm and its "
                                  "ViltProcessor data path (remote, not offline).  The ViLT training step itself is "
                                  "built: wrap a ViltForImagesAndTextClassification in src.vilt.ViltTrainHIP and "
                                  "pass it as the framework's model (Model_.train_loop(..., vilt=True))")
    if args.framework == "flava":
        train, valid, test = flava_data(args, rank, world)
        args, model, optimizer, scheduler = setup_flava(args, len(train))
    else:
        assert args.dataset == "food101", "MMBT is only supported for food101"
        train, valid, test, n_classes, vocab = food101_data(args, rank, world)
        args.n_classes, args.vocab = n_classes, vocab
        args.total_steps = len(train) / args.gradient_accumulation_steps * args.n_epochs
        args, model, optimizer, scheduler = setup_mmbt(args)
    mmbt = args.framework == "mmbt"
    os.makedirs(args.save_path, exist_ok=True)
    history_csv_path = os.path.join(args.save_path, "history.csv")
    if args.resume:
        ck = torch.load(os.path.join(args.save_path, "model_last_epoch.pt"), map_location="cpu", weights_only=True)
        model.load_state_dict(ck["model"])
        H = pd.read_csv(history_csv_path)
        H = {c: list(H[c].values) for c in H.columns if c != "Unnamed: 0"}
        epoch_start = len(H["epoch"]) + 1
    else:
        H = {}
        if rank == 0 and os.path.exists(history_csv_path):
            logger.info("Removing %s", history_csv_path)
            os.remove(history_csv_path)
        epoch_start = 1
    callbacks = _construct_default_callbacks(model, optimizer, H, args.save_path, checkpoint_monitor="val_acc") \
        if rank == 0 else []
    for c in callbacks:
        c.set_save_path(args.save_path)
        c.set_model(model, ignore=False)
        c.set_optimizer(optimizer)
    m = Model_(model=model, optimizer=optimizer, scheduler=scheduler, data_forming_func=args.data_forming_func,
               metrics=args.metrics, verbose=True)
    for c in callbacks:
        c.set_model_pytoune(m)
    if (args.use_gpu or world > 1) and torch.cuda.is_available():
        m.to(torch.device("cuda:{}".format(args.device)))
    elif not torch.cuda.is_available():
        raise RuntimeError("the MMBT / FLAVA paths run on MI355X HIP kernels: no GPU visible")
    if world > 1:
        if mmbt:
            _dp_wrap(model, optimizer, args.gradient_accumulation_steps, bool(getattr(args, "sync_bn", 0)))
        else:
            if getattr(args, "sync_bn", 0):
                raise SystemExit("--sync_bn (whole-batch BatchNorm under DP) is implemented for the MMBT trunk only")
            _dp_wrap_flat(model, optimizer)
        # evaluation sharded over the ranks, sample-weighted sums combined in eval_loop
        valid, test = (shard_eval_loader(dl, world, rank) for dl in (valid, test))
        m.shard_eval = True
    m.train_loop(train, valid_generator=valid, test_generator=test, steps_per_epoch=len(train),
                 validation_steps=len(valid), test_steps=len(test), epochs=args.n_epochs, callbacks=callbacks,
                 patience=args.patience, epoch_start=epoch_start, scheduler_step_on=args.scheduler_step_on,
                 auc=args.auc, vilt=False, mmbt=mmbt, freeze_img=args.freeze_img, freeze_txt=args.freeze_txt,
                 gradient_accumulation_steps=args.gradient_accumulation_steps,
                 scheduler_metric=args.scheduler_metric)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
