"""Poutyne-style training / evaluation loop -- the ``Model_`` API of the reference
src/framework.py (StepIterator :35-95, Model_ :98-354), kept call-compatible:

  Model_(model, optimizer, scheduler, data_forming_func, *, metrics=[], verbose=True)
  .to(device) / .to_device(x)
  .eval_loop(generator, phase, *, steps=None, auc=False, mmbt=False, vilt=False) -> {phase_loss, phase_<metric>...}
  .train_loop(train, test_generator=None, valid_generator=None, *, epochs, steps_per_epoch, validation_steps,
              test_steps, patience, callbacks, epoch_start, scheduler_step_on, auc, mmbt, vilt,
              freeze_img=, freeze_txt=, gradient_accumulation_steps=, scheduler_metric=)

Semantics reproduced on purpose (documented in DESIGN.md):
  * MMBT micro-batches zero the gradients FIRST (src/framework.py:281), so an
    optimizer step every `gradient_accumulation_steps` uses only the last
    micro-batch's gradient / accum;
  * the logged train loss is the loss after the division by accum;
  * freeze epochs: image trunk frozen while epoch < freeze_img, BERT encoder while epoch < freeze_txt;
  * early stop after `patience` epochs with train acc == 100, NaN loss stops training.
Difference: the per-batch loss and metric values reach the host in ONE transfer
(the reference syncs twice per micro-batch), which keeps the GPU queue fed.
"""
import itertools
import logging
import math
import timeit

import numpy as np
import torch

from .callbacks import CallbackList, ProgressionCallback, ValidationProgressionCallback

logger = logging.getLogger(__name__)

warning_settings = {"batch_size": "warn"}


def cycle(iterable):
    while True:
        yield from iterable


def _set_sampler_epoch(generator, epoch):
    """Reshuffle a DistributedSampler per epoch (the reference's single-process DataLoader
    reshuffles every epoch by itself; a DistributedSampler only does when told the epoch)."""
    sampler = getattr(generator, "sampler", None)
    if isinstance(sampler, torch.utils.data.DistributedSampler):
        sampler.set_epoch(epoch)


def _all_ranks_any(flag, device=None):
    """True on every rank when any rank's flag is True (no-op without torch.distributed)."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return bool(flag)
    if dist.get_backend() != "nccl":
        dev = torch.device("cpu")
    else:
        dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return bool(t.item())


class ShardSampler(torch.utils.data.Sampler):
    """Evaluation shard of one data-parallel rank: samples rank, rank + world, ... in order
    (no padding, so every sample is evaluated exactly once over the ranks)."""

    def __init__(self, data_source, world, rank):
        self.n, self.world, self.rank = len(data_source), world, rank

    def __iter__(self):
        return iter(range(self.rank, self.n, self.world))

    def __len__(self):
        return len(range(self.rank, self.n, self.world))


def shard_eval_loader(loader, world, rank):
    """The same evaluation loader over this rank's ShardSampler (DevicePrefetcher kept)."""
    inner = getattr(loader, "loader", loader)
    dl = torch.utils.data.DataLoader(inner.dataset, batch_size=inner.batch_size, shuffle=False,
                                     sampler=ShardSampler(inner.dataset, world, rank), num_workers=inner.num_workers,
                                     collate_fn=inner.collate_fn, pin_memory=inner.pin_memory)
    if inner is not loader:
        return type(loader)(dl, loader.device, loader.mean, loader.std, loader.dtype)
    return dl


def _combine_over_ranks(it, preds, labels, want_preds):
    """Sample-weighted loss / metric sums (and, for AUC, predictions) of the ranks' eval
    shards combined: the values a single process evaluating the whole split reports."""
    import torch.distributed as dist
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([it.losses_sum, it.sizes_sum] + list(it.metrics_sum), dtype=torch.float64, device=dev)
    dist.all_reduce(t)
    t = t.cpu().numpy()
    it.losses_sum, it.sizes_sum, it.metrics_sum = float(t[0]), float(t[1]), t[2:]
    if want_preds:
        parts = [None] * dist.get_world_size()
        dist.all_gather_object(parts, (preds, labels))
        preds = np.concatenate([p for p, _ in parts])
        labels = np.concatenate([lb for _, lb in parts])
    return preds, labels


def _get_step_iterator(steps, generator):
    if steps is None:
        return zip(itertools.count(1), generator)
    return zip(range(1, steps + 1), cycle(generator))


class StepIterator:
    """Iterates (step_dict, batch) pairs, firing batch hooks and keeping size-weighted sums.
    The consumer fills step_dict['loss'], ['metrics'], ['size'] (+ any extra keys)."""

    defaultfields = ("loss", "metrics", "number", "size")

    def __init__(self, generator, steps_per_epoch, callback, metrics_names):
        self.generator = generator
        self.steps_per_epoch = steps_per_epoch
        self.callback = callback
        self.metrics_names = metrics_names
        self.losses_sum = 0.0
        self.metrics_sum = np.zeros(len(metrics_names))
        self.sizes_sum = 0.0
        self.extra_lists = {}

    @property
    def loss(self):
        return self.losses_sum / self.sizes_sum if self.sizes_sum != 0 else 0

    @property
    def metrics(self):
        vals = self.metrics_sum / self.sizes_sum if self.sizes_sum != 0 else np.zeros(len(self.metrics_names))
        return dict(zip(self.metrics_names, vals))

    def __iter__(self):
        for number, data in _get_step_iterator(self.steps_per_epoch, self.generator):
            t0 = timeit.default_timer()
            self.callback.on_batch_begin(number, {})
            self.callback.on_forward_begin(number, data)
            step = {"number": number}
            yield step, data
            size = step["size"]
            self.losses_sum += step["loss"] * size
            self.metrics_sum += step["metrics"] * size
            self.sizes_sum += size
            for k, v in step.items():
                if k not in self.defaultfields:
                    self.extra_lists.setdefault(k, []).append(v)
            logs = {"batch": number, "size": size, "time": timeit.default_timer() - t0, "batch_begin_time": t0,
                    "loss": step["loss"], **dict(zip(self.metrics_names, step["metrics"]))}
            self.callback.on_batch_end(number, logs)


class Model_:
    def __init__(self, model, optimizer, scheduler, data_forming_func, *, metrics=[], verbose=True):
        self.model = model
        self.optimizer = optimizer
        self.scheduler = scheduler
        self.data_forming = data_forming_func
        self.metrics = metrics
        self.metrics_names = [m.__name__ for m in metrics]
        self.device = None
        self.verbose = verbose
        self.verbose_logs = {}
        self.shard_eval = False  # data parallel: eval loaders hold per-rank shards (train.py), combined here

    # ------------------------------------------------------------------ helpers
    def _metric_tensors(self, pred_y, y, eval, dummy_dim):
        return [m(pred_y, y, eval, dummy_dim) for m in self.metrics]

    def _compute_metrics(self, pred_y, y, eval, dummy_dim):
        return np.array([float(v) for v in self._metric_tensors(pred_y, y, eval, dummy_dim)])

    def _host_values(self, loss, metric_vals):
        """loss + metrics to host with one device->host copy."""
        vals = [loss.detach().reshape(()).float()] + [torch.as_tensor(v, device=loss.device).detach().reshape(()).float()
                                                    for v in metric_vals]
        host = torch.stack(vals).cpu().double().numpy()
        return float(host[0]), host[1:]

    def _transfer_optimizer_state_to_right_device(self):
        for group in self.optimizer.param_groups:
            for p in group["params"]:
                for v in self.optimizer.state.get(p, {}).values():
                    if torch.is_tensor(v) and v.device != p.device:
                        v.data = v.data.to(p.device)

    def to(self, device):
        self.device = device
        self.model.to(device)
        for m in self.metrics:
            if isinstance(m, torch.nn.Module):
                m.to(device)
        return self

    def to_device(self, x):
        if isinstance(x, tuple):
            return [t.to(self.device) for t in x]
        return x.to(self.device)

    def _prepare(self, batch, phase):
        x, y = batch
        x, y = self.data_forming(x, y, phase=phase)
        return self.to_device(x), self.to_device(y)

    # ------------------------------------------------------------------ evaluation
    def eval_loop(self, generator, phase, *, steps=None, auc=False, mmbt=False, vilt=False):
        if steps is None:
            steps = len(generator)
        progress = ValidationProgressionCallback(phase=phase, steps=steps, metrics_names=["loss"] + self.metrics_names)
        it = StepIterator(generator, steps, progress, self.metrics_names)
        self.model.eval()
        preds, labels = [], []
        with torch.no_grad():
            for step, batch in it:
                if vilt:
                    batch = {k: v.to(self.device) for k, v in batch.items()}
                    out = self.model(**batch)
                    loss, outputs, y = out.loss, out.logits, batch["labels"]
                else:
                    x, y = self._prepare(batch, "eval")
                    outputs = self.model(*x) if mmbt else self.model(x)
                    loss = self.model.compute_loss(outputs, y, eval=True)
                step["size"] = len(y)
                mvals = self._metric_tensors(outputs, y, True, not (vilt or mmbt))
                step["loss"], step["metrics"] = self._host_values(loss, mvals)
                preds.append(outputs if vilt else outputs.mean(1))
                labels.append(y)
        preds = torch.cat(preds, dim=0).cpu().numpy()
        labels = torch.cat(labels, dim=0).cpu().numpy()
        if self.shard_eval:  # data parallel: each rank evaluated its ShardSampler slice
            preds, labels = _combine_over_ranks(it, preds, labels, auc)
        out = {f"{phase}_loss": it.loss}
        out.update({f"{phase}_{k}": v for k, v in it.extra_lists.items()})
        out.update({f"{phase}_{k}": v for k, v in it.metrics.items()})
        if auc:
            from sklearn.metrics import roc_auc_score
            out[f"{phase}_auc"] = roc_auc_score(labels, preds[:, 1])
        return out

    # ------------------------------------------------------------------ training
    def _set_freeze(self, freeze_img, freeze_txt):
        enc = self.model.enc
        for p in enc.img_encoder.parameters():
            p.requires_grad = not freeze_img
        for p in enc.encoder.parameters():
            p.requires_grad = not freeze_txt

    def train_loop(self, train_generator, test_generator=None, valid_generator=None, *, epochs=1000,
                   steps_per_epoch=None, validation_steps=None, test_steps=None, patience=10, callbacks=[],
                   epoch_start=1, scheduler_step_on="epoch", auc=False, mmbt=False, vilt=False, **kwargs):
        self._transfer_optimizer_state_to_right_device()
        cbs = CallbackList(callbacks)
        cbs.append(ProgressionCallback())
        cbs.set_params({"epochs": epochs, "steps": steps_per_epoch})
        cbs.set_model_pytoune(self)
        accum = kwargs.get("gradient_accumulation_steps", 1)
        stop_training, stopped_epoch, counter, global_step = False, 0, 0, 0
        cbs.on_train_begin({})
        for epoch in range(epoch_start, epochs + 1):
            if mmbt:
                freeze_img = epoch < kwargs["freeze_img"]
                freeze_txt = epoch < kwargs["freeze_txt"]
            cbs.on_epoch_begin(epoch, {})
            _set_sampler_epoch(train_generator, epoch)
            t_epoch = timeit.default_timer()
            it = StepIterator(train_generator, steps_per_epoch, cbs, self.metrics_names)
            self.model.train(True)
            with torch.enable_grad():
                for step, batch in it:
                    if vilt:
                        batch = {k: v.to(self.device) for k, v in batch.items()}
                        y = batch["labels"]
                        self.optimizer.zero_grad()
                        out = self.model(**batch)
                        y_pred, loss = out.logits, out.loss
                    else:
                        x, y = self._prepare(batch, "train")
                        self.optimizer.zero_grad()
                        if mmbt:
                            self._set_freeze(freeze_img, freeze_txt)
                            y_pred = self.model(*x)
                        else:
                            y_pred = self.model(x)
                        loss = self.model.compute_loss(y_pred, y)
                    step["size"] = len(y)
                    if (mmbt or vilt) and kwargs["gradient_accumulation_steps"] > 1:
                        loss = loss / kwargs["gradient_accumulation_steps"]
                    loss.backward()
                    if mmbt or vilt:
                        global_step += 1
                        if global_step % accum == 0:
                            self.optimizer.step()
                            self.optimizer.zero_grad()
                    else:
                        self.optimizer.step()
                    with torch.no_grad():
                        mvals = self._metric_tensors(y_pred, y, False, not (vilt or mmbt))
                    cbs.on_backward_end(step["number"])
                    if scheduler_step_on == "batch":
                        self.scheduler.step()
                    step["loss"], step["metrics"] = self._host_values(loss, mvals)
                    if math.isnan(step["loss"]):
                        stop_training = True
            train_dict = {"loss": it.loss, **{f"train_{k}": v for k, v in it.extra_lists.items()}, **it.metrics}
            val_dict = self.eval_loop(valid_generator, "val", steps=validation_steps, auc=auc, mmbt=mmbt, vilt=vilt)
            test_dict = self.eval_loop(test_generator, "test", steps=test_steps, auc=auc, mmbt=mmbt, vilt=vilt)
            epoch_log = {"epoch": epoch, "time": timeit.default_timer() - t_epoch, "epoch_begin_time": t_epoch,
                         **train_dict, **val_dict, **test_dict}
            if scheduler_step_on == "epoch":
                self.scheduler.step(epoch_log[kwargs["scheduler_metric"]])
            cbs.on_epoch_end(epoch, epoch_log)
            if epoch_log["acc"] == 100:
                counter += 1
            if counter >= patience:
                stopped_epoch, stop_training = epoch, True
            # under DP each rank trains on its own shard: stop together or a rank that broke
            # out would leave the others blocked in the next gradient all-reduce
            stop_training = _all_ranks_any(stop_training, self.device)
            if stop_training and stopped_epoch == 0 and counter >= patience:
                stopped_epoch = epoch
            if stop_training:
                break
        cbs.on_train_end({})
        if stopped_epoch > 0:
            print("Epoch %05d: completed stopping" % stopped_epoch)
