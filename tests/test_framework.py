"""CPU: the build's Model_ / callbacks / training_loop reproduce the reference loop.

tests/golden/framework_tiny.json was written by the reference src/framework.py
(oracle/gen_golden.py --what framework) driving oracle/tiny_model.TinyMMBT for 2
epochs x 3 steps with freeze schedule, accum=2, SGD + ReduceLROnPlateau and the
default callbacks.  The same run through this build must give the same history,
files, checkpoint layout and final weights.
"""
import json
import os
import tempfile

import numpy as np
import pandas as pd
import pytest
import torch

GOLD = os.path.join(os.path.dirname(__file__), "golden")
TIMING = {"time", "epoch_begin_time"}


def run_build_loop(d, epochs=2, **kw):
    from oracle.tiny_model import TinyMMBT, tiny_batches, acc
    from src import framework, training_loop
    model = TinyMMBT()
    opt = torch.optim.SGD(model.parameters(), lr=0.05, momentum=0.9)
    sched = torch.optim.lr_scheduler.ReduceLROnPlateau(opt, "max", patience=0, factor=0.5)
    train, val, test = tiny_batches(3, seed=1), tiny_batches(2, seed=2), tiny_batches(2, seed=3)
    H = {}
    cbs = training_loop._construct_default_callbacks(model, opt, H, d, checkpoint_monitor="val_acc")
    for c in cbs:
        c.set_save_path(d)
        c.set_model(model, ignore=False)
        c.set_optimizer(opt)
    m = framework.Model_(model=model, optimizer=opt, scheduler=sched,
                         data_forming_func=lambda x, y, phase="train": (x, y), metrics=[acc])
    for c in cbs:
        c.set_model_pytoune(m)
    args = dict(valid_generator=val, test_generator=test, steps_per_epoch=len(train), validation_steps=len(val),
                test_steps=len(test), epochs=epochs, callbacks=cbs, patience=10, epoch_start=1,
                scheduler_step_on="epoch", auc=False, vilt=False, mmbt=True, freeze_img=2, freeze_txt=3,
                gradient_accumulation_steps=2, scheduler_metric="val_acc")
    args.update(kw)
    m.train_loop(train, **args)
    return model, opt, H


def test_train_loop_matches_reference_history():
    ref = json.load(open(os.path.join(GOLD, "framework_tiny.json")))
    with tempfile.TemporaryDirectory() as d:
        model, opt, H = run_build_loop(d)
        files = sorted(os.listdir(d))
        ck = torch.load(os.path.join(d, "model_last_epoch.pt"), weights_only=True)
        csv_cols = list(pd.read_csv(os.path.join(d, "history.csv")).columns)
    assert files == ref["files"]
    assert sorted(ck.keys()) == ref["ckpt_keys"]
    assert list(ck["model"].keys()) == ref["model_keys"]
    assert sorted(ck["optimizer"].keys()) == ref["optimizer_state_keys"]
    assert csv_cols == ref["csv_columns"]
    assert list(H.keys()) == list(ref["history"].keys())
    for k, vals in ref["history"].items():
        if k in TIMING:
            continue
        np.testing.assert_allclose(np.array(H[k], dtype=float), np.array(vals, dtype=float), rtol=1e-6, atol=1e-7,
                                   err_msg=k)
    for k, v in ref["final_params"].items():
        np.testing.assert_allclose(model.state_dict()[k].numpy(), np.array(v), rtol=1e-5, atol=1e-6, err_msg=k)


def test_eval_loop_keys_and_weighting():
    from oracle.tiny_model import TinyMMBT, tiny_batches, acc
    from src.framework import Model_
    model = TinyMMBT()
    m = Model_(model, None, None, lambda x, y, phase="train": (x, y), metrics=[acc])
    batches = tiny_batches(3, bsz=4, seed=9)
    out = m.eval_loop(batches, "val", mmbt=True)
    assert list(out.keys()) == ["val_loss", "val_acc"]
    tot, n = 0.0, 0
    with torch.no_grad():
        for x, y in batches:
            tot += float(model.compute_loss(model(*x), y)) * len(y)
            n += len(y)
    assert abs(out["val_loss"] - tot / n) < 1e-6


def test_nan_loss_stops_training():
    from oracle.tiny_model import TinyMMBT
    with tempfile.TemporaryDirectory() as d:
        orig = TinyMMBT.compute_loss
        TinyMMBT.compute_loss = lambda self, y_hat, y, eval=False: orig(self, y_hat, y) * float("nan")
        try:
            _, _, H = run_build_loop(d, epochs=3)
        finally:
            TinyMMBT.compute_loss = orig
    assert H["epoch"] == [1]


def test_load_pretrained_model_roundtrip():
    from oracle.tiny_model import TinyMMBT
    from src.training_loop import _load_pretrained_model
    from src.utils import save_weights
    a, b = TinyMMBT(seed=1), TinyMMBT(seed=2)
    opt = torch.optim.SGD(a.parameters(), lr=0.1)
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "ck.pt")
        save_weights(a, opt, p)
        _load_pretrained_model(b, p)
    for k, v in a.state_dict().items():
        assert torch.equal(v, b.state_dict()[k])


def test_callbacks_protocol():
    from src.callbacks import Callback, CallbackList, LambdaCallback, ModelCheckpoint
    seen = []

    class Rec(Callback):
        def on_batch_end(self, batch, logs):
            seen.append(("be", batch, dict(logs)))

        def on_forward_begin(self, batch, data):
            seen.append(("fb", batch, data))

        def on_backward_end(self, batch):
            seen.append(("bwe", batch))

    cl = CallbackList([Rec(), LambdaCallback(on_epoch_end=lambda e, logs: seen.append(("ee", e)))])
    cl.on_train_begin()
    cl.on_batch_begin(1)
    cl.on_forward_begin(1, "x")
    cl.on_backward_end(1)
    cl.on_batch_end(1, {"loss": 1.0})
    cl.on_epoch_end(3)
    cl.on_train_end({})
    assert seen == [("fb", 1, "x"), ("bwe", 1), ("be", 1, {"loss": 1.0}), ("ee", 3)]
    mc = ModelCheckpoint("x.pt", monitor="val_acc")
    assert mc.monitor_op is np.greater and mc.best == -np.inf
    mc = ModelCheckpoint("x.pt", monitor="val_loss")
    assert mc.monitor_op is np.less and mc.best == np.inf
