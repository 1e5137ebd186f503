"""Keras-style callback protocol of the reference training framework.

Same classes, hook names, setters and printed progress lines as the reference
src/callbacks.py (CallbackList :16-80, Callback :82-152, LambdaCallback :154-186,
ModelCheckpoint :188-254, ProgressionCallback :256-316,
ValidationProgressionCallback :318-356); hooks are dispatched generically.
"""
import itertools
import logging
import sys
import timeit

import numpy as np

from .utils import save_weights

logger = logging.getLogger(__name__)

# hook name -> True if its second argument is a logs dict that defaults to {}
HOOKS = {"on_epoch_begin": True, "on_epoch_end": True, "on_batch_begin": True, "on_batch_end": True,
         "on_train_begin": True, "on_train_end": True, "on_val_batch_end": True,
         "on_forward_begin": False, "on_backward_end": False}


def _noop(*args, **kwargs):
    return None


class Callback(object):
    """Base callback: every hook is a no-op; models/optimizer/paths are injected by setters."""

    def __init__(self):
        pass

    def __getattr__(self, name):
        if name in HOOKS:
            return _noop
        raise AttributeError(name)

    # setters
    def set_meta_data(self, meta_data):
        self.meta_data = meta_data

    def set_save_path(self, save_path):
        self.save_path = save_path

    def set_optimizer(self, optimizer):
        self.optimizer = optimizer

    def set_model(self, model, ignore=True):
        if not ignore:
            self.model = model

    def set_model_pytoune(self, model_pytoune):
        self.model_pytoune = model_pytoune

    def set_params(self, params):
        self.params = params

    def set_dataloader(self, data):
        self.data = data

    # getters
    def get_dataloader(self):
        return self.data

    def get_meta_data(self):
        return self.meta_dataset_model_pytoune

    def get_optimizer(self):
        return self.optimizer

    def get_params(self):
        return self.params

    def get_model(self):
        return self.model

    def get_save_path(self):
        return self.save_path


class CallbackList:
    """Broadcasts setters and hooks to every member, in order."""

    def __init__(self, callbacks=None):
        self.callbacks = list(callbacks or [])

    def append(self, callback):
        self.callbacks.append(callback)

    def __iter__(self):
        return iter(self.callbacks)

    def _broadcast(self, name, *args):
        for cb in self.callbacks:
            getattr(cb, name)(*args)

    def set_params(self, params):
        self._broadcast("set_params", params)

    def set_model(self, model):
        self._broadcast("set_model", model)

    def set_model_pytoune(self, model_pytoune):
        self._broadcast("set_model_pytoune", model_pytoune)

    def __getattr__(self, name):
        if name not in HOOKS:
            raise AttributeError(name)
        with_logs = HOOKS[name]

        def hook(first, second=None):
            if with_logs:
                second = second or {}
                self._broadcast(name, first, second)
            elif name == "on_forward_begin":
                self._broadcast(name, first, second)
            else:
                self._broadcast(name, first)

        def hook1(logs=None):  # on_train_begin / on_train_end take logs only
            self._broadcast(name, logs or {})

        return hook1 if name in ("on_train_begin", "on_train_end") else hook


class LambdaCallback(Callback):
    """Callback built from plain functions (keyword per hook; missing ones are no-ops)."""

    def __init__(self, on_epoch_begin=None, on_epoch_end=None, on_batch_begin=None, on_batch_end=None,
                 on_train_begin=None, on_train_end=None):
        super().__init__()
        given = dict(on_epoch_begin=on_epoch_begin, on_epoch_end=on_epoch_end, on_batch_begin=on_batch_begin,
                     on_batch_end=on_batch_end, on_train_begin=on_train_begin, on_train_end=on_train_end)
        for name, fn in given.items():
            setattr(self, name, fn if fn is not None else _noop)


class ModelCheckpoint(Callback):
    """Saves {'model','optimizer'} state dicts every `period` epochs, or only on improvement of `monitor`."""

    def __init__(self, filepath, monitor="val_loss", verbose=0, save_best_only=False, mode="auto", period=1):
        super().__init__()
        self.filepath, self.monitor, self.verbose = filepath, monitor, verbose
        self.save_best_only, self.period = save_best_only, period
        self.epochs_since_last_save = 0
        if mode not in ("auto", "min", "max"):
            mode = "auto"
        maximize = mode == "max" or (mode == "auto" and ("acc" in monitor or monitor.startswith("fmeasure")))
        self.monitor_op = np.greater if maximize else np.less
        self.best = -np.inf if maximize else np.inf

    def __getstate__(self):
        state = dict(self.__dict__)
        state.pop("model", None)
        state.pop("optimizer", None)
        return state

    def __setstate__(self, newstate):
        newstate["model"] = getattr(self, "model", None)
        newstate["optimizer"] = getattr(self, "optimizer", None)
        self.__dict__.update(newstate)

    def on_epoch_end(self, epoch, logs=None):
        logs = logs or {}
        self.epochs_since_last_save += 1
        if self.epochs_since_last_save < self.period:
            return
        self.epochs_since_last_save = 0
        if not self.save_best_only:
            if self.verbose > 0:  # the reference only writes in verbose mode here (src/callbacks.py:251-254)
                print("Epoch %05d: saving model to %s" % (epoch, self.filepath))
                save_weights(self.model, self.optimizer, self.filepath)
            return
        current = logs.get(self.monitor)
        if current is None:
            logging.warning("Can save best model only with %s available, skipping." % self.monitor)
            return
        if self.monitor_op(current, self.best):
            if self.verbose > 0:
                print("Epoch %05d: %s improved from %0.5f to %0.5f, saving model to %s"
                      % (epoch, self.monitor, self.best, current, self.filepath))
            self.best = current
            save_weights(self.model, self.optimizer, self.filepath)
        elif self.verbose > 0:
            print("Epoch %05d: %s did not improve" % (epoch, self.monitor))


def _fmt(pairs):
    return ", ".join("{}: {:f}".format(k, v) for k, v in pairs)


class ProgressionCallback(Callback):
    """Per-batch ETA line and per-epoch summary on stdout."""

    def __init__(self, other_metrics=[]):
        self.other_metrics = list(other_metrics)

    def on_train_begin(self, logs):
        self.metrics = ["loss"] + self.model_pytoune.metrics_names
        self.epochs, self.steps = self.params["epochs"], self.params["steps"]

    def on_epoch_begin(self, epoch, logs):
        self.step_times_sum = 0.0
        self.epoch = epoch
        sys.stdout.write("\rEpoch %d/%d" % (self.epoch, self.epochs))
        sys.stdout.flush()

    def _metrics_str(self, logs):
        train = ((k, logs[k]) for k in self.metrics if logs.get(k) is not None)
        val = (("val_" + k, logs["val_" + k]) for k in self.metrics if logs.get("val_" + k) is not None)
        return _fmt(itertools.chain(train, val))

    def _other_str(self, logs):
        return _fmt((k, logs[k]) for k in self.other_metrics if logs.get(k) is not None)

    def on_epoch_end(self, epoch, logs):
        last = self.steps if self.steps is not None else self.last_step
        print("\rEpoch %d/%d %.2fs/%.2fs: Step %d/%d: %s. %s" % (
            self.epoch, self.epochs, logs["time"], timeit.default_timer() - logs["epoch_begin_time"], last, last,
            self._metrics_str(logs), self._other_str(logs)))

    def on_batch_end(self, batch, logs):
        self.step_times_sum += timeit.default_timer() - logs["batch_begin_time"]
        ms, other = self._metrics_str(logs), self._other_str(logs)
        mean = self.step_times_sum / batch
        if self.steps is not None:
            sys.stdout.write("\rEpoch %d/%d ETA %.2fs Step %d/%d: %s. %s" % (
                self.epoch, self.epochs, mean * (self.steps - batch), batch, self.steps, ms, other))
            if "cumsum_iol" in other:
                sys.stdout.write("\n")
        else:
            sys.stdout.write("\rEpoch %d/%d %.2fs/step Step %d: %s. %s" % (self.epoch, self.epochs, mean, batch, ms,
                                                                          other))
            self.last_step = batch
        sys.stdout.flush()


class ValidationProgressionCallback(Callback):
    """ETA line of an evaluation phase (val / test)."""

    def __init__(self, phase, metrics_names, steps=None):
        self.params = {"steps": steps, "phase": phase}
        self.metrics = metrics_names
        super().__init__()

    def on_batch_begin(self, batch, logs):
        if batch == 1:
            self.step_times_sum = 0.0
        self.steps = self.params["steps"]

    def on_batch_end(self, batch, logs):
        self.step_times_sum += timeit.default_timer() - logs["batch_begin_time"]
        phase = self.params["phase"]
        ms = _fmt((phase + "_" + k, logs[k]) for k in self.metrics if logs.get(k) is not None)
        mean = self.step_times_sum / batch
        if self.steps is not None:
            sys.stdout.write("\r%s ETA %.2fs Step %d/%d: %s." % (phase, mean * (self.steps - batch), batch,
                                                               self.steps, ms))
        else:
            sys.stdout.write("\r%s %.2fs/step Step %d: %s." % (phase, mean, batch, ms))
            self.last_step = batch
        sys.stdout.flush()
