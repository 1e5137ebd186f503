"""Default callbacks (history CSV, best/last/per-epoch checkpoints) and checkpoint
reloading -- the reference src/training_loop.py (:23-47, :50-69, :72-77)."""
import logging
import os
from functools import partial

import numpy as np
import pandas as pd
import torch

from .callbacks import LambdaCallback, ModelCheckpoint
from .utils import save_weights

logger = logging.getLogger(__name__)

_SCALARS = (int, float, complex, np.int64, np.int32, np.float32, np.float64, getattr(np, "float128", np.float64), str)
types_of_instance_to_save_in_csv = _SCALARS
types_of_instance_to_save_in_history = _SCALARS + (np.ndarray,)


def _append_to_history_csv(epoch, logs, H):
    for k, v in logs.items():
        H.setdefault(k, []).append(v)


def _save_history_csv(epoch, logs, save_path, H):
    logger.info("".join(f"{k}={v}\t" for k, v in logs.items() if isinstance(v, _SCALARS)))
    path = os.path.join(save_path, "history.csv")
    logger.info("Saving history to " + path)
    cols = {k: v for k, v in H.items() if isinstance(v[-1], _SCALARS)}
    pd.DataFrame(cols).to_csv(path, index=False)


def _construct_default_callbacks(model, optimizer, H, save_path, checkpoint_monitor):
    """history bookkeeping, history.csv, model_best_val.pt (max of `checkpoint_monitor`),
    model_epoch_{e}.pt and model_last_epoch.pt every epoch."""

    def save_epoch(epoch, logs):
        logger.info("Saving model from epoch " + str(epoch))
        save_weights(model, optimizer, os.path.join(save_path, f"model_epoch_{epoch}.pt"))
        save_weights(model, optimizer, os.path.join(save_path, "model_last_epoch.pt"))

    return [LambdaCallback(on_epoch_end=partial(_append_to_history_csv, H=H)),
            LambdaCallback(on_epoch_end=partial(_save_history_csv, save_path=save_path, H=H)),
            ModelCheckpoint(monitor=checkpoint_monitor, save_best_only=True, mode="max",
                            filepath=os.path.join(save_path, "model_best_val.pt")),
            LambdaCallback(on_epoch_end=save_epoch)]


def _load_pretrained_model(model, save_path):
    """Load checkpoint['model'] over the model's state dict, strict (tensor-only loader)."""
    checkpoint = torch.load(save_path, map_location="cpu", weights_only=True)
    state = model.state_dict()
    state.update(checkpoint["model"])
    model.load_state_dict(state, strict=True)
    logger.info("Done reloading!")
