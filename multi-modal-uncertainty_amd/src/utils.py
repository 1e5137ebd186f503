"""Seeding, checkpoint writing and tensor-tree helpers used by the training path
(reference src/utils.py: set_seed :14-21, torch_to :89-90, save_weights :98-106,
numpy_seed :167-181, configure_logger :122-165)."""
import logging
import random
import sys
from contextlib import contextmanager

import numpy as np
import torch

logger = logging.getLogger(__name__)


def set_seed(seed):
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)
    torch.backends.cudnn.deterministic = True
    torch.backends.cudnn.benchmark = False


def _map(obj, fn):
    if isinstance(obj, (list, tuple)):
        return type(obj)(_map(o, fn) for o in obj)
    if isinstance(obj, dict):
        return {k: _map(v, fn) for k, v in obj.items()}
    return fn(obj)


def torch_apply(obj, func):
    return _map(obj, lambda t: func(t) if torch.is_tensor(t) else t)


def torch_to(obj, *args, **kwargs):
    return torch_apply(obj, lambda t: t.to(*args, **kwargs))


def numpy_to_torch(obj):
    return _map(obj, lambda a: torch.from_numpy(a) if isinstance(a, np.ndarray) else a)


def torch_to_numpy(obj, copy=False):
    return torch_apply(obj, (lambda t: t.cpu().detach().numpy().copy()) if copy else (lambda t: t.cpu().detach().numpy()))


def save_weights(model, optimizer, filename):
    """Checkpoint format of the reference: {'model': state_dict, 'optimizer': state_dict}."""
    torch.save({"model": model.state_dict(), "optimizer": optimizer.state_dict()}, filename)


@contextmanager
def numpy_seed(seed, *addl_seeds):
    """Seed numpy's global RNG inside the block and restore its state afterwards."""
    if seed is None:
        yield
        return
    if addl_seeds:
        seed = int(hash((seed, *addl_seeds)) % 1e6)
    saved = np.random.get_state()
    np.random.seed(seed)
    try:
        yield
    finally:
        np.random.set_state(saved)


def configure_logger(name="", console_logging_level=logging.INFO, file_logging_level=None, log_file=None):
    lg = logging.getLogger(name)
    if lg.handlers or (console_logging_level is None and file_logging_level is None):
        return None
    lg.setLevel(logging.DEBUG)
    fmt = logging.Formatter("%(asctime)s - %(name)s - %(levelname)s - %(message)s")
    if console_logging_level is not None:
        h = logging.StreamHandler(sys.stdout)
        h.setFormatter(fmt)
        h.setLevel(console_logging_level)
        lg.addHandler(h)
    if file_logging_level is not None:
        if log_file is None:
            raise ValueError("If file logging enabled, log_file path is required")
        import logging.handlers
        fh = logging.handlers.RotatingFileHandler(log_file, maxBytes=5 * 1048576, backupCount=7)
        fh.setFormatter(fmt)
        lg.addHandler(fh)
    return lg
