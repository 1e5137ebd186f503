"""Minimal torchvision stand-in for oracle/gen_golden.py (see ../README.md)."""
from . import models  # noqa: F401
