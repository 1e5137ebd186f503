"""MI355X-native MMBT hot path (drop-in for the reference's ``src`` package API).

Put ``multi-modal-uncertainty_amd/`` on PYTHONPATH and ``from src.framework import
Model_``, ``from src.mmbt import MultimodalBertClf`` etc. resolve to this build.
Unlike the reference ``src/__init__.py:1-16`` no plotting/Keras side effects run
at import; the DATA_DIR / RESULTS_DIR defaults are kept.
"""
import os

DATA_DIR = os.environ.get("DATA_DIR", os.path.join(os.path.dirname(__file__), "data"))
RESULTS_DIR = os.environ.get("RESULTS_DIR", os.path.join(os.path.dirname(__file__), "results"))
