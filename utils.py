"""Reference-compatible constants module (``utils.py`` of the reference).

Values come from :class:`mpi_pytorch_amd.config.Config` defaults + ``MPA_*`` environment
overrides, so ``import utils; utils.MODEL_NAME`` keeps working for reference users.
"""
from mpi_pytorch_amd.config import Config as _Config

_cfg = _Config.from_env()
globals().update({k: v for k, v in _cfg.to_dict().items() if k.isupper()})
CONFIG = _cfg
