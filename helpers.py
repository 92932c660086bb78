"""Reference-compatible checkpoint helpers (``helpers.py`` of the reference)."""
from mpi_pytorch_amd.checkpoint import save_checkpoint, load_checkpoint  # noqa: F401
