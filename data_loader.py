"""Reference-compatible dataset class (``data_loader.py`` of the reference)."""
from mpi_pytorch_amd.data.dataset import GetData  # noqa: F401
