"""Reference-compatible model factory (``models.py`` of the reference)."""
from mpi_pytorch_amd.models import initialize_model, set_parameter_requires_grad  # noqa: F401
