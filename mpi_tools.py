"""Reference-compatible communication helpers (``mpi_tools.py`` of the reference), backed by
torch.distributed (RCCL over xGMI on MI355X, gloo on CPU)."""
from mpi_pytorch_amd.parallel.comm import (num_processes, mpi_all_reduce, mpi_sum,  # noqa: F401
                                           mpi_avg_grads, mpi_broadcast, sync_params)
