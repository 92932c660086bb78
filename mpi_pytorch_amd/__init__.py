"""mpi_pytorch_amd - an MI355X-native data-parallel CNN training / inference engine with
the capabilities of erick093/MPI_Pytorch.

Layers (bottom -> top): ``csrc/`` HIP/CDNA4 kernels + C++ runtime (``_C``), ``ops`` autograd
layer, ``parallel`` (process group, flat arena, bucketed RCCL all-reduce), ``models``
(torchvision-named zoo), ``data``, ``engine`` (trainer, HIP-stream eval pipeline),
``checkpoint``, ``config``.
"""
__version__ = "0.1.0"

from .config import Config  # noqa: F401
