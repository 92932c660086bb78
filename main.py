"""Data-parallel training entry point (reference: ``main.py``).

    python main.py --MODEL_NAME resnet18 --NUM_EPOCHS 10          # 1 process
    python -m mpi_pytorch_amd.launch -n 8 main.py --DEBUG false  # 8 ranks, one per GPU
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 main.py

Every ``utils.py`` field of the reference is a flag (``--FIELD value``) or an environment
variable (``MPA_FIELD=value``); see ``mpi_pytorch_amd/config.py``.
"""
import sys

from mpi_pytorch_amd.config import Config
from mpi_pytorch_amd.engine.trainer import run_training


def main(argv=None):
    cfg = Config.from_args(argv)
    out = run_training(cfg)
    from mpi_pytorch_amd.parallel import shutdown
    shutdown()
    return out


if __name__ == "__main__":
    main(sys.argv[1:])
