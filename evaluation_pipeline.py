"""Pipelined evaluation entry point (reference: ``evaluation_pipeline.py``).

    python evaluation_pipeline.py --eval_lanes 4 --MODEL_NAME resnet18

read -> resize -> normalize -> predict run as HIP-stream stages on one GPU (the reference
needs >= 4 MPI ranks, one per stage); several GPUs split the test manifest and
SUM-reduce the accuracy.  Logs go to ``evaluation.log`` like the reference.
"""
import sys

from mpi_pytorch_amd.config import Config
from mpi_pytorch_amd.engine.eval_pipeline import run_pipeline


def pipeline(argv=None):
    cfg = Config.from_args(argv, log_file="evaluation.log")
    acc = run_pipeline(cfg)
    from mpi_pytorch_amd.parallel import shutdown
    shutdown()
    return acc


if __name__ == "__main__":
    pipeline(sys.argv[1:])
