"""Offline dataset sampling entry point (reference: ``create_dataset.py``)."""
import sys

from mpi_pytorch_amd.data.create_dataset import main

if __name__ == "__main__":
    main(sys.argv[1:])
