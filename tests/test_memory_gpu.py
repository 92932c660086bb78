"""Device-memory reservation (engine.reserve_device_memory, docs/NOTES.md "Slow processes"):
one up-front caching-allocator segment that later tensors are carved from, so a run does not
hipMalloc while a previous process's memory is still being reclaimed."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_reserve_device_memory_serves_later_tensors():
    from mpi_pytorch_amd.engine import reserve_device_memory
    dev = torch.device("cuda", 0)
    torch.cuda.empty_cache()
    got = reserve_device_memory(dev, 2.0)
    assert 1.9 <= got <= 2.0
    n0 = torch.cuda.memory_stats(dev)["num_device_alloc"]
    ts = [torch.empty(64 << 20, dtype=torch.uint8, device=dev) for _ in range(8)]
    assert torch.cuda.memory_stats(dev)["num_device_alloc"] == n0  # carved from the segment
    del ts
    torch.cuda.empty_cache()
    assert reserve_device_memory(dev, 0.0) == 0.0
    assert reserve_device_memory(torch.device("cpu"), 2.0) == 0.0
