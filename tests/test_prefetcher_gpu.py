"""DevicePrefetcher on the GPU: the one-batch lookahead (H2D copy + preprocess of batch i+1
issued on the copy stream during step i) yields exactly the batches of the in-order path,
also when the consumer overwrites the previous batch while the next one is being prepared."""
import pytest
import torch

from mpi_pytorch_amd.data import DevicePrefetcher

pytestmark = pytest.mark.gpu


def _take(pf, n, clobber):
    out = []
    for _ in range(n):
        x, y = pf.next()
        out.append((x.clone(), y.clone()))
        if clobber:  # a consumer that reuses its input buffer on the compute stream
            x.fill_(0)
            y.fill_(-1)
    return out


@pytest.mark.parametrize("depth", [2, 4])
def test_lookahead_matches_in_order(gpu, depth):
    kw = dict(seed=7, depth=depth, threads=1)
    ref = DevicePrefetcher(gpu, 6, (40, 40), (32, 32), 1000, lookahead=False, **kw)
    la = DevicePrefetcher(gpu, 6, (40, 40), (32, 32), 1000, lookahead=True, **kw)
    try:
        a = _take(ref, 5, clobber=False)
        b = _take(la, 5, clobber=True)
    finally:
        ref.close()
        la.close()
    torch.cuda.synchronize()
    for (xa, ya), (xb, yb) in zip(a, b):
        assert xa.shape == xb.shape and xa.dtype == xb.dtype
        assert torch.equal(ya, yb)
        assert torch.equal(xa, xb)
    assert not torch.equal(a[0][0], a[1][0])  # distinct batches
