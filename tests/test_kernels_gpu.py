"""Numerics of every native gfx950 kernel against the plain-PyTorch fp32 oracle
(``mpi_pytorch_amd/ops/ref.py``) on identical bf16 inputs."""
import math

import pytest
import torch

from mpi_pytorch_amd.ops import ref

pytestmark = pytest.mark.gpu


def C():
    from mpi_pytorch_amd.ops import _ext
    return _ext.ext()


def rel(a, b):
    a = a.float()
    b = b.float()
    return float((a - b).abs().max() / (b.abs().max() + 1e-6))


def bf(*shape, dev, scale=1.0):
    return (torch.randn(*shape, device=dev) * scale).to(torch.bfloat16)


CONV_CASES = [
    # N, H, W, C, K, R, S, stride, pad
    (2, 32, 32, 3, 64, 7, 7, 2, 3),       # stem (C=3 scalar path)
    (2, 14, 14, 64, 64, 3, 3, 1, 1),
    (2, 14, 14, 64, 128, 3, 3, 2, 1),
    (2, 14, 14, 64, 128, 1, 1, 2, 0),      # downsample
    (3, 9, 11, 96, 48, 3, 3, 1, 1),        # odd spatial, BN=64 tile
    (2, 12, 12, 32, 32, 1, 7, 1, (0, 3)),  # asymmetric 1x7
    (2, 12, 12, 40, 24, 7, 1, 1, (3, 0)),  # asymmetric 7x1, BN=32 tile, C%8==0
    (2, 17, 17, 64, 200, 3, 3, 2, 0),      # K not multiple of tile, stride 2 no pad
    (2, 8, 8, 256, 512, 3, 3, 1, 1),       # deep K (split-K candidate)
    (1, 13, 13, 12, 20, 5, 5, 1, 2),       # C%8 != 0 (VW=4)
    (2, 20, 20, 16, 64, 11, 11, 4, 2),     # AlexNet-style 11x11 s4
    (2, 7, 7, 512, 512, 3, 3, 1, 1),       # small M, deep K: split-K + stats + shift path
    (8, 56, 56, 64, 64, 3, 3, 1, 1),       # large pixel count: wgrad split slab path
    (2, 32, 32, 8, 64, 7, 7, 2, 3),        # padded stem (C=8: 16-B granular, DMA path)
    (4, 28, 28, 128, 128, 3, 3, 1, 1),     # 128x128 tile, several K-tiles
    (8, 40, 40, 3, 5, 3, 3, 1, 1),         # split wgrad, Kout*R*S*C % 4 != 0 (scalar reduce)
    (2, 17, 17, 48, 64, 5, 5, 1, 2),       # Inception 5x5_2: C = 48, padded-K uniform taps
    (2, 15, 13, 80, 192, 3, 3, 1, 0),      # Inception Conv2d_4a: C = 80, valid 3x3
]


def _pair(v):
    return v if isinstance(v, tuple) else (v, v)


@pytest.fixture(autouse=True)
def _halo_off(gpu):
    """The halo-staged 3x3 kernel (conv_halo.hip) sums K in a different order than the
    implicit-GEMM engines; it runs only where a test enables it (engine "dma-halo",
    test_conv_halo_*), so the bitwise cross-engine checks compare like with like."""
    C().igemm_set_halo(0)
    yield
    C().igemm_set_halo(1)


@pytest.fixture(params=[(2, 1, 1), (2, 1, 0), (2, 0, 0), (0, 1, 0)],
                ids=["dma-halo", "dma", "dma-generic", "reg"])
def engine(request, gpu):
    """Run a GEMM test on the LDS-DMA engine (with and without the halo-staged 3x3/s1
    kernel; uniform-tap fast path and generic gather) and on the register-staged engine."""
    prev = C().igemm_engine()
    eng, uni, halo = request.param
    C().igemm_set_engine(eng)
    C().igemm_set_dma_uni(uni)
    C().igemm_set_halo(halo)
    yield eng
    C().igemm_set_engine(prev)
    C().igemm_set_dma_uni(1)
    C().igemm_set_halo(0)


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_fwd(gpu, engine, case):
    torch.manual_seed(0)
    N, H, W, Cc, K, R, S, st, pd = case
    ph, pw = _pair(pd)
    x = bf(N, H, W, Cc, dev=gpu)
    w = bf(K, R, S, Cc, dev=gpu, scale=1.0 / math.sqrt(R * S * Cc))
    b = torch.randn(K, device=gpu)
    st_c = torch.zeros(2, K, device=gpu)
    st_r = torch.zeros(2, K, device=gpu)
    shift = torch.randn(K, device=gpu) * 0.1
    y = C().conv_fwd(x, w, b, st, st, ph, pw, True, st_c, shift)
    yr = ref.conv_fwd(x, w, b, st, st, ph, pw, True, st_r, shift)
    torch.cuda.synchronize()
    assert y.shape == yr.shape
    assert rel(y, yr) < 2e-2
    assert rel(st_c, st_r) < 2e-2


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_dgrad(gpu, engine, case):
    torch.manual_seed(1)
    N, H, W, Cc, K, R, S, st, pd = case
    ph, pw = _pair(pd)
    P = (H + 2 * ph - R) // st + 1
    Q = (W + 2 * pw - S) // st + 1
    dy = bf(N, P, Q, K, dev=gpu)
    w = bf(K, R, S, Cc, dev=gpu, scale=1.0 / math.sqrt(R * S * K))
    dx = C().conv_dgrad(dy, w, H, W, st, st, ph, pw)
    dxr = ref.conv_dgrad(dy, w, H, W, st, st, ph, pw)
    torch.cuda.synchronize()
    assert rel(dx, dxr) < 2e-2


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_dgrad_accumulate(gpu, engine, case):
    """dgrad accumulated into an existing gradient (GradJoin: residual-block inputs):
    dx = acc + dgrad in the epilogue, on every engine, split-K and stride-phase layout
    (including the 1x1/s2 downsample whose tap-less phases must keep `acc` untouched)."""
    torch.manual_seed(2)
    N, H, W, Cc, K, R, S, st, pd = case
    ph, pw = _pair(pd)
    P = (H + 2 * ph - R) // st + 1
    Q = (W + 2 * pw - S) // st + 1
    dy = bf(N, P, Q, K, dev=gpu)
    w = bf(K, R, S, Cc, dev=gpu, scale=1.0 / math.sqrt(R * S * K))
    acc0 = bf(N, H, W, Cc, dev=gpu)
    acc = acc0.clone()
    out = C().conv_dgrad(dy, w, H, W, st, st, ph, pw, None, acc)
    exp = acc0.float() + ref.conv_dgrad(dy, w, H, W, st, st, ph, pw).float()
    torch.cuda.synchronize()
    assert out.data_ptr() == acc.data_ptr()
    assert rel(out, exp) < 2e-2
    if Cc % 8 == 0 and K % 8 == 0:  # transposed-weight (K-contiguous B) path too
        wt = w.permute(3, 1, 2, 0).reshape(Cc, R * S, K).contiguous()
        acc2 = acc0.clone()
        C().conv_dgrad(dy, w, H, W, st, st, ph, pw, wt, acc2)
        torch.cuda.synchronize()
        if C().igemm_halo_enabled():  # 3x3/s1 from wt runs on the halo kernel: other K order
            assert rel(acc2, out) < 1e-2
        else:
            assert torch.equal(acc2, out)


@pytest.mark.parametrize("case", [c for c in CONV_CASES if c[3] % 8 == 0 and c[4] % 8 == 0])
def test_conv_dgrad_transposed_weight(gpu, engine, case):
    """dgrad from the transposed weight copy [C][R*S][K] (K-contiguous B, weight-tap row
    map) feeds the MFMAs the same fragments in the same K order as the N-contiguous path:
    bitwise equal, on every engine and stride-phase layout."""
    torch.manual_seed(1)
    N, H, W, Cc, K, R, S, st, pd = case
    ph, pw = _pair(pd)
    P = (H + 2 * ph - R) // st + 1
    Q = (W + 2 * pw - S) // st + 1
    dy = bf(N, P, Q, K, dev=gpu)
    w = bf(K, R, S, Cc, dev=gpu, scale=1.0 / math.sqrt(R * S * K))
    wt = w.permute(3, 1, 2, 0).reshape(Cc, R * S, K).contiguous()
    dx = C().conv_dgrad(dy, w, H, W, st, st, ph, pw)
    dxt = C().conv_dgrad(dy, w, H, W, st, st, ph, pw, wt)
    torch.cuda.synchronize()
    if C().igemm_halo_enabled():
        assert rel(dxt, dx) < 1e-2
    else:
        assert torch.equal(dx, dxt), rel(dxt, dx)


@pytest.mark.parametrize("case", [(2, 14, 14, 64, 128), (4, 28, 28, 128, 256), (3, 15, 13, 64, 64),
                                  (2, 56, 56, 64, 128)])
def test_conv_dgrad_pair(gpu, case):
    """A residual stage's 3x3/s2 conv1 dgrad and its 1x1/s2 shortcut dgrad in ONE merged
    stride-phase launch (the shortcut's tap is extra K of the (even, even) phase) == the
    two oracle dgrads summed; and close to the two-launch form (dgrad + accumulate)."""
    torch.manual_seed(12)
    N, H, W, Cc, K = case
    P, Q = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    dy = bf(N, P, Q, K, dev=gpu)
    dy2 = bf(N, P, Q, K, dev=gpu)
    w = bf(K, 3, 3, Cc, dev=gpu, scale=1.0 / math.sqrt(9 * K))
    w2 = bf(K, 1, 1, Cc, dev=gpu, scale=1.0 / math.sqrt(K))
    wt = w.permute(3, 1, 2, 0).reshape(Cc, 9, K).contiguous()
    wt2 = w2.permute(3, 1, 2, 0).reshape(Cc, 1, K).contiguous()
    dx = C().conv_dgrad_pair(dy, w, wt, H, W, 2, 2, 1, 1, dy2, w2, wt2, 0, 0)
    assert dx is not None, "merged launch unavailable on the LDS-DMA engine"
    exp = ref.conv_dgrad_pair(dy, w, wt, H, W, 2, 2, 1, 1, dy2, w2, wt2, 0, 0)
    two = C().conv_dgrad(dy2, w2, H, W, 2, 2, 0, 0, wt2,
                         C().conv_dgrad(dy, w, H, W, 2, 2, 1, 1, wt))
    torch.cuda.synchronize()
    assert dx.shape == (N, H, W, Cc)
    assert rel(dx, exp) < 1e-2
    assert rel(two, exp) < 2e-2
    # the odd phases carry no shortcut tap: bitwise the single dgrad there
    one = C().conv_dgrad(dy, w, H, W, 2, 2, 1, 1, wt)
    torch.cuda.synchronize()
    assert torch.equal(dx[:, 1::2], one[:, 1::2]) and torch.equal(dx[:, :, 1::2], one[:, :, 1::2])


@pytest.mark.parametrize("case", [(2, 14, 14, 64, 64), (4, 56, 56, 64, 64), (2, 28, 28, 128, 128),
                                  (1, 112, 112, 64, 64)])
def test_conv_dgrad_masked_residual(gpu, case):
    """conv1's stride-1 halo dgrad + the identity shortcut's gradient dy_res * (y > 0) read
    in the epilogue (conv_dgrad_res: the masked residual is never written) == the oracle,
    and == the written-then-accumulated form bit for bit (same single rounding)."""
    torch.manual_seed(13)
    N, H, W, Cc, K = case
    dy = bf(N, H, W, K, dev=gpu)
    w = bf(K, 3, 3, Cc, dev=gpu, scale=1.0 / math.sqrt(9 * K))
    wt = w.permute(3, 1, 2, 0).reshape(Cc, 9, K).contiguous()
    res = bf(N, H, W, Cc, dev=gpu)
    yv = bf(N, H, W, Cc, dev=gpu)
    mask = ref.relu_bitmask(yv)
    C().igemm_set_halo(1)
    try:
        dx = C().conv_dgrad_res(dy, w, wt, H, W, 1, 1, res, mask)
        assert dx is not None
        g = (res.float() * (yv.float() > 0)).to(torch.bfloat16)
        two = C().conv_dgrad(dy, w, H, W, 1, 1, 1, 1, wt, g.clone())
        torch.cuda.synchronize()
    finally:
        C().igemm_set_halo(0)
    exp = ref.conv_dgrad_res(dy, w, wt, H, W, 1, 1, res, mask)
    assert rel(dx, exp) < 2e-2
    assert torch.equal(dx, two)


@pytest.mark.parametrize("case", [(2, 14, 14, 64, 64, 3, 3, 1, 1), (2, 14, 14, 64, 128, 3, 3, 2, 1),
                                  (4, 28, 28, 128, 128, 3, 3, 1, 1), (3, 9, 11, 96, 48, 3, 3, 1, 1)])
def test_conv_dgrad_fused_bn_reduction(gpu, case):
    """dgrad whose epilogue applies the producer's ReLU mask and reduces (sum g,
    sum g*xhat) == unfused dgrad + oracle reduction; apply pass with the sums == bn_bwd."""
    torch.manual_seed(11)
    N, H, W, Cc, K, R, S, st, pd = case
    ph, pw = _pair(pd)
    P = (H + 2 * ph - R) // st + 1
    Q = (W + 2 * pw - S) // st + 1
    dy = bf(N, P, Q, K, dev=gpu)
    w = bf(K, R, S, Cc, dev=gpu, scale=1.0 / math.sqrt(R * S * K))
    wt = w.permute(3, 1, 2, 0).reshape(Cc, R * S, K).contiguous()
    z = bf(N, H, W, Cc, dev=gpu, scale=2.0)
    mean = torch.randn(Cc, device=gpu) * 0.3
    rstd = torch.rand(Cc, device=gpu) + 0.5
    y = torch.relu(z.float() - 0.2).to(torch.bfloat16)  # a ReLU output: mask source
    assert C().conv_bnred_ok(K, Cc)
    g, sums = C().conv_dgrad_bnred(dy, w, H, W, st, st, ph, pw, wt, z, y, mean, rstd)
    dx = C().conv_dgrad(dy, w, H, W, st, st, ph, pw, wt)
    gr, sr = ref.conv_dgrad_bnred(dy, w, H, W, st, st, ph, pw, None, z, y, mean, rstd)
    torch.cuda.synchronize()
    # (the unfused dgrad may split K where the fused one does not: compare with tolerance)
    assert rel(g, (dx.float() * (y.float() > 0)).to(torch.bfloat16)) < 1e-2
    assert rel(g, gr) < 2e-2 and rel(sums, sr) < 2e-2
    gamma = torch.rand(Cc, device=gpu) + 0.5
    dg, db = torch.zeros(Cc, device=gpu), torch.zeros(Cc, device=gpu)
    dg2, db2 = dg.clone(), db.clone()
    e = torch.empty(0, device=gpu)
    dz, _ = C().bn_bwd_apply(g, z, e, mean, rstd, gamma, dg, db, sums, True, False)
    dzr, _ = ref.bn_bwd(dx, z, y, mean, rstd, gamma, dg2, db2, True)
    assert rel(dz, dzr) < 3e-2 and rel(dg, dg2) < 2e-2 and rel(db, db2) < 2e-2
    # ReLU mask recomputed from z (y not passed): same mask as bn_fwd_train's rounded y
    beta = torch.randn(Cc, device=gpu) * 0.2
    sc = gamma * rstd
    yz = torch.relu(z.float() * sc + (beta - mean * sc)).to(torch.bfloat16)
    g2, sums2 = C().conv_dgrad_bnred(dy, w, H, W, st, st, ph, pw, wt, z, yz, mean, rstd,
                                     gamma=gamma, beta=beta)
    torch.cuda.synchronize()
    assert rel(g2, (dx.float() * (yz.float() > 0)).to(torch.bfloat16)) < 1e-2
    gr2, sr2 = ref.conv_dgrad_bnred(dy, w, H, W, st, st, ph, pw, None, z, None, mean, rstd,
                                    gamma, beta)
    assert rel(g2, gr2) < 2e-2 and rel(sums2, sr2) < 2e-2


HALO_CASES = [
    # N, H, W, C, K: 3x3 / stride 1 / pad 1
    (2, 56, 56, 64, 64),     # ResNet layer1: resident weights (N = 64, C <= 64)
    (3, 28, 28, 128, 128),   # layer2: two N-tiles, streamed weights
    (5, 14, 14, 256, 256),   # layer3: 256-pixel tiles cross image borders
    (7, 7, 7, 512, 512),     # layer4: a tile spans 6 images (separator slots)
    (3, 9, 11, 96, 128),     # odd W, 3 chunks, two N-tiles, partial last M-tile
    (1, 5, 3, 32, 64),       # single chunk, tiny image, one partial M-tile
    (2, 35, 35, 64, 96),     # Inception-style odd spatial size
    (2, 35, 35, 64, 128),    # halo wgrad at pitch 48
    (3, 17, 17, 128, 64),    # halo wgrad at pitch 32, odd W, tiles across images
    (52, 14, 14, 256, 512),  # 320 tiles on 256 persistent blocks (two rounds), ragged last tile
    (25, 56, 56, 64, 64),    # resident weights, 307 tiles
    (2, 28, 28, 128, 32),    # DenseNet growth conv: 32-wide halo forward, zero-padded wgrad k
    (3, 7, 7, 128, 32),      # DenseNet block 4: 32-wide, tiles across many 7x7 images
    (2, 17, 17, 32, 64),     # 32-channel wgrad partition (second halo chunk empty)
    (2, 9, 9, 96, 96),       # wgrad K and C with a 32-wide remainder partition
    (2, 40, 70, 32, 64),     # 32-channel wgrad, halo wider than one chunk area (ONECH)
    (1, 147, 147, 32, 64),   # Inception Conv2d_2b (ONECH wgrad)
]


def _halo_pair(fn):
    """(halo kernel result, implicit-GEMM result) of fn()."""
    C().igemm_set_halo(1)
    a = fn()
    C().igemm_set_halo(0)
    b = fn()
    torch.cuda.synchronize()
    return a, b


@pytest.mark.parametrize("case", HALO_CASES)
def test_conv_halo_fwd(gpu, case):
    """Halo-staged 3x3/s1 forward == implicit GEMM and the fp32 oracle, in the flavours the
    halo kernel instantiates: shifted BN statistics (the training path), bias + ReLU, and
    bias + statistics (bias + ReLU + statistics falls back to the implicit GEMM)."""
    torch.manual_seed(21)
    N, H, W, Cc, K = case
    x = bf(N, H, W, Cc, dev=gpu)
    w = bf(K, 3, 3, Cc, dev=gpu, scale=1.0 / math.sqrt(9 * Cc))
    b = torch.randn(K, device=gpu)
    e = torch.empty(0, device=gpu)
    shift = torch.randn(K, device=gpu) * 0.1
    for bias, relu, stats in ((e, False, True), (b, True, False), (b, False, True),
                              (b, True, True)):

        def run():
            st = torch.zeros(2, K, device=gpu) if stats else e
            return C().conv_fwd(x, w, bias, 1, 1, 1, 1, relu, st, shift if stats else e), st

        (y, st), (y0, st0) = _halo_pair(run)
        str_ = torch.zeros(2, K, device=gpu) if stats else e
        yr = ref.conv_fwd(x, w, bias, 1, 1, 1, 1, relu, str_, shift if stats else e)
        assert rel(y, y0) < 1e-2 and rel(y, yr) < 2e-2
        if stats:
            assert rel(st, st0) < 1e-3 and rel(st, str_) < 2e-2


@pytest.mark.parametrize("case", HALO_CASES)
def test_conv_halo_dgrad(gpu, case):
    """Stride-1 dgrad from the transposed weight on the halo kernel: plain, accumulating
    (GradJoin) and with the fused BN-backward reduction, against the oracle."""
    torch.manual_seed(22)
    N, H, W, Cc, K = case
    dy = bf(N, H, W, K, dev=gpu)
    w = bf(K, 3, 3, Cc, dev=gpu, scale=1.0 / math.sqrt(9 * K))
    wt = w.permute(3, 1, 2, 0).reshape(Cc, 9, K).contiguous()
    acc0 = bf(N, H, W, Cc, dev=gpu)
    dx, dx0 = _halo_pair(lambda: C().conv_dgrad(dy, w, H, W, 1, 1, 1, 1, wt))
    dxr = ref.conv_dgrad(dy, w, H, W, 1, 1, 1, 1)
    assert rel(dx, dx0) < 1e-2 and rel(dx, dxr) < 2e-2
    acc, _ = _halo_pair(lambda: C().conv_dgrad(dy, w, H, W, 1, 1, 1, 1, wt, acc0.clone()))
    assert rel(acc, acc0.float() + dxr.float()) < 2e-2
    z = bf(N, H, W, Cc, dev=gpu, scale=2.0)
    mean = torch.randn(Cc, device=gpu) * 0.3
    rstd = torch.rand(Cc, device=gpu) + 0.5
    y = torch.relu(z.float() - 0.2).to(torch.bfloat16)
    gamma = torch.rand(Cc, device=gpu) + 0.5
    beta = torch.randn(Cc, device=gpu) * 0.2
    sc = gamma * rstd
    yz = torch.relu(z.float() * sc + (beta - mean * sc)).to(torch.bfloat16)  # forward's y
    # mask from y (implicit GEMM only) and, given gamma / beta, recomputed from z by the halo
    # kernel (y is then the implicit GEMM's mask source)
    for yy, ga, be in ((y, None, None), (yz, gamma, beta)):
        (g, sums), (g0, sums0) = _halo_pair(
            lambda: C().conv_dgrad_bnred(dy, w, H, W, 1, 1, 1, 1, wt, z, yy, mean, rstd,
                                         gamma=ga, beta=be))
        gr, sr = ref.conv_dgrad_bnred(dy, w, H, W, 1, 1, 1, 1, None, z,
                                      yy if ga is None else None, mean, rstd, ga, be)
        assert rel(g, g0) < 1e-2 and rel(sums, sums0) < 1e-2
        assert rel(g, gr) < 2e-2 and rel(sums, sr) < 2e-2


STRIP_CASES = [
    # N, H, W, C, K, MPA_HALO_STRIP mode
    (2, 112, 112, 64, 64, 1),   # VGG 112^2 (resident weights, one 112-wide strip)
    (1, 224, 224, 64, 64, 1),   # VGG 224^2 (two 112-wide strips)
    (2, 33, 150, 64, 128, 1),   # partial row bands and strips, two column tiles
    (3, 20, 131, 96, 64, 1),    # three channel chunks: streamed weights
    (1, 147, 147, 32, 64, 1),   # Inception Conv2d_2b
    (4, 56, 56, 64, 64, 2),     # ResNet layer1: 4 x 56 tiles, 3-stage ring
    (2, 56, 56, 64, 64, 0),     # (linear tiles, for comparison)
]


@pytest.mark.parametrize("case", STRIP_CASES)
def test_conv_halo_strip(gpu, case):
    """Strip-tiled halo kernel (2-D tiles, images wider than the linear tiles hold; 3-stage
    ring for resident-weight layer1 shapes): forward with BN statistics, bias + ReLU,
    dgrad plain / accumulating / fused BN reduction == implicit GEMM and the oracle."""
    torch.manual_seed(25)
    N, H, W, Cc, K, mode = case
    C().igemm_set_halo_strip(mode)
    try:
        x = bf(N, H, W, Cc, dev=gpu)
        w = bf(K, 3, 3, Cc, dev=gpu, scale=1.0 / math.sqrt(9 * Cc))
        b = torch.randn(K, device=gpu)
        e = torch.empty(0, device=gpu)
        shift = torch.randn(K, device=gpu) * 0.1
        for bias, relu, stats in ((e, False, True), (b, True, False)):

            def run():
                st = torch.zeros(2, K, device=gpu) if stats else e
                return C().conv_fwd(x, w, bias, 1, 1, 1, 1, relu, st, shift if stats else e), st

            (y, st), (y0, st0) = _halo_pair(run)
            str_ = torch.zeros(2, K, device=gpu) if stats else e
            yr = ref.conv_fwd(x, w, bias, 1, 1, 1, 1, relu, str_, shift if stats else e)
            assert rel(y, y0) < 1e-2 and rel(y, yr) < 2e-2
            if stats:
                assert rel(st, st0) < 1e-3 and rel(st, str_) < 2e-2
        dy = bf(N, H, W, K, dev=gpu)
        wd = bf(K, 3, 3, Cc, dev=gpu, scale=1.0 / math.sqrt(9 * K))
        wt = wd.permute(3, 1, 2, 0).reshape(Cc, 9, K).contiguous()
        dx, dx0 = _halo_pair(lambda: C().conv_dgrad(dy, wd, H, W, 1, 1, 1, 1, wt))
        dxr = ref.conv_dgrad(dy, wd, H, W, 1, 1, 1, 1)
        assert rel(dx, dx0) < 1e-2 and rel(dx, dxr) < 2e-2
        acc0 = bf(N, H, W, Cc, dev=gpu)
        acc, _ = _halo_pair(lambda: C().conv_dgrad(dy, wd, H, W, 1, 1, 1, 1, wt, acc0.clone()))
        assert rel(acc, acc0.float() + dxr.float()) < 2e-2
        z = bf(N, H, W, Cc, dev=gpu, scale=2.0)
        mean = torch.randn(Cc, device=gpu) * 0.3
        rstd = torch.rand(Cc, device=gpu) + 0.5
        gamma = torch.rand(Cc, device=gpu) + 0.5
        beta = torch.randn(Cc, device=gpu) * 0.2
        sc = gamma * rstd
        yz = torch.relu(z.float() * sc + (beta - mean * sc)).to(torch.bfloat16)
        (g, sums), (g0, sums0) = _halo_pair(
            lambda: C().conv_dgrad_bnred(dy, wd, H, W, 1, 1, 1, 1, wt, z, yz, mean, rstd,
                                         gamma=gamma, beta=beta))
        gr, sr = ref.conv_dgrad_bnred(dy, wd, H, W, 1, 1, 1, 1, None, z, None, mean, rstd,
                                      gamma, beta)
        assert rel(g, g0) < 1e-2 and rel(sums, sums0) < 1e-2
        assert rel(g, gr) < 2e-2 and rel(sums, sr) < 2e-2
        # weight gradient (strip tiles where the linear 128-pixel tiles do not fit)
        dw0 = torch.randn(K, 3, 3, Cc, device=gpu)

        def wg():
            dw = dw0.clone()
            C().conv_wgrad(dy, x, dw, 1, 1, 1, 1)
            return dw

        dw, dwi = _halo_pair(wg)
        dwr = dw0.clone()
        ref.conv_wgrad(dy, x, dwr, 1, 1, 1, 1)
        assert rel(dw - dw0, dwi - dw0) < 1e-2 and rel(dw - dw0, dwr - dw0) < 2e-2
        # persistent ring: repeated launches bitwise identical (race screen)
        C().igemm_set_halo(1)
        outs = [C().conv_dgrad(dy, wd, H, W, 1, 1, 1, 1, wt) for _ in range(3)]
        torch.cuda.synchronize()
        assert all(torch.equal(o, outs[0]) for o in outs[1:])
    finally:
        C().igemm_set_halo_strip(1)
        C().igemm_set_halo(0)


@pytest.mark.parametrize("case", [(2, 37, 41, 32, 32), (1, 149, 149, 32, 32),
                                  (2, 20, 70, 64, 64), (2, 30, 30, 64, 32)])
def test_conv_halo_strip_valid(gpu, case):
    """Unpadded ("valid") 3x3 convs on the strip-tiled halo kernels (Inception's
    Conv2d_2a): the shifted tap set in the forward (output 2 smaller), its dgrad (padding
    2, output 2 larger: plain, accumulating, fused BN reduction) and the weight gradient ==
    implicit GEMM and the oracle; 32-wide outputs run the NJ = 2 form."""
    torch.manual_seed(26)
    N, H, W, Cc, K = case
    P, Q = H - 2, W - 2
    C().igemm_set_halo_strip(1)
    try:
        x = bf(N, H, W, Cc, dev=gpu)
        w = bf(K, 3, 3, Cc, dev=gpu, scale=1.0 / math.sqrt(9 * Cc))
        e = torch.empty(0, device=gpu)
        shift = torch.randn(K, device=gpu) * 0.1

        def run():
            st = torch.zeros(2, K, device=gpu)
            return C().conv_fwd(x, w, e, 1, 1, 0, 0, False, st, shift), st

        (y, st), (y0, st0) = _halo_pair(run)
        str_ = torch.zeros(2, K, device=gpu)
        yr = ref.conv_fwd(x, w, e, 1, 1, 0, 0, False, str_, shift)
        assert y.shape == (N, P, Q, K)
        assert rel(y, y0) < 1e-2 and rel(y, yr) < 2e-2
        assert rel(st, st0) < 1e-3 and rel(st, str_) < 2e-2
        dy = bf(N, P, Q, K, dev=gpu)
        wt = w.permute(3, 1, 2, 0).reshape(Cc, 9, K).contiguous()
        dx, dx0 = _halo_pair(lambda: C().conv_dgrad(dy, w, H, W, 1, 1, 0, 0, wt))
        dxr = ref.conv_dgrad(dy, w, H, W, 1, 1, 0, 0)
        assert rel(dx, dx0) < 1e-2 and rel(dx, dxr) < 2e-2
        acc0 = bf(N, H, W, Cc, dev=gpu)
        acc, _ = _halo_pair(lambda: C().conv_dgrad(dy, w, H, W, 1, 1, 0, 0, wt, acc0.clone()))
        assert rel(acc, acc0.float() + dxr.float()) < 2e-2
        z = bf(N, H, W, Cc, dev=gpu, scale=2.0)
        mean = torch.randn(Cc, device=gpu) * 0.3
        rstd = torch.rand(Cc, device=gpu) + 0.5
        gamma = torch.rand(Cc, device=gpu) + 0.5
        beta = torch.randn(Cc, device=gpu) * 0.2
        sc = gamma * rstd
        yz = torch.relu(z.float() * sc + (beta - mean * sc)).to(torch.bfloat16)
        (g, sums), (g0, sums0) = _halo_pair(
            lambda: C().conv_dgrad_bnred(dy, w, H, W, 1, 1, 0, 0, wt, z, yz, mean, rstd,
                                         gamma=gamma, beta=beta))
        gr, sr = ref.conv_dgrad_bnred(dy, w, H, W, 1, 1, 0, 0, None, z, None, mean, rstd,
                                      gamma, beta)
        assert rel(g, g0) < 1e-2 and rel(sums, sums0) < 1e-2
        assert rel(g, gr) < 2e-2 and rel(sums, sr) < 2e-2
        dw0 = torch.randn(K, 3, 3, Cc, device=gpu)

        def wg():
            dw = dw0.clone()
            C().conv_wgrad(dy, x, dw, 1, 1, 0, 0)
            return dw

        dw, dwi = _halo_pair(wg)
        dwr = dw0.clone()
        ref.conv_wgrad(dy, x, dwr, 1, 1, 0, 0)
        assert rel(dw - dw0, dwi - dw0) < 1e-2 and rel(dw - dw0, dwr - dw0) < 2e-2
    finally:
        C().igemm_set_halo(0)


@pytest.mark.parametrize("case", HALO_CASES)
def test_conv_halo_wgrad(gpu, case):
    """Halo-staged 3x3/s1 weight gradient (slab partials + reduce, accumulating into dw)
    == implicit-GEMM wgrad and the fp32 oracle."""
    torch.manual_seed(24)
    N, H, W, Cc, K = case
    x = bf(N, H, W, Cc, dev=gpu)
    dy = bf(N, H, W, K, dev=gpu)
    dw0 = torch.randn(K, 3, 3, Cc, device=gpu)

    def run():
        dw = dw0.clone()
        C().conv_wgrad(dy, x, dw, 1, 1, 1, 1)
        return dw

    dw, dwi = _halo_pair(run)
    dwr = dw0.clone()
    ref.conv_wgrad(dy, x, dwr, 1, 1, 1, 1)
    assert rel(dw, dwi) < 1e-3 and rel(dw - dw0, dwr - dw0) < 1e-2


@pytest.mark.parametrize("case", [
    (16, 28, 28, 128, 128),  # ResNet layer2: 4 partitions x 64 z lanes
    (16, 14, 14, 256, 256),  # layer3: 16 partitions x 16 z lanes
    (32, 7, 7, 512, 512),    # layer4: 64 partitions x 4 z lanes
    (8, 17, 17, 96, 96),     # 32-wide remainder partitions
])
def test_halo_wgrad_xmap_bitwise(gpu, case):
    """XCD-grouped weight-gradient block order (round 6, MPA_HALO_WXMAP): every (z lane,
    partition) block does the same work and writes the same slab, only its placement on
    the XCDs changes - bitwise equal to the plain order, in both the 4-wave and the
    producer-wave forms; and the fp32 oracle."""
    torch.manual_seed(29)
    N, H, W, Cc, K = case
    x = bf(N, H, W, Cc, dev=gpu)
    dy = bf(N, H, W, K, dev=gpu)
    dw0 = torch.randn(K, 3, 3, Cc, device=gpu)
    out = {}
    try:
        C().igemm_set_halo(1)
        for prod in (0, 1):
            C().igemm_set_halo_wprod(prod)
            for xm in (0, 1):
                C().igemm_set_halo_wxmap(xm)
                dw = dw0.clone()
                C().conv_wgrad(dy, x, dw, 1, 1, 1, 1)
                out[prod, xm] = dw
        torch.cuda.synchronize()
    finally:
        C().igemm_set_halo_wxmap(1)
        C().igemm_set_halo_wprod(1)
        C().igemm_set_halo(0)
    for prod in (0, 1):
        assert torch.equal(out[prod, 0], out[prod, 1])
    dwr = dw0.clone()
    ref.conv_wgrad(dy, x, dwr, 1, 1, 1, 1)
    assert rel(out[1, 1] - dw0, dwr - dw0) < 1e-2


@pytest.mark.parametrize("case", [
    # N, H, W, C, K, R, stride, pad: strided 3x3, 1x1 downsample, deep-K strided
    (4, 14, 14, 64, 128, 3, 2, 1),
    (4, 14, 14, 64, 128, 1, 2, 0),
    (2, 7, 7, 256, 512, 3, 2, 1),
])
def test_gemm_autotune(gpu, case):
    """Tile autotuner (igemm.hip, MPA_TUNE): the tuned plans give the static plans' results
    (rows GEMMs keep their K order; a wgrad's split count may change) and the choices are
    cached per shape."""
    torch.manual_seed(31)
    N, H, W, Cc, K, R, st, pd = case
    P = (H + 2 * pd - R) // st + 1
    x = bf(N, H, W, Cc, dev=gpu)
    w = bf(K, R, R, Cc, dev=gpu, scale=1.0 / math.sqrt(R * R * Cc))
    wt = w.permute(3, 1, 2, 0).reshape(Cc, R * R, K).contiguous()
    dy = bf(N, P, P, K, dev=gpu)
    e = torch.empty(0, device=gpu)

    def run():
        stt = torch.zeros(2, K, device=gpu)
        y = C().conv_fwd(x, w, e, st, st, pd, pd, False, stt, e)
        dx = C().conv_dgrad(dy, w, H, W, st, st, pd, pd, wt)
        dw = torch.zeros(K, R, R, Cc, device=gpu)
        C().conv_wgrad(dy, x, dw, st, st, pd, pd)
        torch.cuda.synchronize()
        return y, stt, dx, dw

    C().igemm_set_tune(0)
    try:
        ref0 = run()
    finally:
        C().igemm_set_tune(1)
    tuned = run()   # first call: tunes, then runs the chosen tiles
    again = run()   # cached choice
    for a, b, c in zip(ref0, tuned, again):
        assert torch.isfinite(b.float()).all()
        assert rel(b, a) < 1e-3 and torch.equal(b, c)
    table = C().igemm_tuned_table()
    assert "rows" in table and "wgrad" in table


@pytest.mark.parametrize("case", [
    # N, H, W, C, K: 1x1 convs deep enough in K to split (split-K finalize, 32 / 64 columns)
    (64, 7, 7, 544, 32),
    (16, 5, 5, 768, 96),
    (4, 7, 7, 1024, 512),
])
def test_splitk_finalize(gpu, case):
    """Split-K forward (fp32 partial slab + splitk_finalize: sum, bias, ReLU, bf16, shifted
    BN statistics) == the fp32 oracle, for 32-column and wider GEMMs."""
    torch.manual_seed(27)
    N, H, W, Cc, K = case
    x = bf(N, H, W, Cc, dev=gpu)
    w = bf(K, 1, 1, Cc, dev=gpu, scale=1.0 / math.sqrt(Cc))
    e = torch.empty(0, device=gpu)
    b = torch.randn(K, device=gpu)
    shift = torch.randn(K, device=gpu) * 0.1
    for bias, relu, stats in ((e, False, True), (b, True, False), (b, False, True)):
        st = torch.zeros(2, K, device=gpu) if stats else e
        y = C().conv_fwd(x, w, bias, 1, 1, 0, 0, relu, st, shift if stats else e)
        str_ = torch.zeros(2, K, device=gpu) if stats else e
        yr = ref.conv_fwd(x, w, bias, 1, 1, 0, 0, relu, str_, shift if stats else e)
        torch.cuda.synchronize()
        assert rel(y, yr) < 2e-2
        if stats:
            assert rel(st, str_) < 2e-2


@pytest.mark.parametrize("gdt", [torch.bfloat16, torch.float32])
def test_dense_deferred_norm1_backward(gpu, gdt):
    """DenseNet norm1 -> conv1 hand-off: the 1x1 dgrad epilogue adds gamma*rstd * g into the
    block gradient's channel prefix and reduces (sum g, sum g*xhat); bn_defer_step folds the
    per-channel corrections and finishes a channel slice - both == the fp32 oracle."""
    torch.manual_seed(41)
    N, H, W, ctot, Ci, K = 3, 14, 14, 320, 256, 128
    buf = bf(N, H, W, ctot, dev=gpu, scale=2.0)
    dz = bf(N, H, W, K, dev=gpu)
    w = bf(K, 1, 1, Ci, dev=gpu, scale=1.0 / math.sqrt(K))
    wt = w.permute(3, 1, 2, 0).reshape(Ci, 1, K).contiguous()
    mean = torch.randn(ctot, device=gpu) * 0.3
    rstd = torch.rand(ctot, device=gpu) + 0.5
    gamma = torch.rand(Ci, device=gpu) + 0.5
    beta = torch.randn(Ci, device=gpu) * 0.2
    G0 = torch.randn(N, H, W, ctot, device=gpu).to(gdt)
    G, Gr = G0.clone(), G0.clone()
    sums = C().conv_dgrad_bnred_gacc(dz, w, wt, buf, mean, rstd, gamma, beta, G)
    sr = ref.conv_dgrad_bnred_gacc(dz, w, wt, buf, mean, rstd, gamma, beta, Gr)
    torch.cuda.synchronize()
    assert rel(G, Gr) < 1e-2 and rel(sums, sr) < 2e-2
    assert torch.equal(G[..., Ci:], G0[..., Ci:])  # channels past the prefix untouched
    for s0 in (224, 0):  # a 32-channel slice (layer i > 0), the whole prefix (layer 0)
        k12 = torch.randn(2, ctot, device=gpu)
        k12_0 = k12.clone()
        dg, db = torch.zeros(Ci, device=gpu), torch.zeros(Ci, device=gpu)
        k12r, dgr, dbr = k12.clone(), dg.clone(), db.clone()
        G1, G1r = G.clone(), G.clone()
        C().bn_defer_step(sums, gamma, mean, rstd, s0, k12, dg, db, G1, buf)
        ref.bn_defer_step(sums, gamma, mean, rstd, s0, k12r, dgr, dbr, G1r, buf)
        torch.cuda.synchronize()
        assert rel(G1, G1r) < 1e-2 and rel(k12, k12r) < 1e-5
        assert rel(dg, dgr) < 1e-5 and rel(db, dbr) < 1e-5
        assert torch.equal(G1[..., :s0], G[..., :s0]) and torch.equal(G1[..., Ci:], G[..., Ci:])
        # handover form: the finished slice goes to `out` (G's copy left as it was)
        G2 = G.clone()
        o = torch.empty(N, H, W, Ci - s0, device=gpu, dtype=torch.bfloat16)
        e = torch.empty(0, device=gpu)
        C().bn_defer_step(sums, gamma, mean, rstd, s0, k12_0, e, e, G2, buf, o)
        torch.cuda.synchronize()
        assert torch.equal(G2, G) and rel(o, G1r[..., s0:Ci]) < 1e-2


@pytest.mark.parametrize("shape", [(2, 56, 56, 256), (3, 14, 10, 64)])
def test_bn_relu_avgpool2(gpu, shape):
    """relu(bn(z)) -> 2x2/s2 average pool in one pass (DenseNet transitions): statistics
    half + fused pool == the oracle; running stats and num_batches_tracked updated once."""
    torch.manual_seed(43)
    N, H, W, Cc = shape
    z = bf(N, H, W, Cc, dev=gpu, scale=1.5)
    st = torch.stack([z.float().reshape(-1, Cc).mean(0),
                      z.float().reshape(-1, Cc).var(0, unbiased=False)])
    g = torch.rand(Cc, device=gpu) + 0.5
    b = torch.randn(Cc, device=gpu) * 0.5
    rm, rv = torch.zeros(Cc, device=gpu), torch.ones(Cc, device=gpu)
    rm2, rv2 = rm.clone(), rv.clone()
    cnt = torch.tensor(3, dtype=torch.long, device=gpu)
    mean, rstd, aff = C().bn_stats_affine(z, st, g, b, rm, rv, 0.1, 1e-5, cnt)
    meanr, rstdr, affr = ref.bn_stats_affine(z, st, g, b, rm2, rv2, 0.1, 1e-5)
    y = C().bn_relu_avgpool2_fwd(z, aff)
    yr = ref.bn_relu_avgpool2_fwd(z, affr)
    torch.cuda.synchronize()
    assert int(cnt) == 4
    assert rel(mean, meanr) < 1e-3 and rel(rstd, rstdr) < 1e-3 and rel(aff, affr) < 1e-3
    assert rel(rm, rm2) < 1e-3 and rel(rv, rv2) < 1e-3
    assert y.shape == yr.shape and rel(y, yr) < 1e-2


def test_conv_halo_repeatable(gpu):
    """Persistent 2-stage ring: repeated launches are bitwise identical (race screen)."""
    torch.manual_seed(23)
    x = bf(16, 28, 28, 128, dev=gpu)
    w = bf(128, 3, 3, 128, dev=gpu, scale=1.0 / math.sqrt(9 * 128))
    e = torch.empty(0, device=gpu)
    C().igemm_set_halo(1)
    outs = [C().conv_fwd(x, w, e, 1, 1, 1, 1, False, torch.zeros(2, 128, device=gpu), e)
            for _ in range(4)]
    torch.cuda.synchronize()
    for o in outs[1:]:
        assert torch.equal(o, outs[0])


def test_transpose_krsc_and_linear_dgrad_transposed(gpu):
    torch.manual_seed(9)
    shapes = [(64, 9, 8), (200, 1, 512), (136, 9, 264), (64512, 1, 512)]
    ws = [bf(K, RS, Cc, dev=gpu) for K, RS, Cc in shapes]
    src = torch.cat([w.reshape(-1) for w in ws])
    dst = torch.zeros_like(src)
    rows, off, tiles = [], 0, 0
    for (K, RS, Cc), w in zip(shapes, ws):
        rows.append([off, off, K, RS, Cc, tiles])
        tiles += RS * ((K + 63) // 64) * ((Cc + 63) // 64)
        off += w.numel()
    C().transpose_krsc(src, dst, torch.tensor(rows, device=gpu), tiles)
    off = 0
    for (K, RS, Cc), w in zip(shapes, ws):
        got = dst[off:off + w.numel()].view(Cc, RS, K)
        assert torch.equal(got, w.permute(2, 1, 0)), (K, RS, Cc)
        off += w.numel()
    # linear dgrad through the transposed weight [in][out]
    B, Cin, Cout = 32, 512, 64512
    w = bf(Cout, Cin, dev=gpu, scale=1.0 / math.sqrt(Cout))
    dy = bf(B, Cout, dev=gpu)
    a = C().linear_dgrad(dy, w)
    b = C().linear_dgrad(dy, w, w.t().contiguous())
    assert rel(b, ref.linear_dgrad(dy, w)) < 2e-2 and rel(a, b) < 1e-2


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_wgrad(gpu, engine, case):
    torch.manual_seed(2)
    N, H, W, Cc, K, R, S, st, pd = case
    ph, pw = _pair(pd)
    P = (H + 2 * ph - R) // st + 1
    Q = (W + 2 * pw - S) // st + 1
    dy = bf(N, P, Q, K, dev=gpu)
    x = bf(N, H, W, Cc, dev=gpu)
    dw = torch.full((K, R, S, Cc), 0.5, device=gpu)   # accumulates into existing contents
    dwr = dw.clone()
    C().conv_wgrad(dy, x, dw, st, st, ph, pw)
    ref.conv_wgrad(dy, x, dwr, st, st, ph, pw)
    torch.cuda.synchronize()
    assert rel(dw, dwr) < 1e-2


@pytest.mark.parametrize("case", [CONV_CASES[i] for i in (1, 2, 4, 6, 7, 11, 12, 13, 14)])
def test_engines_bitwise_equal(gpu, case):
    """Both staging engines run the same MFMA sequence over the same LDS images, so every
    output must match bit for bit; repeated launches screen the DMA ring for races."""
    torch.manual_seed(5)
    N, H, W, Cc, K, R, S, st, pd = case
    ph, pw = _pair(pd)
    P = (H + 2 * ph - R) // st + 1
    Q = (W + 2 * pw - S) // st + 1
    x = bf(N, H, W, Cc, dev=gpu)
    w = bf(K, R, S, Cc, dev=gpu, scale=1.0 / math.sqrt(R * S * Cc))
    dy = bf(N, P, Q, K, dev=gpu)
    e = torch.empty(0, device=gpu)
    prev = C().igemm_engine()
    outs = {}
    try:
        for eng, uni in ((0, 1), (2, 0), (2, 1)):
            C().igemm_set_engine(eng)
            C().igemm_set_dma_uni(uni)
            for rep in range(3 if eng else 1):
                stt = torch.zeros(2, K, device=gpu)
                y = C().conv_fwd(x, w, e, st, st, ph, pw, False, stt, e)
                dx = C().conv_dgrad(dy, w, H, W, st, st, ph, pw)
                dw = torch.zeros(K, R, S, Cc, device=gpu)
                C().conv_wgrad(dy, x, dw, st, st, ph, pw)
                outs[(eng, uni, rep)] = (y, stt, dx, dw)
    finally:
        C().igemm_set_engine(prev)
        C().igemm_set_dma_uni(1)
    torch.cuda.synchronize()
    base = outs[(0, 1, 0)]
    for key, o in outs.items():
        for a, b, nm in zip(o, base, ("y", "stats", "dx", "dw")):
            if Cc == 8 and key[0] == 2 and key[1] == 1 and nm in ("y", "stats"):
                # 8-channel stem on the super-tap path: K is grouped by 4 kernel columns
                # (zero-padded), a different fp32 summation order than (r, s, c) tiles
                assert rel(a, b) < 1e-2, (key, nm, rel(a, b))
            elif nm == "stats":
                # per-tile partial sums: the engines may pick different tile heights
                assert rel(a, b) < 1e-5, (key, nm, rel(a, b))
            else:
                assert torch.equal(a, b), (key, nm, rel(a, b))


TILES = [(256, 256), (256, 128), (128, 128), (256, 64), (128, 32), (128, 256), (64, 128)]


@pytest.mark.parametrize("case", [(2, 16, 16, 256, 256, 3, 3, 1, 1), (3, 15, 13, 136, 264, 3, 3, 2, 1),
                                  (2, 20, 20, 64, 128, 1, 1, 1, 0)])
def test_forced_tiles_bitwise(gpu, case):
    """Every tile shape of both engines, with split-K pinned to 1, accumulates each output
    over K in the same order: all must agree bit for bit with the register engine's
    default tile, and that one with the fp32 oracle."""
    torch.manual_seed(6)
    N, H, W, Cc, K, R, S, st, pd = case
    ph, pw = _pair(pd)
    P = (H + 2 * ph - R) // st + 1
    Q = (W + 2 * pw - S) // st + 1
    x = bf(N, H, W, Cc, dev=gpu)
    w = bf(K, R, S, Cc, dev=gpu, scale=1.0 / math.sqrt(R * S * Cc))
    dy = bf(N, P, Q, K, dev=gpu)
    e = torch.empty(0, device=gpu)

    def run():
        stt = torch.zeros(2, K, device=gpu)
        y = C().conv_fwd(x, w, e, st, st, ph, pw, False, stt, e)
        dx = C().conv_dgrad(dy, w, H, W, st, st, ph, pw)
        dw = torch.zeros(K, R, S, Cc, device=gpu)
        C().conv_wgrad(dy, x, dw, st, st, ph, pw)
        return y, stt, dx, dw

    prev = C().igemm_engine()
    try:
        C().igemm_set_engine(0)
        C().igemm_force_tile(0, 0, 1)
        base = run()
        for eng in (0, 2):
            C().igemm_set_engine(eng)
            for bm, bn in TILES:
                C().igemm_force_tile(bm, bn, 1)
                out = run()
                for a, b, nm in zip(out, base, ("y", "stats", "dx", "dw")):
                    if nm == "stats":  # per-tile partial sums: order depends on BM
                        assert rel(a, b) < 1e-5, (eng, bm, bn, rel(a, b))
                    else:
                        assert torch.equal(a, b), (eng, bm, bn, nm, rel(a, b))
    finally:
        C().igemm_force_tile(0, 0, 0)
        C().igemm_set_engine(prev)
    dwr = torch.zeros(K, R, S, Cc, device=gpu)
    ref.conv_wgrad(dy, x, dwr, st, st, ph, pw)
    assert rel(base[0], ref.conv_fwd(x, w, e, st, st, ph, pw, False, None, None)) < 2e-2
    assert rel(base[2], ref.conv_dgrad(dy, w, H, W, st, st, ph, pw)) < 2e-2
    assert rel(base[3], dwr) < 1e-2


@pytest.mark.parametrize("B,Cin,Cout", [(8, 512, 1000), (128, 512, 64500), (16, 72, 36),
                                        (32, 4096, 4096)])
def test_linear(gpu, engine, B, Cin, Cout):
    torch.manual_seed(3)
    x = bf(B, Cin, dev=gpu)
    w = bf(Cout, Cin, dev=gpu, scale=1.0 / math.sqrt(Cin))
    b = torch.randn(Cout, device=gpu)
    y = C().linear_fwd(x, w, b, False)
    assert rel(y, ref.linear_fwd(x, w, b, False)) < 2e-2
    dy = bf(B, Cout, dev=gpu)
    assert rel(C().linear_dgrad(dy, w), ref.linear_dgrad(dy, w)) < 2e-2
    dw = torch.zeros(Cout, Cin, device=gpu)
    dwr = torch.zeros(Cout, Cin, device=gpu)
    C().linear_wgrad(dy, x, dw)
    ref.linear_wgrad(dy, x, dwr)
    assert rel(dw, dwr) < 1e-2


@pytest.mark.parametrize("M,Cc", [(4096, 64), (1000, 96), (37, 2048), (5000, 24),
                                  (200000, 64), (70001, 128)])  # last two: 4-row unrolled sweeps
@pytest.mark.parametrize("relu,res", [(True, True), (False, False), (True, False)])
def test_bn(gpu, M, Cc, relu, res):
    torch.manual_seed(4)
    x = bf(M, Cc, dev=gpu, scale=2.0) + 0.5
    x = x.to(torch.bfloat16)
    g = torch.rand(Cc, device=gpu) + 0.5
    b = torch.randn(Cc, device=gpu)
    r = bf(M, Cc, dev=gpu) if res else torch.empty(0, device=gpu)
    rm, rv = torch.zeros(Cc, device=gpu), torch.ones(Cc, device=gpu)
    rm2, rv2 = rm.clone(), rv.clone()
    e = torch.empty(0, device=gpu)
    cnt = torch.tensor(7, dtype=torch.long, device=gpu)
    y, mean, rstd = C().bn_fwd_train(x, e, g, b, rm, rv, 0.1, 1e-5, r, relu, cnt)
    yr, meanr, rstdr = ref.bn_fwd_train(x, e, g, b, rm2, rv2, 0.1, 1e-5, r, relu)
    assert int(cnt) == 8  # num_batches_tracked bumped inside the kernel
    assert rel(y, yr) < 2e-2
    assert rel(mean, meanr) < 1e-3 and rel(rstd, rstdr) < 1e-3
    assert rel(rm, rm2) < 1e-3 and rel(rv, rv2) < 1e-3
    ye = C().bn_fwd_eval(x, g, b, rm, rv, 1e-5, r, relu)
    assert rel(ye, ref.bn_fwd_eval(x, g, b, rm2, rv2, 1e-5, r, relu)) < 2e-2
    dy = bf(M, Cc, dev=gpu)
    dg, db = torch.zeros(Cc, device=gpu), torch.zeros(Cc, device=gpu)
    dg2, db2 = dg.clone(), db.clone()
    yy = y if relu else e
    dx, gg = C().bn_bwd(dy, x, yy, mean, rstd, g, dg, db, True, True)
    # same ReLU mask on both sides: native and oracle y differ by bf16 rounding, and a
    # value at 0 flips the mask (with 12.8M elements some always do)
    dxr, ggr = ref.bn_bwd(dy, x, yy, meanr, rstdr, g, dg2, db2, True)
    assert rel(dx, dxr) < 3e-2
    assert rel(gg, ggr) < 2e-2
    assert rel(dg, dg2) < 1e-2 and rel(db, db2) < 1e-2


@pytest.mark.parametrize("M,Cc", [(4096, 64), (1000, 136)])
def test_bn_bwd_mask_from_z(gpu, M, Cc):
    """relu(bn(z)) backward with the mask recomputed from z (no y read) == the y-masked
    backward, bit for bit: the recomputation replays bn_fwd_train's fma and rounding."""
    torch.manual_seed(14)
    x = (bf(M, Cc, dev=gpu, scale=2.0) + 0.3).to(torch.bfloat16)
    g = torch.rand(Cc, device=gpu) + 0.5
    b = torch.randn(Cc, device=gpu)
    e = torch.empty(0, device=gpu)
    rm, rv = torch.zeros(Cc, device=gpu), torch.ones(Cc, device=gpu)
    y, mean, rstd = C().bn_fwd_train(x, e, g, b, rm, rv, 0.1, 1e-5, e, True, e)
    dy = bf(M, Cc, dev=gpu)
    dg, db = torch.zeros(Cc, device=gpu), torch.zeros(Cc, device=gpu)
    dg2, db2 = dg.clone(), db.clone()
    dx, gg = C().bn_bwd(dy, x, y, mean, rstd, g, dg, db, True, True)
    dxz, ggz = C().bn_bwd(dy, x, e, mean, rstd, g, dg2, db2, True, True, b)
    torch.cuda.synchronize()
    assert torch.equal(gg, ggz) and torch.equal(dx, dxz)
    assert torch.equal(dg, dg2) and torch.equal(db, db2)


@pytest.mark.parametrize("M,Cc", [(4096, 64), (1003, 24)])
def test_bn_relu_bitmask(gpu, M, Cc):
    """relu(bn(z) + res): the forward's 1-bit ReLU mask equals (y > 0) packed 8 per byte, and
    the backward from the mask == the backward from y, bit for bit (residual blocks)."""
    torch.manual_seed(15)
    x = (bf(M, Cc, dev=gpu, scale=2.0) + 0.3).to(torch.bfloat16)
    r = bf(M, Cc, dev=gpu)
    g = torch.rand(Cc, device=gpu) + 0.5
    b = torch.randn(Cc, device=gpu)
    e = torch.empty(0, device=gpu)
    rm, rv = torch.zeros(Cc, device=gpu), torch.ones(Cc, device=gpu)
    mask = torch.empty(M * Cc // 8, dtype=torch.uint8, device=gpu)
    y, mean, rstd = C().bn_fwd_train(x, e, g, b, rm, rv, 0.1, 1e-5, r, True, e, mask)
    torch.cuda.synchronize()
    assert torch.equal(mask, ref.relu_bitmask(y))
    assert torch.equal(ref.bitmask_unpack(mask, y.shape), y > 0)
    dy = bf(M, Cc, dev=gpu)
    dg, db = torch.zeros(Cc, device=gpu), torch.zeros(Cc, device=gpu)
    dg2, db2 = dg.clone(), db.clone()
    dx, gg = C().bn_bwd(dy, x, y, mean, rstd, g, dg, db, True, True)
    dxm, ggm = C().bn_bwd(dy, x, e, mean, rstd, g, dg2, db2, True, True, None, mask)
    torch.cuda.synchronize()
    assert torch.equal(gg, ggm) and torch.equal(dx, dxm)
    assert torch.equal(dg, dg2) and torch.equal(db, db2)


@pytest.mark.parametrize("M,Cc", [(4096, 64), (100352, 128), (1003, 24)])
def test_bn_bwd_pair_residual_deferred_bn(gpu, M, Cc):
    """relu(bn(x) + bn2(x2)) backward with both BNs in train mode (ResNet bn2 + the deferred
    downsample BN): bn_bwd_pair's dx / dx2 / affine gradients == the oracle, and == the
    two-stage form (bn_bwd writing g, then bn_bwd of the second BN on g) to bf16 rounding."""
    torch.manual_seed(16)
    x = (bf(M, Cc, dev=gpu, scale=2.0) + 0.3).to(torch.bfloat16)
    x2 = (bf(M, Cc, dev=gpu, scale=1.5) - 0.2).to(torch.bfloat16)
    e = torch.empty(0, device=gpu)
    g, b = torch.rand(Cc, device=gpu) + 0.5, torch.randn(Cc, device=gpu)
    g2, b2 = torch.rand(Cc, device=gpu) + 0.5, torch.randn(Cc, device=gpu)
    rm, rv = torch.zeros(Cc, device=gpu), torch.ones(Cc, device=gpu)
    st2 = C().bn_stats(x2, e)
    mean2, rstd2, aff2 = C().bn_stats_affine(x2.reshape(M, Cc), st2, g2, b2, rm.clone(), rv.clone(),
                                             0.1, 1e-5, e)
    mask = torch.empty(M * Cc // 8, dtype=torch.uint8, device=gpu)
    y, mean, rstd = C().bn_fwd_train(x, e, g, b, rm, rv, 0.1, 1e-5, x2, True, e, mask,
                                     res_affine=aff2)
    dy = bf(M, Cc, dev=gpu)
    C().set_deterministic(1)  # fixed-order slab combine: the bitwise check below
    try:
        _bn_pair_checks(dy, x, x2, mask, mean, rstd, g, mean2, rstd2, g2, Cc, gpu)
    finally:
        C().set_deterministic(0)


def _bn_pair_checks(dy, x, x2, mask, mean, rstd, g, mean2, rstd2, g2, Cc, gpu):
    e = torch.empty(0, device=gpu)
    sk = [torch.zeros(Cc, device=gpu) for _ in range(4)]
    dx, dx2 = C().bn_bwd_pair(dy, x, mask, mean, rstd, g, sk[0], sk[1], x2, mean2, rstd2, g2,
                              sk[2], sk[3])
    rk = [torch.zeros(Cc, device=gpu) for _ in range(4)]
    rx, rx2 = ref.bn_bwd_pair(dy, x, mask, mean, rstd, g, rk[0], rk[1], x2, mean2, rstd2, g2,
                              rk[2], rk[3])
    tk = [torch.zeros(Cc, device=gpu) for _ in range(4)]
    tx, tg = C().bn_bwd(dy, x, e, mean, rstd, g, tk[0], tk[1], True, True, None, mask)
    tx2, _ = C().bn_bwd(tg, x2, e, mean2, rstd2, g2, tk[2], tk[3], True, False)
    torch.cuda.synchronize()
    assert rel(dx, rx) < 1e-2 and rel(dx2, rx2) < 1e-2
    for u, v in zip(sk, rk):
        assert rel(u, v) < 1e-3
    assert torch.equal(dx, tx)  # same sums, same apply arithmetic
    assert rel(dx2, tx2) < 1e-2  # (the two-stage form rounds g to bf16 first)


@pytest.mark.parametrize("N,H,W,Cc", [(2, 8, 10, 64), (4, 56, 56, 128), (1, 224, 224, 64)])
def test_maxpool2_fast_path_and_relu_handoff(gpu, N, H, W, Cc):
    """2x2/s2 max pool fast kernels == the generic window kernels' argmax encoding and the
    oracle (forward values, backward routing), and the ReLU-linked backward (mask from the
    pooled value, bias-gradient sums) == generic backward of the masked gradient."""
    torch.manual_seed(31)
    x = torch.relu(bf(N, H, W, Cc, dev=gpu)).to(torch.bfloat16)  # a ReLU output (ties at 0)
    y, idx = C().maxpool_fwd(x, 2, 2, 2, 2, 0, 0, False)
    yr, _ = ref.maxpool_fwd(x, 2, 2, 2, 2, 0, 0, False)
    assert torch.equal(y, yr.to(y.dtype))
    # generic kernels (3-wide window trick: kernel 2 via a non-fast shape is not reachable,
    # so check the encoding directly: tap a*2+b holds the max and is the first max)
    xv = x.float().reshape(N, H // 2, 2, W // 2, 2, Cc).permute(0, 1, 3, 2, 4, 5)
    xv = xv.reshape(N, H // 2, W // 2, 4, Cc)
    first = (xv == y.float().unsqueeze(3)).float().argmax(3)
    assert torch.equal(idx.long(), first)
    dy = bf(N, H // 2, W // 2, Cc, dev=gpu)
    dx = C().maxpool_bwd(dy, idx, H, W, 2, 2, 2, 2, 0, 0, False)
    exp = torch.zeros(N, H // 2, W // 2, 4, Cc, device=gpu)
    exp.scatter_(3, idx.long().unsqueeze(3), dy.float().unsqueeze(3))
    exp = exp.reshape(N, H // 2, W // 2, 2, 2, Cc).permute(0, 1, 3, 2, 4, 5).reshape(N, H, W, Cc)
    assert torch.equal(dx.float(), exp)
    dxr, sums = C().maxpool_bwd_relu(dy, idx, y, H, W, 2, 2, 2, 2, 0, 0)
    g = dy.float() * (y.float() > 0)
    dxm = C().maxpool_bwd(g.to(torch.bfloat16), idx, H, W, 2, 2, 2, 2, 0, 0, False)
    torch.cuda.synchronize()
    assert torch.equal(dxr, dxm)
    assert rel(sums, g.reshape(-1, Cc).sum(0)) < 1e-4
    assert C().maxpool_bwd_relu(dy, idx, y, H, W, 3, 3, 2, 2, 1, 1) is None


@pytest.mark.parametrize("M,Cc,Ctot", [(4096, 64, 96), (3001, 136, 256), (50000, 32, 32)])
def test_bn_channel_prefix_and_accumulate(gpu, M, Cc, Ctot):
    """DenseNet block buffer: BN (train / eval forward, z-mask backward) of the first Cc
    channels of a [M, Ctot] buffer with precomputed [2, Ctot] statistics == the same BN of
    a contiguous copy, bit for bit; bn_bwd(gacc=G) adds dx into G's first Cc channels in
    fp32 and leaves the rest untouched; bn_stats / chan_insert against the oracle."""
    torch.manual_seed(21)
    buf = (bf(M, Ctot, dev=gpu, scale=2.0) + 0.3).to(torch.bfloat16)
    xc = buf[:, :Cc].contiguous()
    S = C().bn_stats(buf, torch.empty(0, device=gpu))
    Sr = ref.bn_stats(buf)
    assert rel(S[0], Sr[0]) < 1e-3 and rel(S[1], Sr[1]) < 1e-3
    g = torch.rand(Cc, device=gpu) + 0.5
    b = torch.randn(Cc, device=gpu)
    e = torch.empty(0, device=gpu)
    rm, rv = torch.zeros(Cc, device=gpu), torch.ones(Cc, device=gpu)
    rm2, rv2 = rm.clone(), rv.clone()
    y, mean, rstd = C().bn_fwd_train(buf, S, g, b, rm, rv, 0.1, 1e-5, e, True, e, channels=Cc)
    y2, mean2, rstd2 = C().bn_fwd_train(xc, S[:, :Cc].contiguous(), g, b, rm2, rv2, 0.1, 1e-5, e,
                                        True, e)
    torch.cuda.synchronize()
    assert y.shape == (M, Cc) and torch.equal(y, y2) and torch.equal(rm, rm2)
    assert torch.equal(C().bn_fwd_eval(buf, g, b, rm, rv, 1e-5, e, True, channels=Cc),
                       C().bn_fwd_eval(xc, g, b, rm, rv, 1e-5, e, True))
    dy = bf(M, Cc, dev=gpu)
    G = torch.randn(M, Ctot, device=gpu)
    G0 = G.clone()
    dg, db = torch.zeros(Cc, device=gpu), torch.zeros(Cc, device=gpu)
    dg2, db2 = dg.clone(), db.clone()
    dx0, _ = C().bn_bwd(dy, buf, e, mean, rstd, g, dg, db, True, False, b, gacc=G)
    dx, _ = C().bn_bwd(dy, xc, e, mean2, rstd2, g, dg2, db2, True, False, b)
    torch.cuda.synchronize()
    assert dx0 is None or dx0.numel() == 0
    assert torch.equal(dg, dg2) and torch.equal(db, db2)
    assert torch.equal(G[:, Cc:], G0[:, Cc:])
    want = G0[:, :Cc] + dx.float()
    assert float((G[:, :Cc] - want).abs().max()) <= 1e-2 * float(dx.float().abs().max()) + 1e-6
    # bf16 accumulator (MPA_DENSE_GRAD_BF16): one bf16 rounding of (G + dx) per element
    G16 = torch.randn(M, Ctot, device=gpu).to(torch.bfloat16)
    G16_0 = G16.clone()
    C().bn_bwd(dy, buf, e, mean, rstd, g, torch.zeros_like(dg), torch.zeros_like(db), True,
               False, b, gacc=G16)
    torch.cuda.synchronize()
    assert torch.equal(G16[:, Cc:], G16_0[:, Cc:])
    want16 = G16_0[:, :Cc].float() + dx.float()
    assert float((G16[:, :Cc].float() - want16).abs().max()) <= 2e-2 * float(want16.abs().max())
    assert torch.equal(C().chan_slice(buf, 8, Cc - 8), buf[:, 8:Cc])
    # chan_insert: bf16 activations and fp32 rows
    dst = torch.zeros(M, Ctot + 32, dtype=torch.bfloat16, device=gpu)
    C().chan_insert(dst, 32, buf)
    st = torch.zeros(2, Ctot + 64, device=gpu)
    C().chan_insert(st, 64, S)
    torch.cuda.synchronize()
    assert torch.equal(dst[:, 32:], buf) and not dst[:, :32].any()
    assert torch.equal(st[:, 64:], S) and not st[:, :64].any()


def test_avgpool_channel_window(gpu):
    """3x3/s1 average pool of a channel window of a wider buffer (Inception's grouped pool
    branch) == the pool of a contiguous copy; the backward writes only its window."""
    torch.manual_seed(22)
    z = bf(4, 17, 17, 96, dev=gpu)
    win = z[..., 32:64]
    y = C().avgpool_fwd(win, 3, 3, 1, 1, 1, 1, False, True)
    y2 = C().avgpool_fwd(win.contiguous(), 3, 3, 1, 1, 1, 1, False, True)
    dy = bf(4, 17, 17, 32, dev=gpu)
    dz = torch.zeros(4, 17, 17, 96, dtype=torch.bfloat16, device=gpu)
    C().avgpool_bwd(dy, 17, 17, 3, 3, 1, 1, 1, 1, False, True, dx_out=dz[..., 32:64])
    dx2 = C().avgpool_bwd(dy, 17, 17, 3, 3, 1, 1, 1, 1, False, True)
    torch.cuda.synchronize()
    assert torch.equal(y, y2)
    assert torch.equal(dz[..., 32:64], dx2)
    assert not dz[..., :32].any() and not dz[..., 64:].any()


def test_zero_cols_and_bf16_add(gpu):
    """The two elementwise helpers that keep ATen out of the step: zero a column range of an
    fp32 [rows][period] view (stem gradient fix-up) and a += b in bf16 (GradJoin)."""
    t = torch.randn(64 * 7, 32, device=gpu)
    want = t.clone()
    want[:, 28:32] = 0
    C().zero_cols_f32(t, 32, 28, 4)
    a, b = bf(4096, 24, dev=gpu), bf(4096, 24, dev=gpu)
    want_ab = (a.float() + b.float()).to(torch.bfloat16)
    C().add_bf16_(a, b)
    torch.cuda.synchronize()
    assert torch.equal(t, want)
    assert torch.equal(a, want_ab)


def test_bn_stats_from_conv(gpu):
    """bn_fwd_train fed by conv epilogue statistics == standalone statistics."""
    torch.manual_seed(5)
    x = bf(4, 16, 16, 64, dev=gpu)
    w = bf(128, 3, 3, 64, dev=gpu, scale=0.05)
    st = torch.zeros(2, 128, device=gpu)
    z = C().conv_fwd(x, w, torch.empty(0, device=gpu), 1, 1, 1, 1, False, st,
                     torch.full((128,), 0.3, device=gpu))
    g, b = torch.ones(128, device=gpu), torch.zeros(128, device=gpu)
    e = torch.empty(0, device=gpu)
    y1 = C().bn_fwd_train(z, st, g, b, torch.zeros(128, device=gpu), torch.ones(128, device=gpu),
                          0.1, 1e-5, e, True)[0]
    y2 = C().bn_fwd_train(z, e, g, b, torch.zeros(128, device=gpu), torch.ones(128, device=gpu),
                          0.1, 1e-5, e, True)[0]
    assert rel(y1, y2) < 1e-2


@pytest.mark.parametrize("Cc", [64, 20])
def test_act_bwd(gpu, Cc):
    dy = bf(300, Cc, dev=gpu)
    y = bf(300, Cc, dev=gpu)
    db = torch.zeros(Cc, device=gpu)
    db2 = db.clone()
    g = C().act_bwd(dy, y, db)
    g2 = ref.act_bwd(dy, y, db2)
    assert rel(g, g2) < 1e-2 and rel(db, db2) < 1e-2


POOL_CASES = [
    (2, 112, 112, 64, 3, 3, 2, 2, 1, 1, False),   # resnet maxpool
    (2, 55, 55, 96, 3, 3, 2, 2, 0, 0, True),      # squeezenet ceil
    (2, 14, 14, 32, 2, 2, 2, 2, 0, 0, False),     # vgg
    (2, 9, 9, 12, 3, 3, 2, 2, 0, 0, False),       # scalar channels
]


@pytest.mark.parametrize("case", POOL_CASES)
def test_maxpool(gpu, case):
    N, H, W, Cc, kh, kw, sh, sw, ph, pw, ceil = case
    x = bf(N, H, W, Cc, dev=gpu)
    y, idx = C().maxpool_fwd(x, kh, kw, sh, sw, ph, pw, ceil)
    yr, idxr = ref.maxpool_fwd(x, kh, kw, sh, sw, ph, pw, ceil)
    assert y.shape == yr.shape and rel(y, yr) < 1e-6
    dy = bf(*y.shape, dev=gpu)
    dx = C().maxpool_bwd(dy, idx, H, W, kh, kw, sh, sw, ph, pw, ceil)
    dxr = ref.maxpool_bwd(dy, idxr, H, W, kh, kw, sh, sw, ph, pw, ceil)
    assert rel(dx, dxr) < 1e-2


def _global_idx(idx, H, W, kh, kw, sh, sw, ph, pw):
    """window-local argmax (native) -> flat h*W+w index (oracle's maxpool_bwd).  255 marks a
    ReLU-dead window (no argmax; it passes no gradient): mapped to the window's first
    in-bounds tap, where the oracle's ReLU-masked backward is zero as well."""
    N, P, Q, Cc = idx.shape
    p = torch.arange(P, device=idx.device).view(1, P, 1, 1)
    q = torch.arange(Q, device=idx.device).view(1, 1, Q, 1)
    first = (ph - p * sh).clamp(min=0) * kw + (pw - q * sw).clamp(min=0)
    t = idx.long()
    t = torch.where(t == 255, first.expand_as(t), t)
    i, k = t // kw, t % kw
    h = p * sh - ph + i
    w = q * sw - pw + k
    assert bool(((h >= 0) & (h < H) & (w >= 0) & (w < W)).all())
    return (h * W + w).to(torch.int32)


@pytest.mark.parametrize("case", [(4, 112, 112, 64, 3, 3, 2, 2, 1, 1, False),  # resnet stem
                                  (2, 55, 55, 96, 3, 3, 2, 2, 0, 0, True),     # ceil mode
                                  (2, 71, 71, 192, 3, 3, 2, 2, 0, 0, False),   # inception pool2
                                  (1, 147, 147, 64, 3, 3, 2, 2, 0, 0, False),  # inception pool1
                                  (2, 9, 13, 16, 3, 3, 2, 2, 0, 0, False),     # valid, H != W
                                  (2, 21, 17, 16, 3, 3, 2, 2, 1, 1, False)])
def test_bn_relu_maxpool_fused(gpu, case):
    """Fused stem BN+ReLU+max-pool (forward) and pool-gather+BN backward vs the oracle's
    bn -> relu -> maxpool composition.  The backward oracle routes the pooled gradient
    through the native argmax: values that tie after bf16 rounding may legitimately pick
    a different window element."""
    N, H, W, Cc, kh, kw, sh, sw, ph, pw, ceil = case
    torch.manual_seed(11)
    z = bf(N, H, W, Cc, dev=gpu, scale=1.5) + 0.2
    z = z.to(torch.bfloat16)
    st = torch.stack([z.float().reshape(-1, Cc).mean(0), z.float().reshape(-1, Cc).var(0, unbiased=False)])
    g = torch.rand(Cc, device=gpu) + 0.5
    b = torch.randn(Cc, device=gpu) * 0.5
    rm, rv = torch.zeros(Cc, device=gpu), torch.ones(Cc, device=gpu)
    rm2, rv2 = rm.clone(), rv.clone()
    cnt = torch.tensor(3, dtype=torch.long, device=gpu)
    y, idx, mean, rstd = C().bn_relu_maxpool_fwd(z, st, g, b, rm, rv, 0.1, 1e-5, kh, kw, sh, sw,
                                                 ph, pw, ceil, cnt)
    yr, _, meanr, rstdr = ref.bn_relu_maxpool_fwd(z, st, g, b, rm2, rv2, 0.1, 1e-5, kh, kw, sh,
                                                  sw, ph, pw, ceil)
    assert int(cnt) == 4
    assert y.shape == yr.shape and rel(y, yr) < 1e-2
    assert rel(mean, meanr) < 1e-3 and rel(rstd, rstdr) < 1e-3
    assert rel(rm, rm2) < 1e-3 and rel(rv, rv2) < 1e-3
    gi = _global_idx(idx, H, W, kh, kw, sh, sw, ph, pw)
    # the argmax points at a maximal element of relu(bn(z)) in its window
    yfull = torch.relu((z.float() - mean) * (rstd * g) + b)
    picked = torch.gather(yfull.permute(0, 3, 1, 2).reshape(N, Cc, -1), 2,
                          gi.permute(0, 3, 1, 2).reshape(N, Cc, -1).long())
    assert rel(picked.reshape(N, Cc, *y.shape[1:3]).permute(0, 2, 3, 1), y) < 1e-2
    dp = bf(*y.shape, dev=gpu)
    dg, db = torch.zeros(Cc, device=gpu), torch.zeros(Cc, device=gpu)
    dg2, db2 = dg.clone(), db.clone()
    dz = C().maxpool_bn_bwd(dp, idx, z, mean, rstd, g, b, dg, db, kh, kw, sh, sw, ph, pw)
    dzr = ref.maxpool_bn_bwd(dp, gi, z, mean, rstd, g, b, dg2, db2, kh, kw, sh, sw, ph, pw)
    assert rel(dz, dzr) < 2e-2
    assert rel(dg, dg2) < 1e-2 and rel(db, db2) < 1e-2
    # pooled-only reduction: the forward's zsel (raw z at each argmax) is exactly z gathered
    # at the argmax, and the backward through it matches the full-z reduction
    zsel = torch.empty_like(y)
    rm3, rv3 = torch.zeros(Cc, device=gpu), torch.ones(Cc, device=gpu)
    y3, idx3, _, _ = C().bn_relu_maxpool_fwd(z, st, g, b, rm3, rv3, 0.1, 1e-5, kh, kw, sh, sw,
                                             ph, pw, ceil, zsel_out=zsel)
    assert torch.equal(y3, y) and torch.equal(idx3, idx)
    zg = torch.gather(z.permute(0, 3, 1, 2).reshape(N, Cc, -1), 2,
                      gi.permute(0, 3, 1, 2).reshape(N, Cc, -1).long())
    assert torch.equal(zg.reshape(N, Cc, *y.shape[1:3]).permute(0, 2, 3, 1), zsel)
    dg3, db3 = torch.zeros(Cc, device=gpu), torch.zeros(Cc, device=gpu)
    dz3 = C().maxpool_bn_bwd(dp, idx, z, mean, rstd, g, b, dg3, db3, kh, kw, sh, sw, ph, pw,
                             zsel=zsel)
    assert rel(dz3, dz) < 1e-2 and rel(dz3, dzr) < 2e-2
    assert rel(dg3, dg) < 1e-4 and rel(db3, db) < 1e-4


@pytest.mark.parametrize("N,P,Q,ties", [(2, 112, 112, False), (3, 64, 64, False),
                                         (2, 56, 56, False), (1, 32, 40, False),
                                         (2, 56, 56, True)])
def test_stem_pool_wgrad(gpu, N, P, Q, ties):
    """Fused stem backward (round 6): the pooled-only sums + the weight gradient that forms
    dz = a g + b + cco z in its operand staging (conv_stem.hip, POOL form) against the
    two-pass form (maxpool_bn_bwd writes dz, conv_wgrad reads it: the same bf16 dz, so
    equal to fp32 summation order) and the fp32 oracle.  Channels with gamma < 0, the
    K-step tail rows (2Q % 32 != 0) and the last window row / column are covered; `ties`
    quantises z to halves, so most windows hold tied maxima (the forward's argmax tap is
    the one every form follows)."""
    torch.manual_seed(21)
    Cc = 64
    x = bf(N, 2 * (P - 1) + 7, Q + 3, 8, dev=gpu, scale=0.5)
    z = (bf(N, P, Q, Cc, dev=gpu, scale=1.5) + 0.2).to(torch.bfloat16)
    if ties:
        z = (z.float() * 2).round().div(2).to(torch.bfloat16)
    st = torch.stack([z.float().reshape(-1, Cc).mean(0),
                      z.float().reshape(-1, Cc).var(0, unbiased=False)])
    g = torch.rand(Cc, device=gpu) + 0.5
    g[::3] *= -1.0                                        # gamma < 0 channels
    b = torch.randn(Cc, device=gpu) * 0.5
    rm, rv = torch.zeros(Cc, device=gpu), torch.ones(Cc, device=gpu)
    zsel = torch.empty(N, P // 2, Q // 2, Cc, device=gpu, dtype=torch.bfloat16)
    y, idx, mean, rstd = C().bn_relu_maxpool_fwd(z, st, g, b, rm, rv, 0.1, 1e-5, 3, 3, 2, 2, 1,
                                                 1, False, zsel_out=zsel)
    dp = bf(*y.shape, dev=gpu)
    assert C().stem_pool_wgrad_ok(dp, idx, z, x, torch.zeros(64, 7, 4, 8, device=gpu),
                                  2, 1, 0, 0)
    # two-pass form
    dg0, db0 = torch.zeros(Cc, device=gpu), torch.zeros(Cc, device=gpu)
    dz = C().maxpool_bn_bwd(dp, idx, z, mean, rstd, g, b, dg0, db0, 3, 3, 2, 2, 1, 1, zsel=zsel)
    dw0 = torch.zeros(64, 7, 4, 8, device=gpu)
    C().conv_wgrad(dz, x, dw0, 2, 1, 0, 0)
    # fused form (accumulating into a non-zero gradient, and overwriting)
    dg1, db1 = torch.zeros(Cc, device=gpu), torch.zeros(Cc, device=gpu)
    sums = C().maxpool_bn_bwd_sums(dp, zsel, mean, rstd, g, b, dg1, db1)
    dw1 = torch.full((64, 7, 4, 8), 0.25, device=gpu)
    C().stem_pool_wgrad(dp, idx, z, mean, rstd, g, b, sums, x, dw1, 2, 1, 0, 0, False)
    dw2 = torch.full((64, 7, 4, 8), 7.0, device=gpu)
    C().stem_pool_wgrad(dp, idx, z, mean, rstd, g, b, sums, x, dw2, 2, 1, 0, 0, True)
    torch.cuda.synchronize()
    assert torch.equal(dg1, dg0) and torch.equal(db1, db0)
    assert torch.isfinite(dw2).all()
    assert rel(dw2, dw0) < 1e-4, rel(dw2, dw0)
    assert rel(dw1 - 0.25, dw0) < 1e-4
    # fp32 oracle (its own argmax convention: the native window taps as global indices)
    gi = _global_idx(idx, P, Q, 3, 3, 2, 2, 1, 1)
    dwr = torch.zeros(64, 7, 4, 8, device=gpu)
    ref.stem_pool_wgrad(dp, gi, z, mean, rstd, g, b, sums, x, dwr, 2, 1, 0, 0, True)
    assert rel(dw2, dwr) < 1e-2, rel(dw2, dwr)


@pytest.mark.parametrize("case", POOL_CASES + [(2, 35, 35, 64, 3, 3, 1, 1, 1, 1, False),
                                               (2, 17, 17, 64, 5, 5, 3, 3, 0, 0, False)])
@pytest.mark.parametrize("cip", [True, False])
def test_avgpool(gpu, case, cip):
    N, H, W, Cc, kh, kw, sh, sw, ph, pw, ceil = case
    x = bf(N, H, W, Cc, dev=gpu)
    y = C().avgpool_fwd(x, kh, kw, sh, sw, ph, pw, ceil, cip)
    yr = ref.avgpool_fwd(x, kh, kw, sh, sw, ph, pw, ceil, cip)
    assert y.shape == yr.shape and rel(y, yr) < 1e-2
    dy = bf(*y.shape, dev=gpu)
    dx = C().avgpool_bwd(dy, H, W, kh, kw, sh, sw, ph, pw, ceil, cip)
    assert rel(dx, ref.avgpool_bwd(dy, H, W, kh, kw, sh, sw, ph, pw, ceil, cip)) < 1e-2


@pytest.mark.parametrize("shape,out", [((2, 7, 7, 512), (1, 1)), ((2, 13, 13, 100), (1, 1)),
                                       ((2, 14, 14, 64), (7, 7)), ((2, 13, 13, 16), (6, 6)),
                                       ((2, 5, 5, 8), (7, 7))])
def test_adaptive_avgpool(gpu, shape, out):
    x = bf(*shape, dev=gpu)
    y = C().adaptive_avgpool_fwd(x, *out)
    assert rel(y, ref.adaptive_avgpool_fwd(x, *out)) < 1e-2
    dy = bf(*y.shape, dev=gpu)
    dx = C().adaptive_avgpool_bwd(dy, shape[1], shape[2])
    assert rel(dx, ref.adaptive_avgpool_bwd(dy, shape[1], shape[2])) < 1e-2


def test_cross_entropy_padded_rows(gpu):
    """Classifier heads store 64,512 rows for 64,500 classes: CE / argmax read the padded
    row stride, and the backward returns a view of a zero-padded buffer that the Linear
    backward consumes in place (no pad copy)."""
    from mpi_pytorch_amd.ops.functional import _padded_grad
    torch.manual_seed(8)
    B, NC, LD = 64, 64500, 64512
    full = bf(B, LD, dev=gpu, scale=3.0)
    logits = full[:, :NC]
    labels = torch.randint(0, NC, (B,), device=gpu)
    loss, lse = C().ce_fwd(logits, labels)
    lr, lser = ref.ce_fwd(logits, labels)
    assert rel(loss, lr) < 1e-3 and rel(lse, lser) < 1e-3
    go = torch.ones(1, device=gpu)
    d = C().ce_bwd(logits, labels, lse, go)
    assert d.shape == (B, NC) and d.stride(0) == LD
    assert rel(d, ref.ce_bwd(logits, labels, lser, go)) < 2e-2
    base = _padded_grad(d, LD)
    assert base.data_ptr() == d.data_ptr() and base.shape == (B, LD)  # no copy
    assert float(base[:, NC:].float().abs().max()) == 0.0
    cnt = torch.zeros(1, dtype=torch.long, device=gpu)
    C().argmax_correct(logits, logits.float().argmax(1), cnt)
    assert int(cnt) == B


@pytest.mark.parametrize("B,NC", [(128, 64500), (7, 1000), (5, 33)])
def test_cross_entropy(gpu, B, NC):
    logits = bf(B, NC, dev=gpu, scale=3.0)
    labels = torch.randint(0, NC, (B,), device=gpu)
    loss, lse = C().ce_fwd(logits, labels)
    lr_, lser = ref.ce_fwd(logits, labels)
    assert abs(float(loss) - float(lr_)) < 1e-3 * max(1.0, abs(float(lr_)))
    assert rel(lse, lser) < 1e-4
    go = torch.full((1,), 0.7, device=gpu)
    d = C().ce_bwd(logits, labels, lse, go)
    assert rel(d, ref.ce_bwd(logits, labels, lser, go)) < 2e-2
    cnt = torch.zeros(1, dtype=torch.int64, device=gpu)
    cnt2 = cnt.clone()
    logits2 = logits.clone()
    logits2[torch.arange(B), labels] = 100.0
    logits2[0, (int(labels[0]) + 1) % NC] = 200.0
    C().argmax_correct(logits2, labels, cnt)
    ref.argmax_correct(logits2, labels, cnt2)
    assert int(cnt) == int(cnt2) == B - 1


def test_adam_sgd(gpu):
    n = 4096 + 64
    for kind in ("adam", "sgd"):
        p = torch.randn(n, device=gpu)
        g = torch.randn(n, device=gpu)
        s1 = torch.zeros(n, device=gpu)
        s2 = torch.zeros(n, device=gpu)
        sh = torch.zeros(n, dtype=torch.bfloat16, device=gpu)
        p2, s1b, s2b, shb = p.clone(), s1.clone(), s2.clone(), sh.clone()
        for it in range(3):
            st = torch.full((1,), float(it), device=gpu)
            if kind == "adam":
                C().adam_step(p, g, s1, s2, sh, st, 1e-2, 0.9, 0.999, 1e-8, 0.01, 0.5)
                ref.adam_step(p2, g, s1b, s2b, shb, st, 1e-2, 0.9, 0.999, 1e-8, 0.01, 0.5)
            else:
                C().sgd_step(p, g, s1, sh, st, 1e-2, 0.9, 0.0, 0.01, it == 1, 0.5)
                ref.sgd_step(p2, g, s1b, shb, st, 1e-2, 0.9, 0.0, 0.01, it == 1, 0.5)
        assert rel(p, p2) < 1e-5
        assert rel(sh.float(), p2) < 1e-2


@pytest.mark.parametrize("mode", [0, 2])
@pytest.mark.parametrize("src,dst", [((64, 80), (32, 32)), ((224, 224), (224, 224)),
                                     ((100, 60), (128, 128)),
                                     ((30, 61), (20, 40)),      # 3W % 4 != 0: byte staging
                                     ((12, 1400), (8, 16))])    # W > 1344: unstaged taps
def test_preprocess(gpu, mode, src, dst):
    img = torch.randint(0, 256, (2, src[0], src[1], 3), dtype=torch.uint8, device=gpu)
    mean, std = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)
    out = C().preprocess(img, dst[0], dst[1], list(mean), list(std), mode, 8)
    r = ref.preprocess(img, dst[0], dst[1], mean, std, mode, 8, torch.float32)
    assert out.shape == (2, dst[0], dst[1], 8)
    assert float((out.float() - r).abs().max()) < 0.05
    assert float(out[..., 3:].float().abs().max()) == 0.0


@pytest.mark.parametrize("mode", [0, 2])
@pytest.mark.parametrize("cpad,pad", [(4, (3, 3, 3, 3)), (4, (0, 0, 0, 1)), (8, (1, 2, 3, 4)),
                                      (3, (2, 0, 0, 2))])
def test_preprocess_canvas(gpu, mode, cpad, pad):
    """Zero-bordered canvas output (pixel-pair stem layout): 8-B stores for 4 channels,
    16-B for 8, scalar otherwise; border and padding channels exactly zero."""
    img = torch.randint(0, 256, (2, 50, 60, 3), dtype=torch.uint8, device=gpu)
    mean, std = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)
    out = C().preprocess(img, 40, 44, list(mean), list(std), mode, cpad, list(pad))
    r = ref.preprocess(img, 40, 44, mean, std, mode, cpad, torch.float32, pad)
    t, b, l, rr = pad
    assert out.shape == (2, 40 + t + b, 44 + l + rr, cpad)
    assert float((out.float() - r).abs().max()) < 0.05
    if cpad > 3:
        assert float(out[..., 3:].float().abs().max()) == 0.0
    inner = torch.zeros_like(out, dtype=torch.bool)
    inner[:, t:t + 40, l:l + 44] = True
    assert float(out.float().masked_fill(inner, 0).abs().max()) == 0.0


@pytest.mark.parametrize("hw,pad", [((224, 224), (3, 2, 3, 3)), ((37, 20), (3, 3, 3, 3)),
                                    ((8, 300), (0, 1, 2, 0))])
def test_preprocess_identity_copy(gpu, hw, pad):
    """Identity-size training preprocess (preprocess_copy4_kernel): bitwise equal to the
    bilinear kernel (its weights are exactly 0 / 1 at scale 1), zero border and padding
    channel; W = 300 makes a row need more than one pass of the 64 lanes."""
    H, W = hw
    img = torch.randint(0, 256, (3, H, W, 3), dtype=torch.uint8, device=gpu)
    mean, std = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)
    outs = []
    for on in (1, 0):
        C().preprocess_set_copy(on)
        outs.append(C().preprocess(img, H, W, list(mean), list(std), 0, 4, list(pad)))
    C().preprocess_set_copy(1)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    r = ref.preprocess(img, H, W, mean, std, 0, 4, torch.float32, pad)
    assert float((outs[0].float() - r).abs().max()) < 0.05


def test_dropout(gpu):
    x = torch.ones(1 << 16, device=gpu, dtype=torch.bfloat16)
    y, m = C().dropout_fwd(x, 0.5, 7, 1)
    keep = m.float().mean().item()
    assert 0.47 < keep < 0.53
    assert torch.allclose(y.float(), m.float() * 2.0)
    y2, m2 = C().dropout_fwd(x, 0.5, 7, 2)
    assert not torch.equal(m, m2)
    dx = C().dropout_bwd(torch.ones_like(x), m, 0.5)
    assert torch.allclose(dx.float(), m.float() * 2.0)


@pytest.mark.parametrize("chans", [[64, 32], [256] + [32] * 24 + [32] * 9, [96, 64, 8, 192]])
def test_concat_split_channels(gpu, chans):
    """Native NHWC channel concat / split (concat.hip) against torch.cat / torch.split;
    34 segments exercise the multi-launch path (CAT_MAXSEG = 32)."""
    xs = [bf(3, 7, 5, c, dev=gpu) for c in chans]
    y = C().concat_channels(xs)
    assert torch.equal(y, ref.concat_channels(xs))
    dy = bf(3, 7, 5, sum(chans), dev=gpu)
    for a, b in zip(C().split_channels(dy, chans), ref.split_channels(dy, chans)):
        assert a.is_contiguous() and torch.equal(a, b)


def test_cat_channels_autograd(gpu):
    from mpi_pytorch_amd.ops import functional as Fn
    xs = [bf(2, 4, 4, c, dev=gpu).requires_grad_() for c in (16, 24)]
    y = Fn.cat_channels(xs)
    g = bf(*y.shape, dev=gpu)
    y.backward(g)
    assert torch.equal(y.detach(), torch.cat([x.detach() for x in xs], -1))
    assert torch.equal(xs[0].grad, g[..., :16]) and torch.equal(xs[1].grad, g[..., 16:])


@pytest.mark.parametrize("N,P,Q", [(3, 13, 37), (2, 16, 112), (1, 112, 112), (8, 112, 112)])
def test_conv_stem_direct(gpu, N, P, Q):
    """Direct row-staged pixel-pair stem (conv_stem.hip) vs the implicit-GEMM engine on the
    same super-tap layout: same K order, so bitwise-equal outputs; BN statistics (shifted
    sums, different summation order) to fp32 rounding; and the fp32 oracle.  P % 8 != 0 and
    Q % 16 != 0 exercise the partial item / partial subtile paths."""
    torch.manual_seed(5)
    x = bf(N, 2 * (P - 1) + 7, Q + 3, 8, dev=gpu, scale=0.5)
    w = bf(64, 7, 4, 8, dev=gpu, scale=0.05)
    e = torch.empty(0, device=gpu)
    shift = torch.randn(64, device=gpu) * 0.1
    outs = []
    for on in (1, 0):
        C().igemm_set_stem(on)
        st = torch.empty(2, 64, device=gpu)
        y = C().conv_fwd(x, w, e, 2, 1, 0, 0, False, st, shift)
        outs.append((y, st))
    C().igemm_set_stem(1)
    (y1, s1), (y0, s0) = outs
    assert y1.shape == (N, P, Q, 64)
    assert torch.equal(y1, y0)
    assert rel(s1, s0) < 1e-4
    yr = ref.conv_fwd(x, w, e, 2, 1, 0, 0, False, None, None)
    assert rel(y1, yr) < 1e-2
    yf = y1.float().reshape(-1, 64)
    assert rel(s1[0], yf.mean(0)) < 1e-3 and rel(s1[1], yf.var(0, unbiased=False)) < 1e-3


@pytest.mark.parametrize("N,P,Q", [(96, 112, 112), (3, 13, 37), (2, 8, 117)])
def test_conv_stem_wgrad_plan(gpu, N, P, Q):
    """Pixel-pair stem weight gradient: the halo-staged stem kernel (conv_stem.hip, items of
    two output rows; odd P and 2Q % 32 != 0 exercise the zero-padded item tails) vs the fp32
    oracle, and - with the stem kernels off - the GEMM plan at a production pixel count (two
    64x128 column tiles, split slab, the incremental-pixel DMA kernel with stride (2, 1))
    and the forced 64x256 / 64x128 single-split tiles (fp32 rounding only)."""
    torch.manual_seed(7)
    x = bf(N, 2 * (P - 1) + 7, Q + 3, 8, dev=gpu, scale=0.5)
    dy = bf(N, P, Q, 64, dev=gpu, scale=0.1)

    def run():
        dw = torch.zeros(64, 7, 4, 8, device=gpu)
        C().conv_wgrad(dy, x, dw, 2, 1, 0, 0)
        return dw

    prev = C().igemm_engine()
    try:
        C().igemm_set_engine(1)
        C().igemm_force_tile(0, 0, 0)
        halo = run()
        C().igemm_set_stem(0)
        gemm = run()
        forced = []
        if N * P * Q >= (1 << 20):
            for bm, bn in ((64, 256), (64, 128)):
                C().igemm_force_tile(bm, bn, 1)
                forced.append(run())
    finally:
        C().igemm_set_stem(1)
        C().igemm_force_tile(0, 0, 0)
        C().igemm_set_engine(prev)
    dwr = torch.zeros(64, 7, 4, 8, device=gpu)
    ref.conv_wgrad(dy, x, dwr, 2, 1, 0, 0)
    torch.cuda.synchronize()
    assert torch.isfinite(halo).all()
    assert rel(halo, dwr) < 1e-2
    assert rel(halo, gemm) < 1e-4
    for f in forced:
        assert rel(f, gemm) < 1e-4 and rel(f, dwr) < 1e-2
    if forced:
        assert rel(forced[0], forced[1]) < 1e-5


@pytest.mark.parametrize("reserve", [8, 40])
def test_comm_reserve_grids(gpu, reserve):
    """Comm-aware persistent grids (set_comm_reserve, parallel/ddp.py): with CUs reserved
    for an overlapping collective, the halo fwd / dgrad / wgrad and the stem fwd / wgrad
    launch fewer persistent blocks; every output tile is computed the same way (outputs
    bitwise equal), only the per-block statistics / weight-gradient partials are summed in
    another order (fp32 rounding)."""
    torch.manual_seed(41)
    e = torch.empty(0, device=gpu)
    full = C().active_cus()
    assert C().comm_reserve() == 0

    def halo_run(N, H, W, Cc, K):
        x = bf(N, H, W, Cc, dev=gpu)
        w = bf(K, 3, 3, Cc, dev=gpu, scale=1.0 / math.sqrt(9 * Cc))
        wt = w.permute(3, 1, 2, 0).reshape(Cc, 9, K).contiguous()
        dy = bf(N, H, W, K, dev=gpu)
        shift = torch.randn(K, device=gpu) * 0.1

        def run():
            st = torch.zeros(2, K, device=gpu)
            y = C().conv_fwd(x, w, e, 1, 1, 1, 1, False, st, shift)
            dx = C().conv_dgrad(dy, w, H, W, 1, 1, 1, 1, wt)
            dw = torch.zeros(K, 3, 3, Cc, device=gpu)
            C().conv_wgrad(dy, x, dw, 1, 1, 1, 1)
            return y, st, dx, dw
        return run

    def stem_run(N, P, Q):
        x = bf(N, 2 * (P - 1) + 7, Q + 3, 8, dev=gpu, scale=0.5)
        w = bf(64, 7, 4, 8, dev=gpu, scale=0.05)
        dy = bf(N, P, Q, 64, dev=gpu, scale=0.1)
        shift = torch.randn(64, device=gpu) * 0.1

        def run():
            st = torch.empty(2, 64, device=gpu)
            y = C().conv_fwd(x, w, e, 2, 1, 0, 0, False, st, shift)
            dw = torch.zeros(64, 7, 4, 8, device=gpu)
            C().conv_wgrad(dy, x, dw, 2, 1, 0, 0)
            return y, st, dw
        return run

    C().igemm_set_halo(1)
    cases = [halo_run(25, 56, 56, 64, 64), halo_run(52, 14, 14, 256, 512),
             halo_run(3, 9, 11, 96, 128)]
    stem = stem_run(8, 112, 112)
    base = [f() for f in cases] + [stem()]
    torch.cuda.synchronize()
    try:
        C().set_comm_reserve(reserve)
        assert C().comm_reserve() == reserve
        assert C().active_cus() == max(8, (full - reserve) // 8 * 8)
        got = [f() for f in cases] + [stem()]
        torch.cuda.synchronize()
    finally:
        C().set_comm_reserve(0)
    assert C().active_cus() == full
    for (y0, s0, dx0, dw0), (y1, s1, dx1, dw1) in zip(base[:3], got[:3]):
        assert torch.equal(y0, y1) and torch.equal(dx0, dx1)
        assert rel(s1, s0) < 1e-4 and rel(dw1, dw0) < 1e-4
    (y0, s0, dw0), (y1, s1, dw1) = base[3], got[3]
    assert torch.equal(y0, y1) and rel(s1, s0) < 1e-4 and rel(dw1, dw0) < 1e-4


@pytest.mark.parametrize("kind", ["linear", "halo", "strided", "stem"])
def test_wgrad_overwrite(gpu, kind):
    """overwrite=True (the first gradient since zero_grad, ParamArena.take_fresh): the
    weight gradient is stored over whatever dw held and equals accumulating into zeros;
    overwrite=False still accumulates."""
    torch.manual_seed(43)
    if kind == "linear":
        dy, x = bf(512, 4096, dev=gpu, scale=0.1), bf(512, 512, dev=gpu)
        shape = (4096, 512)
        run = lambda dw, ow: C().linear_wgrad(dy, x, dw, overwrite=ow)
    elif kind == "stem":
        x = bf(4, 2 * 27 + 7, 28 + 3, 8, dev=gpu, scale=0.5)
        dy = bf(4, 28, 28, 64, dev=gpu, scale=0.1)
        shape = (64, 7, 4, 8)
        run = lambda dw, ow: C().conv_wgrad(dy, x, dw, 2, 1, 0, 0, overwrite=ow)
    else:
        st = 1 if kind == "halo" else 2
        x = bf(6, 28, 28, 128, dev=gpu)
        dy = bf(6, 28 // st, 28 // st, 128, dev=gpu, scale=0.1)
        shape = (128, 3, 3, 128)
        run = lambda dw, ow: C().conv_wgrad(dy, x, dw, st, st, 1, 1, overwrite=ow)
    zero = torch.zeros(shape, device=gpu)
    run(zero, False)
    junk = torch.randn(shape, device=gpu) * 1e3
    over = junk.clone()
    run(over, True)
    acc = junk.clone()
    run(acc, False)
    torch.cuda.synchronize()
    assert torch.equal(over, zero)
    assert rel(acc - junk, zero) < 1e-3




@pytest.mark.parametrize("N", [4, 2])
def test_halo_mi7_tiles_bitwise(gpu, N):
    """448-pixel halo tiles (8 whole 56-wide rows per tile, MI = 7, round 6) vs the 256-pixel
    tiles on ResNet layer1's shape: every output accumulates its taps and chunks in the same
    order, so forward, dgrad and accumulating dgrad are bitwise equal; the BN statistics
    (different summation order) agree to fp32 rounding; and the fp32 oracle."""
    torch.manual_seed(17)
    H, Ci, Co = 56, 64, 64
    x = bf(N, H, H, Ci, dev=gpu)
    w = bf(Co, 3, 3, Ci, dev=gpu, scale=0.05)
    dy = bf(N, H, H, Co, dev=gpu)
    e = torch.empty(0, device=gpu)
    shift = torch.randn(Co, device=gpu) * 0.1
    out = {}
    try:
        for on in (0, 1):
            C().igemm_set_halo_mi7(on)
            st = torch.empty(2, Co, device=gpu)
            y = C().conv_fwd(x, w, e, 1, 1, 1, 1, False, st, shift)
            dx = C().conv_dgrad(dy, w, H, H, 1, 1, 1, 1)
            acc = x.clone()
            dxa = C().conv_dgrad(dy, w, H, H, 1, 1, 1, 1, None, acc)
            out[on] = (y, st, dx, dxa)
    finally:
        C().igemm_set_halo_mi7(1)
    (y0, s0, d0, a0), (y1, s1, d1, a1) = out[0], out[1]
    assert torch.equal(y0, y1) and torch.equal(d0, d1) and torch.equal(a0, a1)
    assert rel(s1, s0) < 1e-5
    assert rel(y1, ref.conv_fwd(x, w, e, 1, 1, 1, 1, False, None, None)) < 1e-2
    assert rel(d1, ref.conv_dgrad(dy, w, H, H, 1, 1, 1, 1)) < 1e-2


@pytest.mark.parametrize("N,HW", [(3, 224), (2, 128), (1, 64)])
def test_stem_pool_fused_forward(gpu, N, HW):
    """Fused stem forward (round 6): the 3x3/s2/p1 max-pool taken inside the pixel-pair stem
    conv kernel (conv_stem.hip PF, items of 8 output rows; an item's first pooled row merged
    with the previous item's bottom row by stem_pool_apply) vs the two-pass form (conv_fwd +
    bn_relu_maxpool_fwd).  z and y are bitwise equal; the argmax tap and the selected z
    agree wherever relu(bn(z)) > 0 (where it is 0 the two forms may pick different zeros,
    which carry no gradient); gamma < 0 channels select the window minimum.  (Opt-in,
    MPA_STEM_POOL_FWD=1: slower than the two-pass form, profiles/stem_pool_r6.txt.)"""
    from mpi_pytorch_amd.models.layers import Conv2d
    torch.manual_seed(9)
    P = HW // 2
    x = bf(N, 2 * (P - 1) + 7, P + 3, 8, dev=gpu, scale=0.5)
    w = bf(64, 7, 4, 8, dev=gpu, scale=0.05)
    g = torch.rand(64, device=gpu) + 0.5
    g[1::4] *= -1.0
    b = torch.randn(64, device=gpu) * 0.3
    shift = torch.randn(64, device=gpu) * 0.05
    out = []
    for fused in (True, False):
        rm, rv = torch.zeros(64, device=gpu), torch.ones(64, device=gpu)
        cnt = torch.zeros((), dtype=torch.long, device=gpu)
        st = torch.empty(2, 64, device=gpu)
        if fused:
            r = C().conv_stem_pool_fwd(x, w, 2, 1, 0, 0, st, shift, g, b, rm, rv, 0.1, 1e-5, cnt)
            assert r is not None
            y, idx, mean, rstd, z, zsel = r
        else:
            z = C().conv_fwd(x, w, torch.empty(0, device=gpu), 2, 1, 0, 0, False, st, shift)
            zsel = torch.empty(N, P // 2, P // 2, 64, device=gpu, dtype=torch.bfloat16)
            y, idx, mean, rstd = C().bn_relu_maxpool_fwd(z, st, g, b, rm, rv, 0.1, 1e-5, 3, 3, 2,
                                                         2, 1, 1, False, cnt, zsel_out=zsel)
        out.append((y, idx, mean, rstd, z, zsel, rm, rv, int(cnt)))
    (y1, i1, m1, r1, z1, s1, rm1, rv1, c1), (y0, i0, m0, r0, z0, s0, rm0, rv0, c0) = out
    assert torch.equal(z1, z0)
    assert rel(m1, m0) < 1e-4 and rel(r1, r0) < 1e-4 and rel(rm1, rm0) < 1e-4
    assert rel(rv1, rv0) < 1e-4 and c1 == c0 == 1
    assert rel(y1.float(), y0.float()) < 1e-3
    live = y0 > 0
    assert float(live.float().mean()) > 0.2
    assert torch.equal(i1[live], i0[live]) and torch.equal(s1[live], s0[live])
    # the selected z is an extreme of its window in the gamma-signed order (oracle)
    gi = _global_idx(i1, P, P, 3, 3, 2, 2, 1, 1)
    zr = z1.float().permute(0, 3, 1, 2).reshape(N, 64, -1)
    picked = torch.gather(zr, 2, gi.permute(0, 3, 1, 2).reshape(N, 64, -1).long())
    # (ReLU-dead windows carry the argmax byte 255: no tap to check there)
    assert torch.equal(picked.reshape(N, 64, P // 2, P // 2).permute(0, 2, 3, 1)[live],
                       s1.float()[live])
    assert bool((i1[~live] == 255).all())
    sgn = torch.where(g < 0, -1.0, 1.0).view(1, 64, 1, 1)
    pooled = torch.nn.functional.max_pool2d((zr.reshape(N, 64, P, P) * sgn), 3, 2, 1)
    assert torch.equal(pooled * sgn, s1.float().permute(0, 3, 1, 2))
