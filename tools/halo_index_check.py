"""Host emulation of conv_halo.hip's index math (no GPU): for every 256-pixel tile, fill the
LDS halo image exactly as the DMA lanes do (slot / column / separator mapping with the
magic-number divisions) and check that every fragment read of every tap lands inside the
576-pixel image on the right input pixel (or on a zero).  Run before launching a changed
kernel:  python tools/halo_index_check.py"""
import itertools


def magic(d):
    return (1 << 32) // d + 1


def udiv(n, m):
    return (n * m) >> 32


def check(N, H, W, BM=256, HPX=576, pitch=None):
    HW, W2 = H * W, (pitch(W) if pitch else W + 2)
    M = N * HW
    rows = (BM - 1 + W - 1) // W + 1
    seps = (BM - 1) // HW + 1
    if (rows + 2 + seps) * W2 + (1 if W2 == W + 1 else 0) > HPX:
        return "not eligible"
    mw2, mh1, mhw, mw = magic(W2), magic(H + 1), magic(HW), magic(W)
    for mt in range((M + BM - 1) // BM):
        m0 = mt * BM
        img0 = m0 // HW
        oh0 = (m0 - img0 * HW) // W
        lds = {}
        for hp in range(HPX):
            s = udiv(hp, mw2)
            col = hp - s * W2 - 1
            v = s + oh0 - 1
            d = udiv(v + H + 1, mh1) - 1
            row = v - d * (H + 1)
            img = img0 + d
            lds[hp] = (img, row, col) if (row < H and 0 <= col < W and img < N) else None
        lds[HPX] = "outside the halo image"
        r0 = m0 - img0 * HW
        mlast = M - 1 - img0 * HW
        for rel in range(BM):
            n = min(r0 + rel, mlast)
            di = udiv(n, mhw)
            rem = n - di * HW
            oh = udiv(rem, mw)
            ow = rem - oh * W
            assert di == n // HW and oh == rem // W
            hpb = ((di * (H + 1) + oh) - oh0 + 1) * W2 + ow + 1
            for dh, dw in itertools.product((-1, 0, 1), repeat=2):
                hp = hpb + dh * W2 + dw
                assert 0 <= hp < HPX, (N, H, W, mt, rel, hp)
                r, c = oh + dh, ow + dw
                exp = (img0 + di, r, c) if (0 <= r < H and 0 <= c < W) else None
                assert lds[hp] == exp, (N, H, W, mt, rel, dh, dw, lds[hp], exp)
    return "ok"


if __name__ == "__main__":
    for case in [(2, 56, 56), (3, 28, 28), (5, 14, 14), (7, 7, 7), (3, 9, 11), (1, 5, 3),
                 (2, 35, 35), (4, 1, 1), (3, 2, 2), (64, 7, 7), (2, 17, 17)]:
        print(case, "fwd/dgrad (256-px tiles, pitch W+1 -> x8):",
              check(*case, pitch=lambda w: (w + 1 + 7) // 8 * 8),
              "| wgrad (128-px tiles, pitch W+2 -> x16):",
              check(*case, BM=128, HPX=448, pitch=lambda w: (w + 2 + 15) // 16 * 16))
