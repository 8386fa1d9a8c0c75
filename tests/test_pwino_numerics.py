"""CPU check of the polyphase Winograd algebra behind conv3x3_pwino.h (stride-2 / transposed
form 1): the kernel's tile decomposition, B^T / A^T and the host's U = G g G^T
(tic_runtime.cpp pack_pwino), restated in float64 numpy over a tile loop, reproduce the
oracle's stride-2 'SAME' conv and conv2d_transpose (basic_block/basic_block.py:27-57) to f32
rounding on even and odd sizes — the derivation is pinned before any GPU run."""
import numpy as np
import pytest

from oracle import tic_oracle as o

# 1-D point weights (rows of G) and input transforms, as in conv3x3_pwino.h
GS = np.array([[1, 0, 0], [1, 0, 1], [0, 0, 1], [0, 1, 0], [0, 1, 0]], np.float64)
GT = np.array([[0, 0, 1], [1, 0, 1], [1, 0, 0], [0, 1, 0], [0, 1, 0]], np.float64)
# B^T: stride 2 over 5 samples, transpose over 3 samples
BS = np.array([[1, 0, -1, 0, 0], [0, 0, 1, 0, 0], [0, 0, -1, 0, 1], [0, 1, 0, 0, 0], [0, 0, 0, 1, 0]], np.float64)
BT = np.array([[1, -1, 0], [0, 1, 0], [0, -1, 1], [0, 1, 0], [0, 0, 1]], np.float64)
# A^T: stride 2 two outputs, transpose four outputs (2m, 2m+1, 2m+2, 2m+3)
AS = np.array([[1, 1, 0, 1, 0], [0, 1, 1, 0, 1]], np.float64)
AT = np.array([[1, 1, 0, 0, 0], [0, 0, 0, 1, 0], [0, 1, 1, 0, 0], [0, 0, 0, 0, 1]], np.float64)


def pwino_s2(x, k, pady, padx):
    """x [H,W,Cin], k HWIO; SAME stride 2 with pad_before (pady, padx) (the kernel's tile loop)."""
    H, W, cin = x.shape
    cout = k.shape[3]
    Ho, Wo = (H + 1) // 2, (W + 1) // 2
    U = np.einsum("ay,yxio,bx->abio", GS, k.astype(np.float64), GS)  # [5,5,cin,cout]
    y = np.zeros((Ho, Wo, cout))
    for ty in range((Ho + 1) // 2):
        for tx in range((Wo + 1) // 2):
            d = np.zeros((5, 5, cin))
            for r in range(5):
                for c in range(5):
                    iy, ix = 4 * ty + r - pady, 4 * tx + c - padx
                    if 0 <= iy < H and 0 <= ix < W:
                        d[r, c] = x[iy, ix]
            V = np.einsum("ar,rci,bc->abi", BS, d, BS)
            M = np.einsum("abi,abio->abo", V, U)
            Y = np.einsum("pa,abo,qb->pqo", AS, M, AS)
            for a in range(2):
                for b in range(2):
                    oy, ox = 2 * ty + a, 2 * tx + b
                    if oy < Ho and ox < Wo:
                        y[oy, ox] = Y[a, b]
    return y


def pwino_t2(x, k):
    """x [H,W,Cin], k [kh,kw,Cout,Cin]; conv2d_transpose stride 2 'SAME' to 2H x 2W."""
    H, W, cin = x.shape
    cout = k.shape[2]
    U = np.einsum("ay,yxoi,bx->abio", GT, k.astype(np.float64), GT)
    y = np.zeros((2 * H, 2 * W, cout))
    for ty in range((H + 1) // 2):
        for tx in range((W + 1) // 2):
            d = np.zeros((3, 3, cin))
            for r in range(3):
                for c in range(3):
                    iy, ix = 2 * ty - 1 + r, 2 * tx - 1 + c
                    if 0 <= iy < H and 0 <= ix < W:
                        d[r, c] = x[iy, ix]
            V = np.einsum("ar,rci,bc->abi", BT, d, BT)
            M = np.einsum("abi,abio->abo", V, U)
            Y = np.einsum("pa,abo,qb->pqo", AT, M, AT)
            for a in range(4):
                for b in range(4):
                    oy, ox = 4 * ty + a, 4 * tx + b
                    if oy < 2 * H and ox < 2 * W:
                        y[oy, ox] = Y[a, b]
    return y


@pytest.mark.parametrize("H,W", [(8, 8), (9, 7), (1, 2), (12, 5)])
def test_pwino_stride2_algebra(H, W):
    r = np.random.default_rng(H * 31 + W)
    cin, cout = 3, 4
    x = r.standard_normal((1, H, W, cin)).astype(np.float32)
    k = r.standard_normal((3, 3, cin, cout)).astype(np.float32)
    b = np.zeros(cout, np.float32)
    ref = o.my_conv2d(x, {"l/kernel": k, "l/bias": b}, "l", 2, "identity")[0]
    pady = max((((H + 1) // 2) - 1) * 2 + 3 - H, 0) // 2  # TF SAME pad_before
    padx = max((((W + 1) // 2) - 1) * 2 + 3 - W, 0) // 2
    got = pwino_s2(x[0], k, pady, padx)
    assert np.max(np.abs(got - ref)) <= 1e-5 * max(1.0, np.max(np.abs(ref)))


@pytest.mark.parametrize("H,W", [(4, 4), (5, 3), (1, 1), (6, 7)])
def test_pwino_transpose_algebra(H, W):
    r = np.random.default_rng(H * 17 + W)
    cin, cout = 3, 4
    x = r.standard_normal((1, H, W, cin)).astype(np.float32)
    k = r.standard_normal((3, 3, cout, cin)).astype(np.float32)
    b = np.zeros(cout, np.float32)
    ref = o.my_conv2d_transpose(x, {"l/kernel": k, "l/bias": b}, "l", "identity")[0]
    got = pwino_t2(x[0], k)
    assert np.max(np.abs(got - ref)) <= 1e-5 * max(1.0, np.max(np.abs(ref)))


def test_pwino_point_count():
    """25 transform points per tile against the direct form's 36 products (0.69x)."""
    assert GS.shape[0] * GS.shape[0] == 25 and 4 * 9 == 36
