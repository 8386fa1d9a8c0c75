"""Predicts the parity margin of a Winograd F(m x m, 3 x 3) form before it is built: runs the
oracle codec (oracle/tic_oracle.py) with every stride-1 conv replaced by an f32 emulation of
the Winograd form (transforms and point GEMMs rounded to f32, U = G g G^T in double, rounded
once) and reports what tests/gpu_checks.py::check_codec measures: max |preact - ref| / scale,
symbol mismatches outside the 1e-5 decision band, decoder float error on the [0,255] scale.

Test infrastructure (imports the oracle); not part of the product.

  python tools/wino_numerics.py --model 3 --P 256 --n 2 --m 4
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import tic_oracle as o  # noqa: E402
from tf_image_compression_amd.synthetic import structured_patches  # noqa: E402
from tf_image_compression_amd.weights import SYNTH_MEAN, SYNTH_STD, synthetic_params  # noqa: E402

F32 = np.float32


def cook_toom(pts, m, r=3):
    """A^T (m x n), G (n x r), B^T (n x n) of F(m, r) on the finite points pts plus infinity."""
    n = m + r - 1
    assert len(pts) == n - 1
    AT = np.zeros((m, n))
    G = np.zeros((n, r))
    for i, p in enumerate(pts):
        f = np.prod([p - q for j, q in enumerate(pts) if j != i])
        AT[:, i] = [p ** k for k in range(m)]
        G[i] = [p ** j / f for j in range(r)]
    AT[m - 1, n - 1] = 1
    G[n - 1, r - 1] = 1
    rows, rhs = [], []
    for k in range(m):
        for j in range(r):
            for l in range(n):
                c = np.zeros((n, n))
                c[:, l] = AT[k] * G[:, j]
                rows.append(c.ravel())
                rhs.append(1.0 if l == k + j else 0.0)
    X = np.linalg.lstsq(np.array(rows), np.array(rhs), rcond=None)[0]
    BT = np.round(X.reshape(n, n) * 64) / 64  # dyadic for the point sets used here
    return AT, G, BT


POINTS = {2: (0, 1, -1), 4: (0, 1, -1, 2, -0.5)}


def wino_conv_s1(x, kernel, m):
    AT, G, BT = cook_toom(POINTS[m], m)
    a = m + 2
    n, h, w, c = x.shape
    th, tw = -(-h // m), -(-w // m)
    xp = np.zeros((n, th * m + 2, tw * m + 2, c), F32)
    xp[:, 1:1 + h, 1:1 + w] = x
    s0, s1, s2, s3 = xp.strides
    d = np.lib.stride_tricks.as_strided(xp, (n, th, tw, a, a, c), (s0, s1 * m, s2 * m, s1, s2, s3))
    B = BT.astype(F32)
    A = AT.astype(F32)
    V = np.einsum('ai,ntsijc->ntsajc', B, d).astype(F32)
    V = np.einsum('bj,ntsajc->ntsabc', B, V).astype(F32)
    U = np.einsum('ai,ijcd,bj->abcd', G, np.asarray(kernel, np.float64), G).astype(F32)
    V = V.reshape(-1, a * a, c).transpose(1, 0, 2)  # [pt][tiles][c]
    M = np.matmul(V, U.reshape(a * a, c, -1)).astype(F32)  # [pt][tiles][co]
    M = M.transpose(1, 0, 2).reshape(n, th, tw, a, a, -1)
    T = np.einsum('ia,ntsabd->ntsibd', A, M).astype(F32)
    Y = np.einsum('jb,ntsibd->ntsijd', A, T).astype(F32)
    Y = Y.transpose(0, 1, 3, 2, 4, 5).reshape(n, th * m, tw * m, -1)
    return Y[:, :h, :w]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--model', type=int, default=3)
    ap.add_argument('--P', type=int, default=256)
    ap.add_argument('--n', type=int, default=2)
    ap.add_argument('--m', type=int, default=4)
    ap.add_argument('--seed', type=int, default=301)
    args = ap.parse_args()
    params = synthetic_params(args.model, seed=0)
    x = structured_patches(args.n, args.P, seed=args.seed)
    ref_pre, ref_idx = o.encoder(params, SYNTH_MEAN, SYNTH_STD, x, args.P, 2, args.model)
    exact = o.conv2d_same

    def conv(xx, kernel, stride, acc=np.float64):
        if stride == 1:
            return wino_conv_s1(np.asarray(xx, F32), kernel, args.m)
        return exact(xx, kernel, stride, np.float32)
    o.conv2d_same = conv
    try:
        pre, idx = o.encoder(params, SYNTH_MEAN, SYNTH_STD, x, args.P, 2, args.model, acc=np.float32)
        scale = max(1.0, float(np.max(np.abs(ref_pre))))
        safe = o.decision_margin(ref_pre, 2) > 1e-5 * scale
        mism = int(np.count_nonzero((idx != ref_idx) & safe))
        f, u8 = o.decoder(params, SYNTH_MEAN, SYNTH_STD, idx, 2, args.model, acc=np.float32)
    finally:
        o.conv2d_same = exact
    ref_f, ref_u8 = o.decoder(params, SYNTH_MEAN, SYNTH_STD, idx, 2, args.model)
    print(dict(m=args.m, model=args.model, P=args.P,
               preact_rel=float(np.max(np.abs(pre - ref_pre))) / scale, bar_preact=1e-4,
               sym_mismatch_outside_band=mism, sym_total_mismatch=int(np.count_nonzero(idx != ref_idx)),
               dec_float_err=float(np.max(np.abs(f - ref_f))), bar_dec=1e-2,
               u8_max_diff=int(np.max(np.abs(u8.astype(int) - ref_u8.astype(int))))))


if __name__ == '__main__':
    main()
