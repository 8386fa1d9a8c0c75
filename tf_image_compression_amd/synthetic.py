"""Seeded synthetic inputs: uniform patches for throughput, structured
patches (smooth gradients + sinusoid texture + Gaussian noise sigma 8) for PSNR and
symbol statistics.  No datasets are available offline."""
import numpy as np


def uniform_patches(n, P, seed=0):
    return np.random.default_rng(1234 + seed).integers(0, 256, (n, P, P, 3), dtype=np.uint8)


def structured_patches(n, P, seed=0):
    r = np.random.default_rng(np.random.PCG64(1234 + seed))
    yy, xx = np.meshgrid(np.arange(P), np.arange(P), indexing="ij")
    out = np.empty((n, P, P, 3), np.uint8)
    for i in range(n):
        base = np.zeros((P, P, 3))
        for c in range(3):
            a, b, f1, f2 = r.uniform(-1, 1), r.uniform(-1, 1), r.uniform(0.02, 0.3), r.uniform(0.02, 0.3)
            base[..., c] = (128 + 60 * (a * xx + b * yy) / P
                            + 40 * np.sin(f1 * xx + r.uniform(0, 6)) * np.cos(f2 * yy + r.uniform(0, 6)))
        base += r.normal(0, 8, size=base.shape)
        out[i] = np.clip(np.rint(base), 0, 255).astype(np.uint8)
    return out
