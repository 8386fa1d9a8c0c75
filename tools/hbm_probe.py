#!/usr/bin/env python3
"""HBM calibration on the GPU box: achieved GB/s of the one-pass glue kernels at the sizes
of the full-resolution layers (64 MB f32 = 32 patches x 128^2 x 32 ch), to compare the
full-resolution conv layers against a plain streaming kernel on the same device."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timeit(fn, sync, reps=50):
    fn()
    sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    sync()
    return (time.perf_counter() - t0) / reps


def main():
    from tf_image_compression_amd.codec import Codec
    from tf_image_compression_amd.weights import synthetic_params, SYNTH_MEAN, SYNTH_STD
    c = Codec(0, synthetic_params(0), SYNTH_MEAN, SYNTH_STD, patch_size=256)
    n = 16 << 20  # floats
    a = c.alloc(4 * n)
    a.upload(np.random.default_rng(0).random(n, dtype=np.float32) * 255)
    b = c.alloc(n)
    u = c.alloc(n)
    acc = c.alloc(8)
    t = timeit(lambda: c.round_u8_device(a, n, b), c.synchronize)
    print(f"round_u8 f32->u8 {n*5/1e6:.0f} MB: {t*1e6:.1f} us  {n*5/t/1e9:.0f} GB/s")
    t = timeit(lambda: c.sse_u8_device(b, u, n, acc), c.synchronize)
    print(f"sse_u8 2x u8 read {n*2/1e6:.0f} MB: {t*1e6:.1f} us  {n*2/t/1e9:.0f} GB/s")
    img = c.alloc(4 * n)
    t = timeit(lambda: c.patches_to_image_device(a, 2048, 2048, 256, img), c.synchronize)
    nb = 2048 * 2048 * 3 * 8
    print(f"stitch f32 copy {nb/1e6:.0f} MB: {t*1e6:.1f} us  {nb/t/1e9:.0f} GB/s")
    # layer timings of the last layer per tiling and batch
    P = 256
    x = np.random.default_rng(1).integers(0, 256, (64, P, P, 3), dtype=np.uint8)
    d_in = c.alloc(x.nbytes)
    d_in.upload(x)
    for tile in ["0", "1", "2", "3", "4", "5"]:
        os.environ["TIC_RGB_OUT_TILE"] = tile
        for bs in (32, 64):
            ms = c.profile_layers(d_in, bs, 10)
            print(f"tile {tile} n={bs}: encode_0 {ms[0]*1e3:.1f} us  encode_1 {ms[1]*1e3:.1f}  decode_1 {ms[-2]*1e3:.1f}  decode_0 {ms[-1]*1e3:.1f} us")
    c.close()


if __name__ == "__main__":
    main()
