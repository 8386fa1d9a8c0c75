#!/usr/bin/env python3
"""Per-layer time vs per-launch batch (1..64 patches): separates each layer's fixed
per-launch cost from its per-patch cost (GPU box, HIP events on the lane's stream)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(model=0, P=256):
    from tf_image_compression_amd.codec import Codec
    from tf_image_compression_amd.weights import synthetic_params, SYNTH_MEAN, SYNTH_STD
    c = Codec(model, synthetic_params(model), SYNTH_MEAN, SYNTH_STD, patch_size=P)
    x = np.random.default_rng(1).integers(0, 256, (64, P, P, 3), dtype=np.uint8)
    d = c.alloc(x.nbytes)
    d.upload(x)
    names = [l[0] if isinstance(l, tuple) else l for l in c.layers()]
    res = {}
    for n in (1, 4, 16, 32, 64):
        c.autotune(d, n, reps=3)
        res[n] = c.profile_layers(d, n, 20) * 1e3
    print(f"{'layer':24s}" + "".join(f"{'n=' + str(n):>9s}" for n in res))
    for i, nm in enumerate(names):
        print(f"{str(nm)[:24]:24s}" + "".join(f"{res[n][i]:9.1f}" for n in res))
    print(f"{'sum':24s}" + "".join(f"{res[n].sum():9.1f}" for n in res))
    c.close()


if __name__ == "__main__":
    main(*map(int, sys.argv[1:]))
