"""Where does dec10_kernel's time go?  HIP-event timing of the fused decoder tail of
model_0 (256x256, 32 patches per launch) per variant, including two timing probes whose
results are invalid (variant 8 without: 100 decode_1's MFMAs, 101 decode_0, 102 the input
tile loads, 103 decode_1's weight loads; 104 neither MFMAs nor decode_0, 105 nor the halo,
106 nor the output store, 107 nor the input loads — an empty tile walk)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(v, n):
    sys.path.insert(0, ROOT)
    import numpy as np
    from tf_image_compression_amd.codec import Codec
    from tf_image_compression_amd.weights import synthetic_params, SYNTH_MEAN, SYNTH_STD
    P = 256
    c = Codec(0, synthetic_params(0), SYNTH_MEAN, SYNTH_STD, patch_size=P)
    c.set_option("fuse_tail", 1)
    x = np.random.default_rng(0).integers(0, 256, (n, P, P, 3), dtype=np.uint8)
    d = c.alloc(x.nbytes)
    d.upload(x)
    ms = c.profile_layers(d, n, 30)
    print(json.dumps({"variant": v, "n": n, "dec10_us": round(float(ms[16]) * 1e3, 2),
                      "empty_us": round(float(ms[17]) * 1e3, 2), "kernel": c.layer_kernels(n)[16]}), flush=True)
    c.close()


if __name__ == "__main__":
    if len(sys.argv) > 1:
        child(int(sys.argv[1]), int(sys.argv[2]))
    else:
        for n in (32, 64):
            for v in (0, 8, 9, 12, 100, 101, 102, 103, 104, 105, 106, 107):
                env = dict(os.environ, TIC_DEC10_VARIANT=str(v))
                subprocess.run([sys.executable, __file__, str(v), str(n)], env=env, check=True, timeout=120)
