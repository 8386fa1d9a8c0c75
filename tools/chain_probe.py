"""Where does wino_chain_kernel's time go?  Per-layer HIP-event timing (profile_layers)
of model_0 at 256x256, lane batch 32, with the chain off, on, and with timing probes that
drop the hand-off (TIC_CHAIN_PROBE=1) or its wait + halo read (=2) — probe results are
numerically invalid and only timed.  Prints one JSON line per configuration."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(cfg):
    sys.path.insert(0, ROOT)
    import numpy as np
    from tf_image_compression_amd.codec import Codec
    from tf_image_compression_amd.weights import synthetic_params, SYNTH_MEAN, SYNTH_STD
    n, P = int(cfg.get("n", 32)), 256
    c = Codec(0, synthetic_params(0), SYNTH_MEAN, SYNTH_STD, patch_size=P)
    c.set_option("chain", int(cfg["chain"]))
    d0 = None
    x = np.random.default_rng(0).integers(0, 256, (n, P, P, 3), dtype=np.uint8)
    d = c.alloc(x.nbytes)
    d.upload(x)
    c.autotune(d, n, reps=3)
    ms = c.profile_layers(d, n, 20)
    names = [l[0] for l in c.layers()]
    print(json.dumps({"cfg": cfg, "layers": {k: round(float(v) * 1e3, 2) for k, v in zip(names, ms)},
                      "kernels": c.layer_kernels(n)}), flush=True)
    c.close()


if __name__ == "__main__":
    if len(sys.argv) > 1:
        child(json.loads(sys.argv[1]))
    else:
        for cfg in [{"chain": 0}, {"chain": 1}, {"chain": 1, "probe": 1}, {"chain": 0, "n": 64}, {"chain": 1, "n": 64},
                    {"chain": 1, "n": 8}, {"chain": 0, "n": 8}]:
            env = dict(os.environ)
            if "probe" in cfg:
                env["TIC_CHAIN_PROBE"] = str(cfg["probe"])
            subprocess.run([sys.executable, __file__, json.dumps(cfg)], env=env, check=True, timeout=120)
