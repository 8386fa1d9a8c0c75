"""Per-layer HIP-event timing (Codec.profile_layers) of one codec configuration, one child
process per setting: `python tools/layer_probe.py MODEL N 'ENV=..,opt:name=val' ...` prints one
JSON line per setting with every launch's microseconds and kernel instance.  Settings are
comma-separated environment variables (TIC_*) and `opt:` codec options."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(model, n, setting):
    sys.path.insert(0, ROOT)
    import numpy as np
    from tf_image_compression_amd.codec import Codec
    from tf_image_compression_amd.weights import synthetic_params, SYNTH_MEAN, SYNTH_STD
    P = 256
    c = Codec(model, synthetic_params(model), SYNTH_MEAN, SYNTH_STD, patch_size=P)
    for kv in filter(None, setting.split(",")):
        if kv.startswith("opt:"):
            k, v = kv[4:].split("=")
            c.set_option(k, int(v))
    x = np.random.default_rng(0).integers(0, 256, (n, P, P, 3), dtype=np.uint8)
    d = c.alloc(x.nbytes)
    d.upload(x)
    c.autotune(d, n, reps=5)  # tiling choices per layer (fused variants pinned by env if given)
    ms = c.profile_layers(d, n, 30)
    kern = c.layer_kernels(n)
    rows = [(k, round(float(ms[i]) * 1e3, 2)) for i, k in enumerate(kern) if k]
    print(json.dumps({"setting": setting, "n": n, "total_us": round(sum(u for _, u in rows), 1), "launches": rows}),
          flush=True)
    c.close()


if __name__ == "__main__":
    if sys.argv[1] == "--child":
        child(int(sys.argv[2]), int(sys.argv[3]), sys.argv[4])
    else:
        model, n = int(sys.argv[1]), int(sys.argv[2])
        for setting in sys.argv[3:]:
            env = dict(os.environ)
            env.update(kv.split("=", 1) for kv in setting.split(",") if kv and not kv.startswith("opt:"))
            subprocess.run([sys.executable, __file__, "--child", str(model), str(n), setting], env=env, check=True,
                           timeout=120)
