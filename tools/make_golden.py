#!/usr/bin/env python3
"""Generate tests/golden/*.npz from the CPU oracle, cross-checked at generation time against
an independent torch-CPU restatement of the TF ops (F.conv2d with explicit TF-SAME pads,
F.conv_transpose2d cropped to 2H).  Run in the build container only:

    python tools/make_golden.py

Weights are NOT stored: they are regenerated from ``synthetic_params(model_id, seed=0)``
(seeded PCG64) and pinned by a SHA-256 digest in each fixture.
"""
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import tic_oracle as o  # noqa: E402
from tf_image_compression_amd.weights import synthetic_params, SYNTH_MEAN, SYNTH_STD  # noqa: E402
from tf_image_compression_amd.synthetic import structured_patches  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")


def torch_conv(x, k, kind):
    """Independent restatement with torch-CPU (float64)."""
    import torch
    import torch.nn.functional as F
    xt = torch.from_numpy(np.asarray(x, np.float64)).permute(0, 3, 1, 2)
    if kind == "convT":
        w = torch.from_numpy(np.asarray(k, np.float64)).permute(3, 2, 0, 1)  # [kh,kw,out,in] -> [in,out,kh,kw]
        h, wd = x.shape[1], x.shape[2]
        y = F.conv_transpose2d(xt, w, stride=2)[:, :, :2 * h, :2 * wd]
    else:
        s = 1 if kind == "conv_s1" else 2
        _, pt, pb = o.tf_same_pads(x.shape[1], s)
        _, pl, pr = o.tf_same_pads(x.shape[2], s)
        w = torch.from_numpy(np.asarray(k, np.float64)).permute(3, 2, 0, 1)  # HWIO -> OIHW
        y = F.conv2d(F.pad(xt, (pl, pr, pt, pb)), w, stride=s)
    return y.permute(0, 2, 3, 1).numpy()


def torch_model(params, patches, P, model_id):
    """Encoder + decoder with every conv done by torch (structure from the oracle tables)."""
    enc, dec = o.MODELS[model_id]

    def run(x, layers):
        for name, kind, cin, cout, act in layers:
            if kind == "res":
                y = x
                for j in range(2):
                    nm = f"{name}/conv_{j}"
                    y = torch_conv(y, params[nm + "/kernel"], "conv_s1").astype(np.float32) + params[nm + "/bias"]
                    y = np.maximum(y, 0)
                x = x + y
            else:
                y = torch_conv(x, params[name + "/kernel"], kind).astype(np.float32) + params[name + "/bias"]
                x = np.maximum(y, 0) if act == "relu" else y
        return x

    x = o.normalize(patches, SYNTH_MEAN, SYNTH_STD, P)
    pre = run(x, enc)
    idx = o.quantize(pre, 2)
    y = run(o.dequant_lut(2)[idx.astype(np.int64)], dec)
    return pre, idx, o.denormalize(y, SYNTH_MEAN, SYNTH_STD)


def digest(params):
    h = hashlib.sha256()
    for k in sorted(params):
        h.update(k.encode())
        h.update(np.ascontiguousarray(params[k], np.float32).tobytes())
    return h.hexdigest()


def layers():
    r = np.random.default_rng(np.random.PCG64(777))
    out = {}
    for name, kind, cin, cout, h, w in [("s1", "conv_s1", 16, 16, 9, 7), ("s2", "conv_s2", 16, 32, 10, 8),
                                        ("s2odd", "conv_s2", 8, 16, 9, 7), ("t2", "convT", 32, 16, 5, 6)]:
        x = r.standard_normal((2, h, w, cin)).astype(np.float32)
        kshape = (3, 3, cout, cin) if kind == "convT" else (3, 3, cin, cout)
        k = (r.standard_normal(kshape) * np.sqrt(2 / (9 * cin))).astype(np.float32)
        b = (r.standard_normal(cout) * 0.1).astype(np.float32)
        p = {"l/kernel": k, "l/bias": b}
        if kind == "convT":
            y = o.my_conv2d_transpose(x, p, "l", "relu")
        else:
            y = o.my_conv2d(x, p, "l", 1 if kind == "conv_s1" else 2, "relu")
        ty = np.maximum(torch_conv(x, k, kind).astype(np.float32) + b, 0)
        assert np.max(np.abs(ty - y)) < 1e-5, (name, np.max(np.abs(ty - y)))
        out.update({f"{name}_x": x, f"{name}_k": k, f"{name}_b": b, f"{name}_y": y, f"{name}_kind": np.array(kind)})
    np.savez_compressed(os.path.join(OUT, "layers.npz"), **out)


def codec_case(model_id, P, n, seed, fname, store_f32=True):
    params = synthetic_params(model_id, seed=0)
    patches = structured_patches(n, P, seed=seed)
    pre, idx = o.encoder(params, SYNTH_MEAN, SYNTH_STD, patches, P, 2, model_id)
    f, u8 = o.decoder(params, SYNTH_MEAN, SYNTH_STD, idx, 2, model_id)
    tpre, tidx, tf = torch_model(params, patches, P, model_id)
    scale = np.abs(pre).max()
    assert np.max(np.abs(tpre - pre)) < 1e-4 * scale
    safe = o.decision_margin(pre, 2) > 1e-5 * scale
    assert np.array_equal(tidx[safe], idx[safe])
    # torch decoder ran on its own symbols; compare where symbols agree everywhere
    if np.array_equal(tidx, idx):
        assert np.max(np.abs(tf - f)) < 1e-2
    extra = {"recon_f32": f} if store_f32 else {"recon_f32_sha256": hashlib.sha256(f.tobytes()).hexdigest()}
    np.savez_compressed(os.path.join(OUT, fname), model_id=model_id, patch=P, n=n, seed=seed, patches=patches,
                        preact=pre, idx=idx, recon_u8=u8, weights_sha256=digest(params),
                        mean=SYNTH_MEAN, std=SYNTH_STD, **extra)
    print(fname, "preact max", float(scale), "symbols", idx.shape, "psnr",
          round(o.dataset_psnr(list(zip(patches, u8))), 3))


def main():
    os.makedirs(OUT, exist_ok=True)
    layers()
    codec_case(0, 64, 2, 21, "model0_p64.npz")
    codec_case(3, 64, 2, 23, "model3_p64.npz")
    codec_case(1, 32, 2, 25, "model1_p32.npz")
    codec_case(2, 32, 2, 27, "model2_p32.npz")
    codec_case(0, 256, 1, 29, "model0_p256.npz", store_f32=False)
    total = sum(os.path.getsize(os.path.join(OUT, f)) for f in os.listdir(OUT))
    print("fixtures bytes:", total)


if __name__ == "__main__":
    main()
