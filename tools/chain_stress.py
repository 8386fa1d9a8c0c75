"""Chain hand-off stress: run the codec with wino_chain on in each workgroup shape, lane count
and decoupling mode at a model / patch / batch, and report which combinations leave the
hand-off error word set (a region poll that timed out) and whether the outputs still equal
the chain-off run.  GPU only; prints one JSON line per case.

    python tools/chain_stress.py --model 3 --batch 256 --iters 20
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tf_image_compression_amd.codec import Codec  # noqa: E402
from tf_image_compression_amd.weights import synthetic_params, SYNTH_MEAN, SYNTH_STD  # noqa: E402
from tf_image_compression_amd.sharded import image_batch  # noqa: E402


def run(model, P, batch, opts, x, iters):
    params = synthetic_params(model, seed=0)
    with Codec(model, params, SYNTH_MEAN, SYNTH_STD, patch_size=P, tuning="none") as c:
        for k, v in opts.items():
            c.set_option(k, v)
        eh, ew, ec = c.code_shape
        d_in, d_idx, d_rgb = c.alloc(x.nbytes), c.alloc(batch * eh * ew * ec), c.alloc(x.nbytes)
        d_in.upload(x)
        err = None
        t0 = time.perf_counter()
        try:
            for _ in range(iters):
                c.codec_device(d_in, batch, d_idx, d_rgb)
            c.synchronize()
        except Exception as e:  # the chain error word surfaces here
            err = str(e)
        dt = (time.perf_counter() - t0) / iters * 1e3
        idx = d_idx.download((batch, eh, ew, ec), np.uint8)
        rgb = d_rgb.download(x.shape, np.uint8)
        return err, dt, idx, rgb, c.layer_kernels(batch // opts.get("streams", 2))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", type=int, default=3)
    ap.add_argument("--patch", type=int, default=256)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--wh", default="1,2,3,4")
    ap.add_argument("--streams", default="2,1")
    args = ap.parse_args()
    x = image_batch(0, args.batch, args.patch)
    err0, dt0, idx0, rgb0, _ = run(args.model, args.patch, args.batch, {"chain": 0}, x, 3)
    print(json.dumps({"case": "chain=0", "err": err0, "ms": round(dt0, 3)}), flush=True)
    for streams in [int(s) for s in args.streams.split(",")]:
        for dec in (1, 0):
            for wh in [int(w) for w in args.wh.split(",")]:
                opts = {"streams": streams, "decouple": dec, "chain": 1, "chain_wh": wh}
                err, dt, idx, rgb, kern = run(args.model, args.patch, args.batch, opts, x, args.iters)
                chains = sorted({k for k in kern if "chain" in k})
                print(json.dumps({"case": opts, "err": err, "ms": round(dt, 3), "chains": chains,
                                  "idx_equal": bool(np.array_equal(idx, idx0)),
                                  "rgb_equal": bool(np.array_equal(rgb, rgb0))}), flush=True)


if __name__ == "__main__":
    main()
