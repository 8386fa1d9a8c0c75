#!/usr/bin/env python3
"""Interleaved A/B timing of codec options in ONE process (methodology rule: variants
compared in alternating rounds on the same device).  Usage on the GPU box:

    python tools/ab.py --model 0 --batch 64 --rounds 7 --steps 20 \
        --cfg streams=1 --cfg streams=2 --cfg streams=2,fuse01=1
"""
import argparse
import json
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", type=int, default=0)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--patch", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--cfg", action="append", required=True, help="k=v[,k=v] codec options; env:KEY=V for env")
    ap.add_argument("--tune-file", default=None, help="replay this tf_image_compression_amd/tune/*.json state instead of tuning")
    ap.add_argument("--refork", action="store_true", help="every round starts from a fresh fork of the lanes")
    args = ap.parse_args()
    from tf_image_compression_amd.codec import Codec
    from tf_image_compression_amd.weights import synthetic_params, SYNTH_MEAN, SYNTH_STD
    from tf_image_compression_amd.topology import bottleneck_shape
    P, B, M = args.patch, args.batch, args.model
    codec = Codec(M, synthetic_params(M), SYNTH_MEAN, SYNTH_STD, patch_size=P)
    eh, ew, ec = bottleneck_shape(M, P)
    x = np.random.default_rng(1234).integers(0, 256, (B, P, P, 3), dtype=np.uint8)
    d_in, d_idx, d_rgb = codec.alloc(x.nbytes), codec.alloc(B * eh * ew * ec), codec.alloc(x.nbytes)
    d_in.upload(x)

    def apply(cfg):
        for kv in cfg.split(","):
            k, v = kv.split("=")
            if k.startswith("env:"):
                os.environ[k[4:]] = v
            else:
                codec.set_option(k, int(v))

    if args.tune_file:
        with open(args.tune_file) as f:
            codec.tuning_import(json.load(f)["tuning"])
    for cfg in args.cfg:  # autotune each configuration's lane batch once (no-op where replayed)
        apply(cfg)
        m = [int(kv.split("=")[1]) for kv in cfg.split(",") if kv.startswith("streams=")]
        k = m[-1] if m else 2
        lane_b = -(-B // max(1, min(k, B)))
        codec.autotune(d_in, lane_b, reps=5)
    res = {c: [] for c in args.cfg}
    for r in range(args.rounds):
        for cfg in args.cfg:
            apply(cfg)
            if args.refork:
                codec.synchronize()
                codec.set_option("decouple", 1)  # marks the handle stream dirty: the next call forks
            for _ in range(3):
                codec.codec_device(d_in, B, d_idx, d_rgb)
            codec.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                codec.codec_device(d_in, B, d_idx, d_rgb)
            codec.synchronize()
            res[cfg].append((time.perf_counter() - t0) * 1e3 / args.steps)
    out = {c: {"median_ms": round(statistics.median(v), 4), "min_ms": round(min(v), 4),
               "mpix_s": round(B * P * P / statistics.median(v) / 1e3, 1),
               "rounds_ms": [round(x, 4) for x in v]} for c, v in res.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
