#!/usr/bin/env python3
"""Where one conv3x3_wino4_kernel launch's time goes (the F(4x4,3x3) res-block conv of model_3,
BASELINE configs[2]): the per-layer entry (tic_conv3x3_device) with TIC_WINO4_TIMING set records
per workgroup s_memrealtime stamps (100 MHz) at start, loads issued, tile staged, K loop done,
exchange done, end — plus the CU / XCC it ran on.  Prints the launch span, the median /
90th-percentile phase durations, the mean number of workgroups alive, and how many workgroups
each CU ran.

    python tools/wino4_timing.py [--n 128] [--hw 64] [--res 1] [--reps 3]
"""
import argparse
import json
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TS = 24


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=128)
    ap.add_argument("--hw", type=int, default=64)
    ap.add_argument("--res", type=int, default=1)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--probe", type=int, default=0, help="TIC_WINO4_PROBE bits (results invalid)")
    ap.add_argument("--tile", default=None, help='TIC_FORCE_TILE, e.g. "4,1,5,1,4" (th, 1, 5, 1, tiles per workgroup)')
    args = ap.parse_args()
    if args.tile:
        os.environ["TIC_FORCE_TILE"] = args.tile
    sys.path.insert(0, ROOT)
    from tf_image_compression_amd.codec import Codec
    from tf_image_compression_amd.weights import synthetic_params, SYNTH_MEAN, SYNTH_STD
    c = Codec(3, synthetic_params(3, seed=0), SYNTH_MEAN, SYNTH_STD, patch_size=256)
    c.set_option("s1_form", 2)
    n, H = args.n, args.hw
    r = np.random.default_rng(5)
    x = r.standard_normal((n, H, H, 64)).astype(np.float32)
    k = (r.standard_normal((3, 3, 64, 64)) * 0.06).astype(np.float32)
    b = (r.standard_normal(64) * 0.05).astype(np.float32)
    d_in, d_out, d_res = c.alloc(x.nbytes), c.alloc(x.nbytes), c.alloc(x.nbytes)
    d_in.upload(x)
    d_res.upload(x)
    for _ in range(2):  # warm: code object, caches, clocks
        c.conv3x3_device(0, 1, d_in, n, H, H, 64, 64, k, b, d_res if args.res else None, d_out)
    path = os.path.join(tempfile.mkdtemp(), "w4ts.bin")
    os.environ["TIC_WINO4_TIMING"] = path
    if args.probe:
        os.environ["TIC_WINO4_PROBE"] = str(args.probe)
    for _ in range(args.reps):
        c.conv3x3_device(0, 1, d_in, n, H, H, 64, 64, k, b, d_res if args.res else None, d_out)
    del os.environ["TIC_WINO4_TIMING"]
    raw = open(path, "rb").read()
    off = 0
    for rep in range(args.reps):
        g = int(np.frombuffer(raw[off:off + 8], np.int64)[0])
        t = np.frombuffer(raw[off + 8:off + 8 + 8 * TS * g], np.uint64).reshape(g, TS).astype(np.int64)
        off += 8 + 8 * TS * g
        t = t[t[:, 0] != 0]
        us = lambda a: a / 100.0
        span = us(t[:, 16].max() - t[:, 0].min())
        rep_d = {"rep": rep, "probe": args.probe, "workgroups": int(len(t)), "span_us": round(float(span), 2)}
        kl = t[:, 3:15]
        med = lambda d: [round(float(np.median(d)), 2), round(float(np.percentile(d, 90)), 2)]
        rep_d["issue"] = med(us(t[:, 1] - t[:, 0]))
        rep_d["stage"] = med(us(t[:, 2] - t[:, 1]))
        rep_d["kloop_first_wave"] = med(us(kl.min(1) - t[:, 2]))
        rep_d["kloop_last_wave"] = med(us(kl.max(1) - t[:, 2]))
        rep_d["kloop_by_wave"] = [round(float(np.median(us(kl[:, w] - t[:, 2]))), 2) for w in range(12)]
        # shader clock over wave 0's K loop: shader cycles / (100 MHz ticks / 100) -> MHz
        clk = (t[:, 18] - t[:, 17]) / np.maximum(1, t[:, 3] - t[:, 2]) * 100.0
        rep_d["clock_mhz"] = med(clk)
        rep_d["exchange"] = med(us(t[:, 15] - kl.max(1)))
        rep_d["epilogue"] = med(us(t[:, 16] - t[:, 15]))
        life = us(t[:, 16] - t[:, 0])
        rep_d["wg_life_us"] = med(life)
        rep_d["mean_alive"] = round(float(life.sum() / span), 1)
        hw, xcc = t[:, 22], t[:, 23]
        cu = ((hw >> 8) & 0xF) | (((hw >> 12) & 1) << 4) | (((hw >> 13) & 0x7) << 5)  # CU, SH, SE bits
        key = xcc * 1024 + cu
        cnt = np.unique(key, return_counts=True)[1]
        rep_d["cus_used"] = int(len(cnt))
        rep_d["wg_per_cu"] = [int(cnt.min()), float(round(cnt.mean(), 2)), int(cnt.max())]
        # gaps between consecutive workgroups on one CU (end of one -> start of the next)
        gaps = []
        for kk in np.unique(key):
            s = t[key == kk]
            s = s[np.argsort(s[:, 0])]
            if len(s) > 1:
                gaps.extend(us(s[1:, 0] - s[:-1, 16]).tolist())
        if gaps:
            rep_d["cu_gap_us"] = [round(float(np.median(gaps)), 2), round(float(np.percentile(gaps, 90)), 2)]
        print(json.dumps(rep_d), flush=True)
    c.close()


if __name__ == "__main__":
    main()
