"""Where wino_chain_kernel's (or, --enc01, enc01_kernel's) time goes, phase by phase,
inside the two-lane step.

Runs the bench's configuration (model_0, 256^2, batch 64, the committed tuning replayed)
with TIC_CHAIN_TIMING set: every chain launch records s_memrealtime (100 MHz) at its
phase boundaries (wino_chain.h, CH_TS), and tic_synchronize appends the last launch's
stamps to a file.  Prints, per chain launch (lane, encoder/decoder side), the spread of
workgroup start times and the median / 90th-percentile duration of every phase per layer.

    python tools/chain_timing.py [--tune-file tf_image_compression_amd/tune/model0_p256_b64_s2.json] [--steps 20] [--enc01]
"""
import argparse
import json
import os
import struct
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PHASES = ["mfma", "epilogue", "publish", "wait", "halo"]


def read_dumps(path):
    out = []
    with open(path, "rb") as f:
        while True:
            h = f.read(16)
            if len(h) < 16:
                break
            lane, slot, grid, ts = struct.unpack("4i", h)
            t = np.frombuffer(f.read(8 * grid * ts), dtype=np.uint64).reshape(grid, ts)
            out.append((lane, slot, t))
    return out


def summarise(t, nl):
    us = lambda a: a.astype(np.float64) / 100.0  # 100 MHz ticks -> us
    t = t.astype(np.int64)
    start = t[:, 0]
    rep = {"workgroups": int(t.shape[0]),
           "start_spread_us": round(float(us(start.max() - start.min())), 2),
           "stage_us": round(float(np.median(us(t[:, 1] - t[:, 0]))), 2),
           "kernel_us": round(float(us(t[:, 2 + 6 * (nl - 1) + 2].max() - start.min())), 2),
           "layers": []}
    for l in range(nl):
        b = 2 + 6 * l
        row = {}
        marks = [b, b + 1, b + 2] + ([b + 3, b + 4, b + 5] if l < nl - 1 else [])
        for k in range(len(marks) - 1):
            d = us(t[:, marks[k + 1]] - t[:, marks[k]])
            row[PHASES[k]] = [round(float(np.median(d)), 2), round(float(np.percentile(d, 90)), 2)]
        rep["layers"].append(row)
    # the stride-2 head / transposed tail of a chain_x launch (wino_chain.h CH_HEAD_TS / CH_TAIL_TS:
    # stamps after the 8 layer slots)
    hb = 2 + 6 * 8
    if t.shape[1] >= hb + 12:
        if np.all(t[:, hb + 5] != 0):
            marks = [0] + [hb + k for k in range(6)]
            names = ["window", "mfma", "epilogue", "publish", "wait", "halo"]
            rep["head"] = {names[k]: [round(float(np.median(us(t[:, marks[k + 1]] - t[:, marks[k]]))), 2),
                                      round(float(np.percentile(us(t[:, marks[k + 1]] - t[:, marks[k]]), 90)), 2)]
                           for k in range(6)}
        tb = hb + 6
        if np.all(t[:, tb + 2] != 0):
            # chain_x 2: decode_3 -> LDS tile (+ halo recompute), then decode_2's K loop and stores
            two = np.all(t[:, tb + 4] != 0)
            names = ["mfma", "halo+tile", "d2_mfma", "d2_store"] if two else ["mfma", "store"]
            rep["tail"] = {nm: [round(float(np.median(us(t[:, tb + k + 1] - t[:, tb + k]))), 2),
                                round(float(np.percentile(us(t[:, tb + k + 1] - t[:, tb + k]), 90)), 2)]
                           for k, nm in enumerate(names)}
            rep["kernel_us"] = round(float(us(t[:, tb + len(names)].max() - start.min())), 2)
    # round 6: the same phase ends seen by wave 4 (the second wave on thread 0's SIMD) and the
    # workgroup's end (wino_chain.h CH_W4_TS .. CH_END_TS): "w4_lag" = how much later wave 4
    # finishes a K loop than wave 0, i.e. how much of thread 0's next phase is its wait for it
    w4 = hb + 12
    if t.shape[1] >= w4 + 13:
        med = lambda d: [round(float(np.median(us(d))), 2), round(float(np.percentile(us(d), 90)), 2)]
        lag = {}
        for l in range(nl):
            if np.all(t[:, w4 + l] != 0):
                lag[f"layer{l}"] = med(t[:, w4 + l] - t[:, 2 + 6 * l + 1])
        if np.all(t[:, w4 + 8] != 0) and np.all(t[:, hb + 1] != 0):
            lag["head"] = med(t[:, w4 + 8] - t[:, hb + 1])
        tb = hb + 6
        if np.all(t[:, w4 + 9] != 0):
            lag["tail"] = med(t[:, w4 + 9] - t[:, tb + 1])
        if np.all(t[:, w4 + 10] != 0):
            lag["d2"] = med(t[:, w4 + 10] - t[:, tb + 3])
            rep["w4_d2_store"] = med(t[:, w4 + 11] - t[:, w4 + 10])
        rep["w4_lag"] = lag
        if np.all(t[:, w4 + 12] != 0):
            rep["wg_life_us"] = med(t[:, w4 + 12] - start)
            rep["kernel_us"] = round(float(us(t[:, w4 + 12].max() - start.min())), 2)
    return rep


ENC01_PHASES = ["lut", "stage", "layer0", "layer1", "store"]


def summarise_enc01(t):
    t = t[t[:, 5] != 0].astype(np.int64)  # workgroups of the launched grid
    us = lambda a: a.astype(np.float64) / 100.0
    rep = {"workgroups": int(t.shape[0]),
           "kernel_us": round(float(us(t[:, 5].max() - t[:, 0].min())), 2),
           "wg_life_us": [round(float(np.median(us(t[:, 5] - t[:, 0]))), 2),
                          round(float(np.percentile(us(t[:, 5] - t[:, 0]), 90)), 2)]}
    for k, name in enumerate(ENC01_PHASES):
        d = us(t[:, k + 1] - t[:, k])
        rep[name] = [round(float(np.median(d)), 2), round(float(np.percentile(d, 90)), 2)]
    # average workgroups alive over the launch
    rep["mean_alive"] = round(float(np.sum(t[:, 5] - t[:, 0]) / (t[:, 5].max() - t[:, 0].min())), 1)
    return rep


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tune-file", default=os.path.join(ROOT, "tf_image_compression_amd", "tune", "model0_p256_b64_s2.json"))
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--streams", type=int, default=2)
    ap.add_argument("--batch", type=int, default=64, help="patches per call (one lane: the per-launch batch)")
    ap.add_argument("--enc01", action="store_true")
    ap.add_argument("--chain-wh", type=int, default=0, help="chain workgroup shape (option chain_wh), 0: the tuning's")
    ap.add_argument("--chain-x", type=int, default=-1, help="option chain_x (stride-2 head / tail), -1: the tuning's")
    args = ap.parse_args()
    path = os.path.join(tempfile.mkdtemp(), "chain_ts.bin")
    os.environ["TIC_ENC01_TIMING" if args.enc01 else "TIC_CHAIN_TIMING"] = path
    sys.path.insert(0, ROOT)
    from tf_image_compression_amd.codec import Codec
    from tf_image_compression_amd.weights import synthetic_params, SYNTH_MEAN, SYNTH_STD
    from tf_image_compression_amd.topology import bottleneck_shape
    P, B, M = 256, args.batch, 0
    c = Codec(M, synthetic_params(M, seed=0), SYNTH_MEAN, SYNTH_STD, patch_size=P)
    c.set_option("streams", args.streams)
    with open(args.tune_file) as f:
        c.tuning_import(json.load(f)["tuning"])
    if not args.enc01:
        c.set_option("chain", 1)
        if args.chain_wh:
            c.set_option("chain_wh", args.chain_wh)
        if args.chain_x >= 0:
            c.set_option("chain_x", args.chain_x)
    eh, ew, ec = bottleneck_shape(M, P)
    x = np.random.default_rng(1234).integers(0, 256, (B, P, P, 3), dtype=np.uint8)
    d_in, d_idx, d_rgb = c.alloc(x.nbytes), c.alloc(B * eh * ew * ec), c.alloc(x.nbytes)
    d_in.upload(x)
    for _ in range(args.steps):
        c.codec_device(d_in, B, d_idx, d_rgb)
    c.synchronize()  # dumps the last launch of every lane and side
    dumps = read_dumps(path)
    nl = 5
    for lane, slot, t in dumps:
        if slot == 2:
            rep = summarise_enc01(t)
            rep.update({"lane": lane, "kernel": "enc01"})
            print(json.dumps(rep), flush=True)
            continue
        rep = summarise(t, nl)
        rep.update({"lane": lane, "side": "decoder" if slot else "encoder"})
        print(json.dumps(rep), flush=True)
    c.close()


if __name__ == "__main__":
    main()
