#!/usr/bin/env python3
"""Benchmark: encode+decode MPix/s on 256x256 RGB patches (BASELINE.json metric).

A step = one encode->decode pass (uint8 patches -> symbols -> uint8 reconstruction) of
one batch of synthetic patches already resident in HBM.  Default workload =
BASELINE.json configs[1]: model_0, batch 64, 256x256.  Multi-GPU: one process per GPU
(launched by torch.distributed.run), images sharded, weak scaling, no data-path
collective; RCCL is used for the barrier / max-over-ranks timing and the final
all-gather of per-rank stats.  Rank 0 prints ONE JSON line.

No PyTorch is imported in this process (torch bundles a second HIP runtime); the
torch.distributed launcher only provides RANK/LOCAL_RANK/WORLD_SIZE/MASTER_*.
"""
from __future__ import annotations

import argparse
import json
import re
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_FP32_TFLOPS = 157.3   # MI355X_MICROARCH.md: fp32 MFMA / vector peak (spec)
PEAK_HBM_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E peak (spec)
# Winograd F(2x2,3x3): 16 transform points per 2x2 output tile instead of 4 x 9 taps, so
# the minimal-form FLOP count of a stride-1 layer run in that form is 16/36 of the direct one
WINO_FRAC = 16.0 / 36.0
# Winograd F(4x4,3x3) (s1_form 2, conv3x3_wino4_kernel): 36 points per 4x4 tile, 36/144 = 1/4
WINO4_FRAC = 36.0 / 144.0
# polyphase Winograd of the stride-2 / transposed convs (s2_form 1, conv3x3_pwino_kernel):
# 25 points per tile against 36 products
PWINO_FRAC = 25.0 / 36.0


def wino_frac(kernel, kind="conv_s1"):
    """Minimal-form share of the direct-form FLOPs for a layer of `kind` run by `kernel`
    (Winograd forms of the stride-1 layers; a chain launch's stride-2 head / transposed tail
    runs the direct form, the polyphase kernel the stride-2 / transposed layers)."""
    if kind in ("conv_s1", "res"):
        return WINO4_FRAC if "wino4" in kernel else (WINO_FRAC if "wino" in kernel else 1.0)
    return PWINO_FRAC if "pwino" in kernel else 1.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tune-any-stamp", action="store_true",
                    help="with an explicit --tune-cache file: replay it even when its stamp names other sources")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--model", type=int, default=0)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--patch", type=int, default=256)
    ap.add_argument("--profile-iters", type=int, default=10)
    ap.add_argument("--profile-passes", type=int, default=5,
                    help="one-lane per-layer timing passes; the median picks the dominant launch")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline work (s)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-autotune", action="store_true")
    ap.add_argument("--streams", type=int, default=2, help="execution lanes (HIP streams) per GPU, 1..4")
    ap.add_argument("--tune-step", type=int, default=1,
                    help="rounds of in-situ (whole dual-lane step) tuning after the per-layer autotune; 0 = off")
    ap.add_argument("--graph", action="store_true", help="replay the launch sequence as a HIP graph (opt-in)")
    ap.add_argument("--traffic", default=None,
                    help="PMC summary (tools/pmc_summary.py) supplying roofline.traffic; default: the "
                         "committed tools/pmc/traffic_model<N>.json, used only if its source stamp "
                         "matches these kernel sources and its configuration matches this run")
    ap.add_argument("--tune-cache", default="auto",
                    help="tuning state (tic_tuning_export) to replay instead of tuning: 'auto' = the "
                         "shipped tf_image_compression_amd/tune/<config>.json when its source stamp "
                         "matches (else tune), "
                         "'none' = always tune, PATH = load if present and matching, else tune and save")
    ap.add_argument("--tune-save", default=None,
                    help="directory: save every state tuned in this run there under its canonical "
                         "name (model{M}_p{P}_b{B}_s{S}.json), for tf_image_compression_amd/tune/")
    ap.add_argument("--trace-only", action="store_true",
                    help="stop after the timed steps (for rocprofv3 timelines of the steady state)")
    ap.add_argument("--pmc-plan", default=None,
                    help="PMC mode (tools/pmc_box.sh): tune exactly as the bench does, then run --steps "
                         "steps on ONE lane at the per-lane batch (deterministic dispatch order), write "
                         "the launch plan of one step to this path, print nothing else")
    ap.add_argument("--reheat-s", type=float, default=2.0,
                    help="seconds of untimed two-lane steps after the one-lane profiling, before the in-step "
                         "timing and the timed region (0 = off)")
    ap.add_argument("--preheat-s", type=float, default=3.0,
                    help="seconds of untimed steps before any measurement (fresh-box clock ramp; 0 = off)")
    ap.add_argument("--in-step-min", type=int, default=50,
                    help="at least this many two-lane steps per in-step timing candidate (run before the "
                         "timed region; they also bring the GPU to its steady clock)")
    ap.add_argument("--layers-out", default=os.path.join(ROOT, "gpurun_out", "bench_layers.json"))
    ap.add_argument("--workload", choices=["patches", "image4k", "sharded"], default="patches",
                    help="patches: BASELINE configs[1]/[2] (default); image4k: configs[4], whole "
                         "3840x2160 images tiled 256x256 -> model_3 -> stitch -> rmbe post-filter -> u8; "
                         "sharded: configs[3], a synthetic image set split over the ranks, resident in "
                         "HBM, one step = one pass over every rank's shard + exact SSE + stats all-gather")
    ap.add_argument("--images", type=int, default=None,
                    help="image4k: images per rank per step (default 1); sharded: images in the whole "
                         "set (default 10000)")
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--width", type=int, default=3840)
    args = ap.parse_args()
    if args.workload == "image4k" and "--model" not in sys.argv:
        args.model = 3
    if args.images is None:
        args.images = 10000 if args.workload == "sharded" else 1
    return args


def traffic_path(args, model, lane_b):
    """roofline.traffic source: --traffic, else the committed PMC summary of this model at this
    per-launch batch (tools/pmc/traffic_model{M}_lb{lane_b}.json), else the model's default one
    (tools/pmc/traffic_model{M}.json; pmc_traffic rejects it when its lane batch differs)."""
    if args.traffic is not None:
        return args.traffic
    for name in (f"traffic_model{model}_lb{lane_b}.json", f"traffic_model{model}.json"):
        path = os.path.join(ROOT, "tools", "pmc", name)
        if os.path.exists(path):
            return path
    return ""


def kernel_groups(codec, model_id, P, ms, kernels=None):
    """Group layers by the kernel instance they launch (same template args + shape).  A
    layer whose kernel name is '' ran inside the previous layer's launch (enc01_kernel,
    dec10_kernel: a pair; wino_chain_kernel: a run of stride-1 layers): the launch is one
    group, its work the sum of its layers and its HBM bytes the first layer's input plus the
    last layer's output (the intermediate activations and residual inputs stay on chip); its
    time is the launch's (the layers inside have only an empty event pair of their own).
    A layer inside a Winograd launch counts the Winograd form's FLOPs."""
    from tf_image_compression_amd.topology import layer_work, RMBE_ID, weight_bytes
    work = layer_work(model_id, P)
    L = len(work)
    n_enc = sum(1 for lay, *_ in work if lay.stage == "enc")
    groups = {}
    rows = []
    direct = [f for _, f, _, _ in work]  # every layer's direct-form FLOPs
    if kernels is not None:  # the kernel each layer runs in ('' = the launch before it)
        launch = []
        for k in kernels:
            launch.append(k if k or not launch else launch[-1])
        def form_kernel(i):
            # a chain launch whose decode_2 behind the tail runs the polyphase form (HT bit 8,
            # CH_TAIL2_PW): its last layer counts that form
            m = re.match(r"wino_chain_kernel<\d+,\d+,\d+,(\d+)>", launch[i])
            last = i + 1 >= len(kernels) or kernels[i + 1] != ""
            return "pwino" if m and int(m.group(1)) & 8 and last else launch[i]
        work = [(lay, f * wino_frac(form_kernel(i), lay.kind), b, ho) for i, (lay, f, b, ho) in enumerate(work)]

    def out_res_bytes(i):
        lay, _, _, ho = work[i]
        if model_id != RMBE_ID and i == n_enc - 1:
            out_b = ho * ho * lay.cout  # u8 symbols
        elif i == L - 1:
            out_b = ho * ho * 3 * (4 if model_id == RMBE_ID else 1)
        else:
            out_b = ho * ho * lay.cout * 4
        return out_b, (ho * ho * lay.cout * 4 if lay.residual else 0)

    for i, (lay, flops, nbytes, ho) in enumerate(work):
        role = "rgb_in" if i == 0 else ("rgb_out" if i == L - 1 else
                                        ("quant" if (model_id != RMBE_ID and i == n_enc - 1) else
                                         ("dequant" if (model_id != RMBE_ID and i == n_enc) else "f32")))
        key = (lay.kind, lay.cin, lay.cout, lay.act, lay.residual, role, ho)
        rows.append({"layer": lay.name, "kind": lay.kind, "cin": lay.cin, "cout": lay.cout, "out_hw": ho,
                     "ms": float(ms[i]), "flops_per_patch": flops, "bytes_per_patch": nbytes,
                     "weight_bytes": weight_bytes(lay), "key": list(map(str, key))})
    i = 0
    while i < L:
        lay, flops, nbytes, ho = work[i]
        r = rows[i]
        key, names = tuple(r["key"]), [lay.name]
        f, b, wb, t = flops, nbytes, weight_bytes(lay), float(ms[i])
        fd = direct[i]
        j = i
        while kernels is not None and j + 1 < L and kernels[j + 1] == "":
            j += 1
            nl, nf, _, _ = work[j]
            f += nf
            fd += direct[j]
            wb += weight_bytes(nl)
            names.append(nl.name)  # its own ms is only the event pair recorded after the launch
            key = key + ("fused", nl.name)
        if j > i:  # first layer's input + last layer's output
            o_i, r_i = out_res_bytes(i)
            o_j, _ = out_res_bytes(j)
            b = (nbytes - o_i - r_i) + o_j
        g = groups.setdefault(key, {"layers": [], "ms": 0.0, "flops": f, "direct_flops": fd, "bytes": b, "wbytes": wb,
                                    "launches": 0})
        g["layers"].extend(names)
        g["ms"] += t
        g["launches"] += 1
        i = j + 1
    return groups, rows


def kernel_families(groups, kernels, names):
    """Launch groups merged by kernel template (the instance name up to '<'): the encoder and
    decoder chain runs are one family, as are the same conv template at two shapes.  The
    dominant launch is the family with the most one-lane time per step (a tie between two
    launches of one template, e.g. the two chains at 50.6 / 50.3 us, then cannot flip the pick
    from run to run — VERDICT r03 item 4); its roofline is over all its launches: the mean
    FLOPs / bytes per launch over the mean duration."""
    fams = {}
    for k, g in groups.items():
        inst = kernels[names[g["layers"][0]]] if kernels is not None else "+".join(g["layers"])
        fams.setdefault(inst.split("<")[0], []).append(k)
    out = {}
    for fam, members in fams.items():
        L = sum(groups[k]["launches"] for k in members)
        mean = lambda f: sum(groups[k][f] * groups[k]["launches"] for k in members) / L
        out[fam] = {"members": members, "layers": [nm for k in members for nm in groups[k]["layers"]],
                    "ms": sum(groups[k]["ms"] for k in members), "launches": L,
                    "flops": mean("flops"), "direct_flops": mean("direct_flops"), "bytes": mean("bytes"),
                    "wbytes": mean("wbytes")}
    return out


def roofline_of(group, batch):
    flops = group["flops"] * batch
    nbytes = group["bytes"] * batch + group["wbytes"]
    ms = group["ms"] / group.get("launches", len(group["layers"]))  # mean duration per launch
    t_c = flops / (PEAK_FP32_TFLOPS * 1e12)
    t_m = nbytes / (PEAK_HBM_GBS * 1e9)
    if t_m > t_c:
        achieved = nbytes / (ms * 1e-3) / 1e9
        return {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": round(achieved / PEAK_HBM_GBS, 4)}, ms, flops, nbytes
    achieved = flops / (ms * 1e-3) / 1e12
    return {"bound": "mfma", "achieved": round(achieved, 2), "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
            "frac": round(achieved / PEAK_FP32_TFLOPS, 4)}, ms, flops, nbytes


def step_roofline(rows, batch, step_ms):
    t_min = 0.0
    for r in rows:
        f = r["flops_per_patch"] * batch
        b = r["bytes_per_patch"] * batch + r["weight_bytes"]
        t_min += max(f / (PEAK_FP32_TFLOPS * 1e12), b / (PEAK_HBM_GBS * 1e9))
    return t_min * 1e3 / step_ms


def winograd_note(roof, kernels, group, batch, ms):
    """A group with Winograd layers counts their minimal-form FLOPs (F(2x2,3x3): 16/36,
    F(4x4,3x3): 36/144 of the direct form: kernel_groups), so `achieved`/`frac` are what the
    matrix cores ran and frac <= 1; the direct-form equivalent rate is reported beside it.  A
    mixed-form group (a chain launch with its direct stride-2 head / transposed tail) converts
    only its Winograd layers: the equivalent rate is the group's direct-form FLOPs (every layer
    in the direct form, kernel_groups' `direct_flops`) over the launch time (VERDICT r05 item 6:
    dividing the whole group by 16/36 overstated it by 36 %)."""
    if kernels and all("pwino" in k for k in kernels):
        roof["flop_form"] = "polyphase winograd minimal form: 25/36 of the direct-form FLOPs"
        roof["direct_equiv_tflops"] = round(group["direct_flops"] * batch / (ms * 1e-3) / 1e12, 2)
    elif kernels and any("wino" in k for k in kernels):
        f4 = all("wino4" in k for k in kernels)
        form = ("winograd F(4x4,3x3) minimal form: 36/144 of the direct-form FLOPs" if f4 else
                "winograd F(2x2,3x3) minimal form: 16/36 of the direct-form FLOPs")
        if abs(group["direct_flops"] * wino_frac(kernels[0]) - group["flops"]) > 1e-6 * group["flops"]:
            form += (" for the stride-1 layers; the stride-2 / transposed ones in their own form (direct, or"
                     " polyphase winograd 25/36 where the s2_form policy runs it)")
        roof["flop_form"] = form
        roof["direct_equiv_tflops"] = round(group["direct_flops"] * batch / (ms * 1e-3) / 1e12, 2)


def launch_units(layer_names, kernels, names):
    """Launch units of a kernel group: a layer, or 'a+b' where layer b ran inside layer a's
    launch (kernel name '' = fused into the previous layer)."""
    units = []
    for nm in layer_names:
        i = names[nm]
        if kernels[i] == "":
            continue
        j = i + 1
        unit = [nm]
        inv = {v: k for k, v in names.items()}
        while j < len(kernels) and kernels[j] == "":
            unit.append(inv[j])
            j += 1
        units.append("+".join(unit))
    return units


def pmc_traffic(path, units, cfg):
    """roofline.traffic: HBM bytes per launch of the dominant kernel group from a PMC summary
    written by tools/pmc_summary.py (separate FETCH_SIZE / WRITE_SIZE passes of this same
    bench under rocprofv3, gfx950 corrections), keyed by launch unit.  Used only when the
    summary's source stamp equals these kernel sources and its model / patch / per-launch
    batch equal this run's; otherwise traffic is null and the reason is given."""
    from tf_image_compression_amd._lib import source_digest
    out = {"traffic": None, "traffic_source": None}
    if not path or not os.path.exists(path):
        out["traffic_note"] = "no PMC summary for this model"
        return out
    tr = json.load(open(path))
    meta = tr.get("_meta", {})
    rel = os.path.relpath(path, ROOT)
    if meta.get("source_sha256") != source_digest():
        out["traffic_note"] = f"{rel} was measured on other kernel sources (stamp mismatch): not used"
        return out
    for k, v in cfg.items():
        if meta.get(k) != v:
            out["traffic_note"] = f"{rel} was measured at {k}={meta.get(k)}, this run {k}={v}: not used"
            return out
    ents = [tr["units"][u] for u in units if u in tr.get("units", {})]
    if not ents:
        out["traffic_note"] = f"{rel} has no entry for {units}"
        return out
    out["traffic"] = round(float(np.mean([e["bytes"] for e in ents])))
    out["traffic_source"] = rel
    out["traffic_read_write"] = [round(float(np.mean([e["read_bytes"] for e in ents]))),
                                 round(float(np.mean([e["write_bytes"] for e in ents])))]
    return out


def host_cpu_info():
    """CPUs this process may run on (affinity and cgroup quota), and the CPU model."""
    info = {"nproc": os.cpu_count()}
    try:
        info["affinity"] = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        info["affinity"] = os.cpu_count()
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    info["cgroup_cpus"] = quota
    info["model"] = None
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                info["model"] = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    usable = info["affinity"] or 1
    if quota:
        usable = min(usable, max(1, int(quota)))
    info["usable"] = usable
    return info


def cpu_baseline(model_id, P, params, mean, std, batch, target_s):
    """The oracle in float32 (im2col + OpenBLAS SGEMM on every CPU this job may use) timed
    on the GPU box's host on the same workload: one warm-up run, then the median of >= 5
    timed runs of encode + decode of `batch` patches.  The reference's
    TF-CPU path cannot run here (TF-1.x absent), so this is a disclosed stand-in."""
    from oracle import tic_oracle as o
    try:
        from threadpoolctl import threadpool_limits
    except Exception:  # pragma: no cover
        threadpool_limits = None
    cpu = host_cpu_info()
    cores = cpu["usable"]
    n = batch
    x = np.random.default_rng(99).integers(0, 256, (n, P, P, 3), dtype=np.uint8)
    ctx = threadpool_limits(limits=cores) if threadpool_limits else None
    times = []
    try:
        def run():
            _, idx = o.encoder(params, mean, std, x, P, 2, model_id, acc=np.float32)
            o.decoder(params, mean, std, idx, 2, model_id, acc=np.float32)
        t_begin = time.perf_counter()
        run()  # warm-up
        while True:
            t0 = time.perf_counter()
            run()
            times.append(time.perf_counter() - t0)
            if len(times) >= 5 and time.perf_counter() - t_begin > target_s:
                break
    finally:
        if ctx is not None and hasattr(ctx, "unregister"):
            ctx.unregister()
    med = float(np.median(times))
    return {"value": round(n * P * P / med / 1e6, 3), "unit": "MPix/s", "cores": cores, "kind": "port",
            "host": cpu,
            "sample": f"oracle/tic_oracle.py float32 (im2col + OpenBLAS SGEMM, {cores} threads = every CPU "
                      f"this job may use), model_{model_id} batch {n} x {P}x{P} patches encode+decode, "
                      f"1 warm-up + median of {len(times)} runs ({sum(times):.1f} s timed)"}


def parity_probe(codec, model_id, P, params, mean, std):
    """Delta-PSNR vs the oracle on 2 structured patches (rank 0, outside the timed region)."""
    from oracle import tic_oracle as o
    from tf_image_compression_amd.synthetic import structured_patches
    pats = structured_patches(2, P, seed=5)
    idx, pre = codec.encode(pats, return_preact=True)
    ref_pre, ref_idx = o.encoder(params, mean, std, pats, P, 2, model_id)
    scale = max(1.0, float(np.abs(ref_pre).max()))
    safe = o.decision_margin(ref_pre, 2) > 1e-5 * scale
    rgb = codec.decode(idx)
    _, ref_u8 = o.decoder(params, mean, std, idx, 2, model_id)
    p_gpu = o.dataset_psnr(list(zip(pats, rgb)))
    p_ref = o.dataset_psnr(list(zip(pats, ref_u8)))
    return {"delta_psnr_db": round(abs(p_gpu - p_ref), 5),
            "symbol_mismatch_outside_band": int(np.count_nonzero((idx != ref_idx) & safe)),
            "symbols": int(idx.size)}


def main():
    args = parse()
    if args.workload == "image4k":
        return main_image(args)
    if args.workload == "sharded":
        return main_sharded(args)
    from tf_image_compression_amd.codec import Codec
    from tf_image_compression_amd.weights import synthetic_params, SYNTH_MEAN, SYNTH_STD
    from tf_image_compression_amd.topology import bottleneck_shape, layer_table
    from tf_image_compression_amd import dist

    rank, world, local = dist.env_rank()
    if world != args.gpus:
        # single-process run with --gpus 1, or a launcher mismatch
        if not (world == 1 and args.gpus == 1):
            print(f"warning: WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr)
    P, B, M = args.patch, args.batch, args.model
    params = synthetic_params(M, seed=0)
    # tuning="none": bench.py replays (or re-measures) the tuning state itself, below
    codec = Codec(M, params, SYNTH_MEAN, SYNTH_STD, patch_size=P, quan_scale=2, device=local, tuning="none")
    codec.set_option("streams", args.streams)
    codec.set_option("graph", 1 if args.graph else 0)
    comm = dist.make_comm(codec)
    eh, ew, ec = bottleneck_shape(M, P)

    x = np.random.default_rng(1234 + rank).integers(0, 256, (B, P, P, 3), dtype=np.uint8)
    d_in = codec.alloc(x.nbytes)
    d_in.upload(x)
    d_idx = codec.alloc(B * eh * ew * ec)
    d_rgb = codec.alloc(x.nbytes)

    # per-lane batch: with 2 lanes each kernel launch processes half the batch
    lane_b = -(-B // max(1, min(args.streams, B)))  # largest per-lane part of the batch
    tuning = "none"
    if not args.no_autotune:
        tuning = tune(args, codec, d_in, B, lane_b, M, P)
    if args.pmc_plan:
        return pmc_steady(args, codec, d_in, d_idx, d_rgb, lane_b, M, P)

    # per-layer kernel timing, outside the timed region: HIP events around each launch on
    # the lane's stream, one lane at the per-launch batch (lane_b), each launch running alone
    # (exclusive) — the median of --profile-passes passes; it picks the dominant launch group
    # (the most one-lane time per step) and gives its roofline fraction; the same launches are
    # also timed in-step (below) and reported beside it
    pre = preheat(args, lambda: codec.codec_device(d_in, B, d_idx, d_rgb), codec.synchronize)
    ms = one_lane_ms(codec, d_in, lane_b, args)
    # the one-lane profiling is a light load: the clock can drop during it and take a few
    # hundred steps to come back (two evidence runs of the driver's 20 steps read 7 % slow
    # after a full preheat: profiles/bench_m0_drv_r05{h,j}.json), so the steady two-lane steps
    # run again, right before the in-step timing and the timed region
    pre2 = preheat(args, lambda: codec.codec_device(d_in, B, d_idx, d_rgb), codec.synchronize, args.reheat_s)
    kernels = codec.layer_kernels(lane_b)
    groups, rows = kernel_groups(codec, M, P, ms, kernels)
    names = {lay.name: i for i, lay in enumerate(layer_table(M))}
    # candidates timed in-step: the four largest by one-lane time per step
    fams = kernel_families(groups, kernels, names)
    dom_fam = max(fams, key=lambda f: (fams[f]["ms"], fams[f]["flops"]))
    cands = list(fams[dom_fam]["members"])
    cands += [k for k in sorted(groups, key=lambda k: (-groups[k]["ms"], -groups[k]["flops"])) if k not in cands][
        :max(0, 4 - len(cands))]
    # the candidates' launches timed in-step, BEFORE the timed region: the same steady two-lane
    # steps with an event pair per lane around each candidate launch (inside the timed steps the
    # pairs would cost ≈ 2 %), warm-up steps first to settle the lanes.  Running them here also
    # brings the GPU to the clock it holds under sustained load: the kernels of a step get
    # ≈ 7 % faster over the first ≈ 30 steps after the light one-lane profiling (rocprofv3
    # kernel trace of a 20-step run: step span 411 -> 350 us), which 5 warm-up
    # steps alone do not cover
    in_step = {}
    n_in_step = max(args.in_step_min, min(args.steps, 200))
    if args.trace_only:  # the same sustained steps, without the event pairs
        for _ in range(len(cands) * (args.warmup + n_in_step)):
            codec.codec_device(d_in, B, d_idx, d_rgb)
    else:
        for k in cands:
            codec.set_option("mark_layer", names[groups[k]["layers"][0]])
            for _ in range(args.warmup):
                codec.codec_device(d_in, B, d_idx, d_rgb)
            codec.mark_durations()
            for _ in range(n_in_step):
                codec.codec_device(d_in, B, d_idx, d_rgb)
            in_step[k] = codec.mark_durations()
        codec.set_option("mark_layer", -1)
    for _ in range(args.warmup):
        codec.codec_device(d_in, B, d_idx, d_rgb)
    codec.synchronize()
    comm.barrier(dist.collective_timeout())  # ranks arrive after rank-dependent tuning / profiling
    codec.synchronize()
    t0 = time.perf_counter()
    wall0 = time.time()
    for _ in range(args.steps):
        codec.codec_device(d_in, B, d_idx, d_rgb)
    t_enq = time.perf_counter() - t0  # host time to enqueue the K steps (a host-bound loop shows here)
    codec.synchronize()
    comm.barrier()
    elapsed = time.perf_counter() - t0
    wall1 = time.time()
    t_max = comm.allreduce_max(elapsed)
    in_step = {k: v for k, v in in_step.items() if len(v)}
    # the dominant launch group: a fixed ranking — the most one-lane (exclusive) GPU time per
    # step (cands[0]).  The in-step ranking is reported beside it but does not choose: with
    # two lanes the in-step duration of a launch depends on what the other lane runs beside
    # it, which moves from run to run (model_0: the encoder chain 54 µs in one run, 75 in the
    # next, enc01 72-73 in both; rocprofv3 averages them within 0.1 %), so an in-step pick
    # named a different kernel on every other run
    members = fams[dom_fam]["members"]
    top_in_step = (max(in_step, key=lambda k: float(np.mean(in_step[k])) * groups[k]["launches"])
                   if in_step else None)
    marks = np.concatenate([in_step[k] for k in members if k in in_step] or [np.zeros(0)])
    if args.trace_only:
        if rank == 0:
            print(json.dumps({"trace_only": True, "ms_per_step": t_max * 1e3 / args.steps,
                              "launches_per_lane": sum(1 for k in codec.layer_kernels(lane_b) if k)}), flush=True)
        comm.close()
        codec.close()
        return

    # per-rank stats -> the one RCCL all-gather (SSE of the last reconstruction)
    rec = d_rgb.download(x.shape, np.uint8)
    sse = float(np.sum(np.square(rec.astype(np.float64) - x.astype(np.float64))))
    st = dist.RankStats(sse=sse * args.steps, dims=x.size * args.steps, bits=B * eh * ew * ec * args.steps,
                        images=B * args.steps, t_start=wall0, t_end=wall1)
    gathered = comm.allgather_stats(st)
    summary = dist.combine(gathered)
    ranks = rank_devices(comm, codec, rank, local)

    # the dominant group's roofline from its one-lane (exclusive) launch duration: a
    # kernel-quality figure; beside it the same launches timed in the steady two-lane steps
    # (sharing the chip with the other lane, as rocprofv3 --kernel-trace sees them there)
    dom = dict(fams[dom_fam])
    roof, dom_ms, dom_flops, dom_bytes = roofline_of(dom, lane_b)
    roof["timing"] = (f"one lane, each launch alone: HIP events per launch, median of {args.profile_passes} "
                      f"passes x {args.profile_iters} iterations")
    roof["dominant_by"] = ("the kernel template with the most one-lane (exclusive) GPU time per step, over "
                           "all its launches: a fixed ranking; the in-step duration beside it, and the "
                           "launch with the most in-step time per step (what rocprofv3 --kernel-trace "
                           "ranks first) in most_in_step_time when that is another kernel")
    if len(marks):
        di = dict(dom)
        di["ms"] = float(np.mean(marks)) * di["launches"]
        ri, rmsi, _, _ = roofline_of(di, lane_b)
        roof["ms_per_launch_in_step"] = round(rmsi, 5)
        roof["frac_in_step"] = ri["frac"]
        roof["timing_in_step"] = (f"HIP events around each of its {len(marks)} launches on the lane streams in "
                                  f"{n_in_step} two-lane steps run right before the timed region (mean)")
    # HBM bytes per launch of the dominant kernel instance from the committed PMC summary
    # (tools/pmc_box.sh + tools/pmc_summary.py; FETCH_SIZE x2 + WRITE_SIZE, gfx950 rules)
    dom_kernels = sorted({kernels[names[nm]] for nm in dom["layers"]} - {""})
    roof.update(pmc_traffic(traffic_path(args, M, lane_b), launch_units(dom["layers"], kernels, names),
                            {"model": M, "patch": P, "lane_batch": lane_b}))
    winograd_note(roof, dom_kernels, dom, lane_b, dom_ms)
    roof["kernel"] = " | ".join("+".join(groups[k]["layers"]) for k in members)
    roof["kernel_instance"] = dom_kernels
    roof["launches_per_step_per_lane"] = dom["launches"]
    roof["ms_per_launch"] = round(dom_ms, 5)
    if len(members) > 1:
        # the family mean spans several instances (e.g. model_3's F(4x4,3x3) conv at three
        # tilings and two map sizes): the roofline of its largest member beside it
        big = max(members, key=lambda k: groups[k]["ms"] / groups[k]["launches"])
        rb, rbms, _, _ = roofline_of(groups[big], lane_b)
        roof["largest_member"] = {"kernel": "+".join(groups[big]["layers"]),
                                  "kernel_instance": sorted({kernels[names[nm]] for nm in groups[big]["layers"]} - {""}),
                                  "ms_per_launch": round(rbms, 5), "achieved": rb["achieved"], "frac": rb["frac"]}
    if top_in_step is not None and top_in_step not in members:  # for the record
        r1, ms1, _, _ = roofline_of(groups[top_in_step], lane_b)
        gi = dict(groups[top_in_step])
        gi["ms"] = float(np.mean(in_step[top_in_step])) * gi["launches"]
        ri, rmsi, _, _ = roofline_of(gi, lane_b)
        roof["most_in_step_time"] = {"kernel": "+".join(groups[top_in_step]["layers"]), "frac": r1["frac"],
                                     "ms_per_launch": round(ms1, 5), "ms_per_launch_in_step": round(rmsi, 5),
                                     "frac_in_step": ri["frac"]}
    # every launch group's roofline from the one-lane timing (and in-step for the candidates)
    roof_groups = []
    for k in sorted(groups, key=lambda k: -groups[k]["ms"]):
        rg, rms, _, _ = roofline_of(groups[k], lane_b)
        row = {"kernel": "+".join(groups[k]["layers"]), "launches": groups[k]["launches"],
               "ms_per_launch": round(rms, 5), "bound": rg["bound"], "frac": rg["frac"]}
        if k in in_step:  # in-step duration (two lanes) and the roofline fraction it gives
            gi = dict(groups[k])
            gi["ms"] = float(np.mean(in_step[k])) * gi["launches"]
            ri, rmsi, _, _ = roofline_of(gi, lane_b)
            row.update({"ms_per_launch_in_step": round(rmsi, 5), "frac_in_step": ri["frac"]})
        roof_groups.append(row)

    step_ms = t_max * 1e3 / args.steps
    total_px = world * B * P * P * args.steps
    value = total_px / t_max / 1e6
    out = {
        "metric": "encode+decode MPix/s at 256x256 RGB",
        "value": round(value, 2),
        "unit": "MPix/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(step_ms, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic uniform u8 patches (seed 1234+rank), seeded He-normal weights",
        "config": {"workload": f"model_{M} encode+decode, batch={B} patches of {P}x{P} RGB per GPU",
                   "model": f"model_{M}", "global_batch": B * world, "patch": P,
                   "code_shape": [eh, ew, ec], "parallelism": f"image-parallel x{world}"},
        "roofline": roof,
        "roofline_groups": roof_groups,
        "roofline_step_frac": round(step_roofline(rows, B, step_ms), 4),
        "lanes": {"streams": args.streams, "patches_per_launch": lane_b, "hip_graph": bool(args.graph)},
        "host_enqueue_ms_per_step": round(t_enq * 1e3 / args.steps, 4),
        "preheat": pre,
        "reheat": pre2,
        "ranks": ranks,
        "tuning": tuning,
        "stats_allgather": {"images": summary["images"], "psnr_db": round(summary["psnr_db"], 3),
                            "raw_bpp": round(summary["bpp"], 4)},
    }
    if rank == 0:
        try:
            os.makedirs(os.path.dirname(args.layers_out), exist_ok=True)
            for r, v, kn in zip(rows, codec.layer_variants(lane_b), kernels):
                r["tile"] = list(v)
                r["kernel"] = kn
            json.dump({"config": out["config"], "step_ms": step_ms, "lane_batch": lane_b, "layers": rows,
                       "groups": {",".join(map(str, k)): {"layers": g["layers"], "ms": g["ms"]}
                                  for k, g in groups.items()}},
                      open(args.layers_out, "w"), indent=1)
        except OSError:
            pass
        out["parity"] = parity_probe(codec, M, P, params, SYNTH_MEAN, SYNTH_STD)
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(M, P, params, SYNTH_MEAN, SYNTH_STD,
                                               B if M in (0, 1) else min(B, 8), args.cpu_seconds)
            out["speedup_vs_cpu_baseline"] = round(value / out["cpu_baseline"]["value"], 1)
        print(json.dumps(out), flush=True)
    comm.close()
    codec.close()


def rank_devices(comm, codec, rank, local):
    """Every rank's (rank, LOCAL_RANK, HIP device, PCI address) through one all-gather: a
    multi-GPU record shows which devices RCCL joined."""
    import re
    info = codec.device_info()
    m = re.search(r"device (\d+) \| pci ([0-9a-f]+):([0-9a-f]+):([0-9a-f]+)", info)
    dev, dom, bus, fn = (int(m.group(1)), int(m.group(2), 16), int(m.group(3), 16), int(m.group(4), 16)) if m \
        else (-1, 0, 0, 0)
    rows = comm.allgather_f64([rank, local, dev, dom, bus, fn])
    return [{"rank": int(r[0]), "local_rank": int(r[1]), "device": int(r[2]),
             "pci": f"{int(r[3]):04x}:{int(r[4]):02x}:{int(r[5]):02x}"} for r in rows]


def preheat(args, step, sync, seconds=None):
    """Untimed steps for args.preheat_s seconds before any measurement, in chunks of 10 steps
    with the time of each chunk kept: on a fresh box the first process's steps run ≈ 7 %
    slower than the same steps a few seconds later, which the driver's 5 warm-up
    steps do not cover; the chunk times show the ramp."""
    seconds = args.preheat_s if seconds is None else seconds
    out = {"seconds": seconds, "steps": 0, "ms_per_step_by_chunk": []}
    if seconds <= 0:
        return out
    sync()
    t_start = time.perf_counter()
    while time.perf_counter() - t_start < seconds:
        t = time.perf_counter()
        for _ in range(10):
            step()
        sync()
        out["ms_per_step_by_chunk"].append(round((time.perf_counter() - t) * 100.0, 4))
        out["steps"] += 10
    c = out["ms_per_step_by_chunk"]
    out["ms_per_step_by_chunk"] = c if len(c) <= 12 else c[:6] + c[-6:]  # first and last chunks
    return out


def one_lane_ms(codec, d_in, lane_b, args):
    """Per-layer one-lane launch durations (ms): the median over args.profile_passes passes
    of tic_profile_layers (args.profile_iters iterations each), after a warm pass."""
    codec.profile_layers(d_in, lane_b, 2)  # first use of the one-lane path: allocations, caches
    runs = [codec.profile_layers(d_in, lane_b, args.profile_iters) for _ in range(max(1, args.profile_passes))]
    return np.median(np.stack(runs), axis=0)


def tune_cache_path(args, M, P, B):
    """(state to replay if present and matching, where to save a state tuned in this run)."""
    from tf_image_compression_amd import tuning
    name = os.path.basename(tuning.tune_path(M, P, B, args.streams))
    save = os.path.join(args.tune_save, name) if args.tune_save else None
    if args.tune_cache == "none":
        return None, save
    if args.tune_cache == "auto":
        return tuning.tune_path(M, P, B, args.streams), save
    return args.tune_cache, save or args.tune_cache


def tune(args, codec, d_in, B, lane_b, M, P, search=True):
    """Per-layer autotune + in-situ step tuning (outside the timed region), or the replay of
    the shipped tuning state (tf_image_compression_amd/tune/, the same file Codec applies by
    default) when it was measured on these kernel sources and this configuration.  With
    search False only the replay is done (the runtime's defaults stand without one)."""
    from tf_image_compression_amd import tuning
    path, save = tune_cache_path(args, M, P, B)
    stamp = tuning.stamp(M, P, B, args.streams, args.tune_step)
    if path and os.path.exists(path):
        doc = json.load(open(path))
        if doc.get("_meta") == stamp:
            codec.tuning_import(doc["tuning"])
            return os.path.relpath(path, ROOT)
        if args.tune_any_stamp and args.tune_cache not in ("auto", "none"):
            # investigation runs (tools/kcounters.sh on candidate sources): the same launch plan
            # replayed although its stamp names other sources — never the product's default
            codec.tuning_import(doc["tuning"])
            return os.path.relpath(path, ROOT) + " (replayed despite a stamp mismatch: --tune-any-stamp)"
    if not search:
        return "none (no replayable tuning; a shard smaller than one batch on some rank)"
    codec.autotune(d_in, lane_b, reps=5)  # per-layer tiling choice
    if args.tune_step > 0:  # then per layer by the whole step as it runs (both lanes)
        codec.autotune_step(d_in, B, rounds=args.tune_step, reps=5)
    if save:
        os.makedirs(os.path.dirname(os.path.abspath(save)), exist_ok=True)
        json.dump({"_meta": stamp, "tuning": codec.tuning_export()}, open(save, "w"), indent=1)
    return "tuned in this run"


def pmc_steady(args, codec, d_in, d_idx, d_rgb, lane_b, M, P):
    """--pmc-plan: after the bench's own tuning, run --steps steps on ONE lane at the
    per-lane batch (the tuned choices are keyed by that batch, so every launch is the
    bench's), with the launch plan of one step written for tools/pmc_summary.py."""
    from tf_image_compression_amd._lib import source_digest, lib_digest
    from tf_image_compression_amd.topology import layer_table
    kernels = codec.layer_kernels(lane_b)
    names = [lay.name for lay in layer_table(M)]
    plan = []
    for i, k in enumerate(kernels):
        if k == "":
            plan[-1]["unit"] += "+" + names[i]
            continue
        plan.append({"unit": names[i], "kernel": k})
    codec.set_option("streams", 1)
    for _ in range(args.warmup):
        codec.codec_device(d_in, lane_b, d_idx, d_rgb)
    codec.synchronize()
    for _ in range(args.steps):
        codec.codec_device(d_in, lane_b, d_idx, d_rgb)
    codec.synchronize()
    meta = {"model": M, "patch": P, "lane_batch": lane_b, "steps": args.steps, "source_sha256": source_digest(),
            "libtic_sha256": lib_digest(), "streams_in_bench": args.streams}
    os.makedirs(os.path.dirname(os.path.abspath(args.pmc_plan)), exist_ok=True)
    json.dump({"_meta": meta, "plan": plan}, open(args.pmc_plan, "w"), indent=1)
    codec.close()


def main_sharded(args):
    """BASELINE configs[3]: a synthetic set of args.images 256x256 images split statically
    over the ranks (dist.shard_range), each rank's shard resident in HBM (uploaded before
    the timed region), one step = one pass of tic_codec_device over the shard in batches of
    args.batch (the shipped tuning) + the exact SSE kernel; after the timed steps ONE RCCL
    all-gather of the per-rank stats gives the dataset PSNR (processing_utils/evaluate.py:
    18-32).  value = images x P^2 of all ranks x steps / max-over-ranks time."""
    from tf_image_compression_amd.codec import Codec
    from tf_image_compression_amd.weights import synthetic_params, SYNTH_MEAN, SYNTH_STD
    from tf_image_compression_amd.topology import bottleneck_shape
    from tf_image_compression_amd import dist, sharded

    rank, world, local = dist.env_rank()
    P, B, M, NI = args.patch, args.batch, args.model, args.images
    params = synthetic_params(M, seed=0)
    codec = Codec(M, params, SYNTH_MEAN, SYNTH_STD, patch_size=P, quan_scale=2, device=local, tuning="none")
    codec.set_option("streams", args.streams)
    comm = dist.make_comm(codec)
    eh, ew, ec = bottleneck_shape(M, P)
    lo, hi = dist.shard_range(NI, rank, world)
    t_gen = time.perf_counter()
    shard = sharded.DeviceShard(codec, sharded.shard_images(NI, rank, world, P, "uniform"), B)
    t_gen = time.perf_counter() - t_gen
    lane_b = -(-B // max(1, min(args.streams, B)))
    tuning = "none"
    # the same decision on every rank: searching needs a full batch on the
    # rank's own shard, so it runs everywhere or nowhere; the replay needs no shard
    search = dist.all_ranks(comm, shard.n >= B)
    if not args.no_autotune:
        tuning = tune(args, codec, shard.d_img, B, lane_b, M, P, search=search)
    for _ in range(args.warmup):
        shard.enqueue()
    codec.synchronize()
    comm.barrier(dist.collective_timeout())  # ranks arrive after rank-dependent tuning / profiling
    codec.synchronize()
    t0 = time.perf_counter()
    wall0 = time.time()
    for _ in range(args.steps):
        shard.enqueue()
    codec.synchronize()
    comm.barrier()
    elapsed = time.perf_counter() - t0
    wall1 = time.time()
    t_max = comm.allreduce_max(elapsed)
    st = shard.stats(args.steps, wall0, wall1)
    summary = dist.combine(comm.allgather_stats(st))
    ranks = rank_devices(comm, codec, rank, local)
    # the one-lane roofline of the dominant launch group at the shard's batch (as configs[1])
    ms = one_lane_ms(codec, shard.d_img, lane_b, args) if shard.n >= lane_b else None
    roof = None
    if ms is not None:
        kernels = codec.layer_kernels(lane_b)
        groups, _ = kernel_groups(codec, M, P, ms, kernels)
        from tf_image_compression_amd.topology import layer_table
        names = {lay.name: i for i, lay in enumerate(layer_table(M))}
        fams = kernel_families(groups, kernels, names)
        dom = fams[max(fams, key=lambda f: (fams[f]["ms"], fams[f]["flops"]))]
        roof, dom_ms, dom_flops, _ = roofline_of(dom, lane_b)
        dom_kernels = sorted({kernels[names[nm]] for nm in dom["layers"]} - {""})
        winograd_note(roof, dom_kernels, dom, lane_b, dom_ms)
        roof.update(pmc_traffic(traffic_path(args, M, lane_b), launch_units(dom["layers"], kernels, names),
                                {"model": M, "patch": P, "lane_batch": lane_b}))
        roof["kernel"] = " | ".join("+".join(groups[k]["layers"]) for k in dom["members"])
        roof["kernel_instance"] = dom_kernels
        roof["ms_per_launch"] = round(dom_ms, 5)
        roof["timing"] = "one-lane per-layer HIP events (profile_layers)"
    step_ms = t_max * 1e3 / args.steps
    value = NI * P * P * args.steps / t_max / 1e6
    out = {
        "metric": "encode+decode MPix/s at 256x256 RGB",
        "value": round(value, 2),
        "unit": "MPix/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(step_ms, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic uniform u8 images (seeded by global image index), seeded He-normal weights",
        "config": {"workload": f"model_{M}, {NI}-image synthetic set of {P}x{P} RGB sharded over {world} GPU(s), "
                               f"batches of {B}, RCCL stats all-gather (BASELINE configs[3])",
                   "model": f"model_{M}", "images": NI, "images_per_rank": hi - lo, "patch": P, "batch": B,
                   "code_shape": [eh, ew, ec], "parallelism": f"image-parallel x{world}"},
        "roofline": roof,
        "lanes": {"streams": args.streams, "patches_per_launch": lane_b},
        "tuning": tuning,
        "shard_upload_s": round(t_gen, 2),
        "ranks": ranks,
        "stats_allgather": {"images": summary["images"], "psnr_db": round(summary["psnr_db"], 3),
                            "raw_bpp": round(summary["bpp"], 4), "per_step_images": summary["images"] // args.steps},
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    shard.free()
    comm.close()
    codec.close()


def cpu_baseline_image(model_id, P, params, mean, std, rparams, H, W, target_s):
    """Oracle (float32, OpenBLAS) on a bounded sample — 2 codec patches + 4 rmbe windows,
    timed repeatedly — extrapolated to one HxW image (patch and window counts of the
    image); the reference's TF-CPU path cannot run here."""
    from oracle import tic_oracle as o
    try:
        from threadpoolctl import threadpool_limits
    except Exception:  # pragma: no cover
        threadpool_limits = None
    cpu = host_cpu_info()
    cores = cpu["usable"]
    n_p, n_w = 2, 4
    r = np.random.default_rng(98)
    x = r.integers(0, 256, (n_p, P, P, 3), dtype=np.uint8)
    win = r.random((n_w, 128, 128, 3), dtype=np.float32) * 255
    ctx = threadpool_limits(limits=cores) if threadpool_limits else None
    tp, tw = [], []
    try:
        t_begin = time.perf_counter()
        while True:
            t0 = time.perf_counter()
            _, idx = o.encoder(params, mean, std, x, P, 2, model_id, acc=np.float32)
            o.decoder(params, mean, std, idx, 2, model_id, acc=np.float32)
            t1 = time.perf_counter()
            o.rmbe_model(rparams, mean, std, win, acc=np.float32)
            tw.append(time.perf_counter() - t1)
            tp.append(t1 - t0)
            if time.perf_counter() - t_begin > target_s and len(tp) >= 2:
                break
    finally:
        if ctx is not None and hasattr(ctx, "unregister"):
            ctx.unregister()
    hn, wn = -(-H // P), -(-W // P)
    n_win = (H // 128) * ((W - 64) // 128) + ((H - 64) // 128) * (W // 128)
    t_img = float(np.median(tp)) / n_p * hn * wn + float(np.median(tw)) / n_w * n_win
    return {"value": round(H * W / t_img / 1e6, 4), "unit": "MPix/s", "cores": cores, "kind": "port",
            "host": cpu, "sample": f"oracle/tic_oracle.py float32 (OpenBLAS {cores} threads): model_{model_id} "
                      f"{n_p} x {P}x{P} patches encode+decode and rmbe {n_w} x 128x128 windows, median of "
                      f"{len(tp)} runs, extrapolated to {hn * wn} patches + {n_win} windows of one "
                      f"{W}x{H} image"}


def main_image(args):
    """BASELINE configs[4]: whole images, device-resident from the uint8 image to the uint8
    reconstruction: reflect tiling -> model encode -> decode (f32) -> stitch -> rmbe
    (2 window passes) -> np.around -> uint8.  One step = args.images images per rank."""
    from tf_image_compression_amd.codec import Codec
    from tf_image_compression_amd.image_codec import ImageCodec
    from tf_image_compression_amd.weights import synthetic_params, SYNTH_MEAN, SYNTH_STD
    from tf_image_compression_amd.topology import bottleneck_shape, RMBE_ID
    from tf_image_compression_amd import dist

    rank, world, local = dist.env_rank()
    P, M, H, W, NI = args.patch, args.model, args.height, args.width, args.images
    params = synthetic_params(M, seed=0)
    rparams = synthetic_params(RMBE_ID, seed=0)
    codec = Codec(M, params, SYNTH_MEAN, SYNTH_STD, patch_size=P, quan_scale=2, device=local, tuning="none")
    post = Codec(RMBE_ID, rparams, SYNTH_MEAN, SYNTH_STD, patch_size=128, device=local, tuning="none")
    for c in (codec, post):
        c.set_option("streams", args.streams)
    comm = dist.make_comm(codec)
    ic = ImageCodec(codec, post)
    eh, ew, ec = bottleneck_shape(M, P)
    npat = ic.num_patches(H, W)
    r = np.random.default_rng(1234 + rank)
    imgs = [r.integers(0, 256, (H, W, 3), dtype=np.uint8) for _ in range(NI)]
    d_img = [codec.alloc(H * W * 3) for _ in range(NI)]
    for d, x in zip(d_img, imgs):
        d.upload(x)
    d_sym = [codec.alloc(npat * eh * ew * ec) for _ in range(NI)]
    d_out = [codec.alloc(H * W * 3) for _ in range(NI)]

    lane_b = -(-npat // max(1, min(args.streams, npat)))
    n_win = (H // 128) * ((W - 64) // 128) + ((H - 64) // 128) * (W // 128)
    win_b = min(n_win, 256)  # rmbe windows per launch sequence (the handle's chunk)
    win_lane = -(-win_b // max(1, min(args.streams, win_b)))
    d_pat = codec.alloc(npat * P * P * 3)
    codec.image_to_patches_device(d_img[0], H, W, P, d_pat)
    d_win = post.alloc(win_b * 128 * 128 * 3 * 4)
    d_win.upload(r.random((win_b, 128, 128, 3), dtype=np.float32) * 255)
    tuning = {"codec": "none", "rmbe": "none"}
    if not args.no_autotune:
        # both networks tuned like configs[1]: per-layer autotune + the whole-step tuner
        # (fusions, chain, variants), or the replay of the shipped state for this shape
        tuning["codec"] = tune(args, codec, d_pat, npat, lane_b, M, P)
        tuning["rmbe"] = tune(args, post, d_win, win_b, win_lane, RMBE_ID, 128)

    def step():
        for i in range(NI):
            ic.roundtrip_device(d_img[i], H, W, d_sym[i], d_out[i], post_filter=True)

    for _ in range(args.warmup):
        step()
    ic.synchronize()
    comm.barrier(dist.collective_timeout())  # ranks arrive after rank-dependent tuning / profiling
    ic.synchronize()
    t0 = time.perf_counter()
    wall0 = time.time()
    for _ in range(args.steps):
        step()
    ic.synchronize()
    comm.barrier()
    elapsed = time.perf_counter() - t0
    wall1 = time.time()
    t_max = comm.allreduce_max(elapsed)

    sse = 0.0
    for d, x in zip(d_out, imgs):
        rec = d.download(x.shape, np.uint8)
        sse += float(np.sum(np.square(rec.astype(np.float64) - x.astype(np.float64))))
    st = dist.RankStats(sse=sse * args.steps, dims=NI * H * W * 3 * args.steps,
                        bits=NI * npat * eh * ew * ec * args.steps, images=NI * args.steps,
                        t_start=wall0, t_end=wall1)
    summary = dist.combine(comm.allgather_stats(st))
    ranks = rank_devices(comm, codec, rank, local)

    # per-layer HIP-event timing of both networks at their per-launch batch sizes
    ms_c = one_lane_ms(codec, d_pat, lane_b, args)
    ms_r = one_lane_ms(post, d_win, win_lane, args)
    groups, rows = kernel_groups(codec, M, P, ms_c, codec.layer_kernels(lane_b))
    rgroups, rrows = kernel_groups(post, RMBE_ID, 128, ms_r, post.layer_kernels(win_lane))
    # dominant = largest time per image: per-launch ms x launches per image
    per_img = {("codec",) + k: (g, lane_b, npat) for k, g in groups.items()}
    per_img.update({("rmbe",) + k: (g, win_lane, n_win) for k, g in rgroups.items()})
    dom_key = max(per_img, key=lambda k: per_img[k][0]["ms"] * per_img[k][2] / per_img[k][1])
    g, lb, _ = per_img[dom_key]
    roof, dom_ms, dom_flops, _ = roofline_of(g, lb)
    from tf_image_compression_amd.topology import layer_table
    net, net_id = (post, RMBE_ID) if dom_key[0] == "rmbe" else (codec, M)
    kern = net.layer_kernels(lb)
    idx = {lay.name: i for i, lay in enumerate(layer_table(net_id))}
    dom_kernels = sorted({kern[idx[nm]] for nm in g["layers"]} - {""})
    winograd_note(roof, dom_kernels, g, lb, dom_ms)
    # HBM bytes per launch: only from a PMC summary of this exact configuration
    roof.update(pmc_traffic(traffic_path(args, net_id, lb), launch_units(g["layers"], kern, idx),
                            {"model": net_id, "patch": P if dom_key[0] != "rmbe" else 128, "lane_batch": lb}))
    roof["kernel_instance"] = dom_kernels
    roof["kernel"] = ("rmbe:" if dom_key[0] == "rmbe" else f"model_{M}:") + "+".join(g["layers"])
    roof["ms_per_launch"] = round(dom_ms, 5)
    # step roofline: both networks' layers at the image's patch / window counts
    t_min = 0.0
    for rr, cnt in [(rows, npat), (rrows, n_win)]:
        for x in rr:
            t_min += max(x["flops_per_patch"] * cnt / (PEAK_FP32_TFLOPS * 1e12),
                         (x["bytes_per_patch"] * cnt + x["weight_bytes"]) / (PEAK_HBM_GBS * 1e9))
    step_ms = t_max * 1e3 / args.steps
    value = world * NI * H * W * args.steps / t_max / 1e6
    out = {
        "metric": "encode+decode MPix/s at 256x256 RGB",
        "value": round(value, 2),
        "unit": "MPix/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(step_ms, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic uniform u8 images (seed 1234+rank), seeded He-normal weights",
        "config": {"workload": f"model_{M} + rmbe post-filter, {NI} x {W}x{H} RGB image(s) per GPU tiled "
                               f"{P}x{P} ({npat} patches, {n_win} rmbe windows per image)",
                   "model": f"model_{M}+rmbe", "images_per_gpu": NI, "image": [H, W], "patch": P,
                   "code_shape": [eh, ew, ec], "parallelism": f"image-parallel x{world}"},
        "roofline": roof,
        "roofline_step_frac": round(t_min * NI * 1e3 / step_ms, 4),
        "lanes": {"streams": args.streams, "patches_per_launch": lane_b, "windows_per_launch": win_lane},
        "ranks": ranks,
        "tuning": tuning,
        "stats_allgather": {"images": summary["images"], "psnr_db": round(summary["psnr_db"], 3),
                            "raw_bpp": round(summary["bpp"], 4)},
    }
    if rank == 0:
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline_image(M, P, params, SYNTH_MEAN, SYNTH_STD, rparams, H, W,
                                                     args.cpu_seconds)
            out["speedup_vs_cpu_baseline"] = round(value / out["cpu_baseline"]["value"], 1)
        print(json.dumps(out), flush=True)
    ic.close()
    comm.close()
    post.close()
    codec.close()


if __name__ == "__main__":
    main()
