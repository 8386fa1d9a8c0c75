#!/usr/bin/env python3
"""Drop-in for the reference's decode.py (same flags, paths and file naming):
``.encoded`` dir -> range decoder -> symbols [-1, eh, ew, ec] -> gfx950 decoder ->
stitched, cropped uint8 PNG ``<stem>.png`` (decode.py:143-264), with the optional
submit/2 block-effect post-filter (``--rmbe``, submit/2/decoder.py:184).

Reference: /root/reference/decode.py:20-76 (flags), :79-140 (range decoding, file-name
parsing), :143-264 (uncompress).  ``-g`` accepts -1..7 (-1 is accepted for
compatibility; there is no CPU path, so it maps to device 0 with a warning).
"""
import argparse
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from tf_image_compression_amd import utils  # noqa: E402
from tf_image_compression_amd.config import load_config  # noqa: E402


def my_parse_args(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("-m", "--model_num", type=str, choices=["0", "1", "2", "3"], required=True)
    p.add_argument("-g", "--gpu_num", type=str, choices=[str(i) for i in range(-1, 8)], required=True)
    p.add_argument("-d", "--debug_mode", type=str, choices=["on", "off"], default="off")
    p.add_argument("-p", "--params_file", type=str, default="")
    p.add_argument("-i", "--input_dir", type=str, default="model_{}/encoded_data")
    p.add_argument("-o", "--output_dir", type=str, default="model_{}/recons_data")
    p.add_argument("--norm", type=str, default="data_info/channel_normalization_params.npz")
    p.add_argument("--dist", type=str, default="data_info/distribution_info_{}.npy")
    p.add_argument("--synthetic-weights", action="store_true")
    p.add_argument("--raw", action="store_true", help="symbols stored bit-packed (encode.py --raw)")
    p.add_argument("--rmbe", type=str, default="", help="rmbe post-filter weights .npz (submit/2)")
    p.add_argument("--rmbe-norm", type=str, default="rmbe/channel_normalization_params.npz")
    return p.parse_args(argv)


def get_img_info(filename, config):
    """decode.py:104-115: '<stem>@_@h_w_c@_@len_H_W.encoded' -> (len, H, W)."""
    info = filename.replace(".encoded", "").split(config["name_sep"])[-1]
    seq_len, height, width = (int(v) for v in info.split("_"))
    return seq_len, height, width


def get_recons_image_path(filename, args, config):
    stem = filename.replace(".encoded", "").split(config["name_sep"])[0]
    return str(Path(args.output_dir.format(args.model_num)) / (stem + ".png"))


def get_encoded_shape(input_dir, config):
    """decode.py:130-140: the shape comes from the FIRST file name in the directory."""
    sample = sorted(f for f in os.listdir(input_dir) if f.endswith(".encoded"))[0]
    eh, ew, ec = (int(v) for v in sample.split(config["name_sep"])[1].split("_"))
    return eh, ew, ec


def apply_range_decoder(seq_len, path, cum_freq):
    from tf_image_compression_amd.range_coder import RangeDecoder
    dec = RangeDecoder(path)
    out = dec.decode_array(seq_len, cum_freq)
    dec.close()
    return out


def load_model(args, config):
    from tf_image_compression_amd.weights import load_normalization, synthetic_params
    import importlib
    model = importlib.import_module(f"tf_image_compression_amd.model_{args.model_num}.model")
    params = synthetic_params(int(args.model_num)) if args.synthetic_weights else utils.restore_params(args)
    mean, std = load_normalization(args.norm if os.path.exists(args.norm) else None)
    dev = int(args.gpu_num)
    if dev < 0:
        print("warning: -g -1 (TF-CPU) has no equivalent here; using HIP device 0", file=sys.stderr)
        dev = 0
    model.restore(params, mean, std, device=dev)
    return model


def uncompress(model, args):
    print(args)
    config = load_config(args.model_num)
    print(config)
    P, Q = config["patch_size"], config["quan_scale"]
    input_dir = args.input_dir.format(args.model_num)
    eh, ew, ec = get_encoded_shape(input_dir, config)
    codec = model.codec(P, Q)
    if tuple(codec.code_shape) != (eh, ew, ec):
        raise ValueError(f"encoded shape {(eh, ew, ec)} does not match model_{args.model_num} "
                         f"at patch {P}: {codec.code_shape}")
    cum_freq = None
    if not args.raw:
        from tf_image_compression_amd.range_coder import symbol_table
        cum_freq = symbol_table(np.load(args.dist.format(args.model_num), allow_pickle=False),
                                resolution=config["resolution"])
    post = None
    if args.rmbe:
        from tf_image_compression_amd.rmbe import RmbeFilter
        post = RmbeFilter.from_files(args.rmbe, args.rmbe_norm, device=codec.device)
    from tf_image_compression_amd.image_codec import ImageCodec
    ic = ImageCodec(codec, post.codec if post is not None else None)
    out_dir = args.output_dir.format(args.model_num)
    os.makedirs(out_dir, exist_ok=True)
    t0 = time.time()
    for filename in sorted(os.listdir(input_dir)):
        if not filename.endswith(".encoded"):
            continue
        path = str(Path(input_dir) / filename)
        seq_len, height, width = get_img_info(filename, config)
        if args.raw:
            raw = np.fromfile(path, np.uint8)
            seq = np.unpackbits(raw)[:seq_len] if Q == 2 else raw[:seq_len]
        else:
            seq = apply_range_decoder(seq_len, path, cum_freq)
        symbols = seq.astype(np.uint8).reshape(-1, eh, ew, ec)       # decode.py:204-208
        # decode -> concat_patches -> (rmbe) -> np.around, all on the GPU
        recons = ic.decode_image(symbols, height, width, post_filter=post is not None)
        out_path = get_recons_image_path(filename, args, config)
        print(f"recons_image_path: {out_path}")
        utils.imsave(out_path, recons)
    if args.debug_mode == "on":
        print(f"decode time {time.time() - t0:.3f}s")


if __name__ == "__main__":
    args = my_parse_args()
    cfg = load_config(args.model_num)
    uncompress(load_model(args, cfg), args)
