#!/usr/bin/env python3
"""Drop-in for the reference's encode.py (same flags, paths, file naming and symbol
order): image list -> reflect-padded 256^2 (or 128^2) patches -> gfx950 encoder ->
uint8 symbols (patch-major, then h, w, C) -> range coder -> ``.encoded`` files named
``<stem>@_@{eh}_{ew}_{ec}@_@{len}_{H}_{W}.encoded`` (encode.py:102-122).

Reference: /root/reference/encode.py:17-73 (flags), :76-97 (range coding), :125-212
(compress).  Differences: ``-g`` picks a HIP device (0..7) instead of setting
CUDA_VISIBLE_DEVICES; ``-p`` names the TF checkpoint prefix (read by tf_checkpoint.py) or an
.npz of the same variables; the image is uploaded once and reflect-tiled on the GPU
(image_codec.py), and all its patches go through the encoder in one call instead of
``sess.run`` batches of 64.  Extra optional flags: ``--norm`` (channel statistics
npz), ``--dist`` (symbol distribution npy), ``--synthetic-weights`` (seeded weights when
no checkpoint exists), ``--raw`` (store bit-packed symbols, no entropy coding).
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
    p.add_argument("-m", "--model_num", type=str, choices=["0", "1", "2", "3"], required=True,
                   help="Determine which model to use")
    p.add_argument("-g", "--gpu_num", type=str, choices=[str(i) for i in range(8)], required=True,
                   help="Determine which gpu to use")
    p.add_argument("-d", "--debug_mode", type=str, choices=["on", "off"], default="off")
    p.add_argument("-p", "--params_file", type=str, default="", help="File for model parameters (.npz)")
    p.add_argument("-v", "--data_list", type=str, default="data_info/tiny_valid_data_list.txt",
                   help="File for data_list")
    p.add_argument("-o", "--output_dir", type=str, default="model_{}/encoded_data",
                   help="Directory for output compressed data")
    p.add_argument("--norm", type=str, default="data_info/channel_normalization_params.npz")
    p.add_argument("--dist", type=str, default="data_info/distribution_info_{}.npy")
    p.add_argument("--synthetic-weights", action="store_true")
    p.add_argument("--raw", action="store_true", help="bit-pack symbols instead of range coding")
    return p.parse_args(argv)


def symbol_table(args, config):
    """encode.py:77-86: prob -> prob*resolution+1 -> renormalise -> prob_to_cum_freq."""
    from tf_image_compression_amd.range_coder import symbol_table as table
    path = args.dist.format(args.model_num)
    prob = np.load(path, allow_pickle=False)
    return table(prob, resolution=config["resolution"])


def apply_range_encoder(seq_data, encodepath, args, config, cum_freq):
    from tf_image_compression_amd.range_coder import RangeEncoder
    enc = RangeEncoder(encodepath)
    enc.encode(seq_data, cum_freq)
    enc.close()


def get_encodepath(image_path, image, seq_len, args, config, encoded_patches_shape):
    encoded_save_dir = args.output_dir.format(args.model_num)
    stem = image_path.split("/")[-1].replace(".png", "")
    height, width, _ = image.shape
    eh, ew, ec = encoded_patches_shape
    sep = config["name_sep"]
    info = sep + f"{eh}_{ew}_{ec}" + sep + f"{seq_len}_{height}_{width}"
    return str(Path(encoded_save_dir) / stem) + info + ".encoded"


def load_model(args, config):
    from tf_image_compression_amd.weights import load_normalization, synthetic_params
    import importlib
    model = importlib.import_module(f"tf_image_compression_amd.model_{args.model_num}.model")
    if args.synthetic_weights:
        params = synthetic_params(int(args.model_num))
    else:
        params = utils.restore_params(args)
    mean, std = load_normalization(args.norm if os.path.exists(args.norm) else None)
    model.restore(params, mean, std, device=int(args.gpu_num))
    return model


def compress(model, args):
    print(args)
    config = load_config(args.model_num)
    print(config)
    P, Q = config["patch_size"], config["quan_scale"]
    codec = model.codec(P, Q)
    from tf_image_compression_amd.image_codec import ImageCodec
    ic = ImageCodec(codec)
    cum_freq = None if args.raw else symbol_table(args, config)
    out_dir = args.output_dir.format(args.model_num)
    os.makedirs(out_dir, exist_ok=True)
    t0 = time.time()
    for image_path in utils.read_image_list(args.data_list):
        image = utils.imread(image_path)
        symbols = ic.encode_image(image)                     # [n, eh, ew, ec] uint8
        shape = symbols.shape[1:]
        seq = symbols.reshape(-1)                            # encode.py:175-182 order
        encodepath = get_encodepath(image_path, image, seq.size, args, config, shape)
        if args.raw:
            np.packbits(seq.astype(np.uint8) & 1).tofile(encodepath) if Q == 2 else seq.tofile(encodepath)
        else:
            apply_range_encoder(seq, encodepath, args, config, cum_freq)
        print(f"encodepath: {encodepath}")
    if args.debug_mode == "on":
        print(f"encode time {time.time() - t0:.3f}s")


if __name__ == "__main__":
    args = my_parse_args()
    cfg = load_config(args.model_num)
    compress(load_model(args, cfg), args)
