#!/usr/bin/env python3
"""Drop-in for the reference's get_encoded_distribution.py: the symbol distribution of the
encoder over a list of training patches, saved as ``distribution_info_{N}.npy`` (the
probability table encode.py / decode.py turn into the range coder's cum_freq).

Reference: /root/reference/get_encoded_distribution.py:17-83 (flags), :86-134
(get_distribution: batches of 64 patches -> encoder -> np.histogram(out, range(Q+1))
summed -> prob = freq / sum(freq) -> np.save).  Here each batch is uploaded once,
encoded on the GPU and histogrammed on the GPU (tic_histogram_device accumulates into one
device counter array); the counts come back once at the end.  ``-f/--model_file`` is
accepted for flag compatibility (the model is chosen by ``-m``).  Extra optional flags as
encode.py: ``--norm``, ``--synthetic-weights``.
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from tf_image_compression_amd import utils  # noqa: E402
from tf_image_compression_amd.config import load_config  # noqa: E402

BATCH = 64  # get_encoded_distribution.py:98


def my_parse_args(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("-m", "--model_num", type=str, choices=["0", "1", "2", "3"], required=True,
                   help="Determine which model to use")
    p.add_argument("-g", "--gpu_num", type=str, choices=[str(i) for i in range(8)], required=True,
                   help="Determine which gpu to use")
    p.add_argument("-d", "--debug_mode", type=str, choices=["on", "off"], default="off")
    p.add_argument("-p", "--params_file", type=str, default="", help="File for model parameters")
    p.add_argument("-v", "--data_list", type=str, default="data_info/train_data_patch_list_{}.txt",
                   help="File for data_list ({} = patch size)")
    p.add_argument("-f", "--model_file", type=str, default="model_{}/params_for_test/model.py",
                   help="accepted for compatibility; the model is selected by -m")
    p.add_argument("-o", "--output_file", type=str, default="data_info/distribution_info_{}.npy",
                   help="File to keep encoded distribution info")
    p.add_argument("--norm", type=str, default="data_info/channel_normalization_params.npz")
    p.add_argument("--synthetic-weights", action="store_true")
    return p.parse_args(argv)


def load_model(args):
    import importlib
    from tf_image_compression_amd.weights import load_normalization, synthetic_params
    model = importlib.import_module(f"tf_image_compression_amd.model_{args.model_num}.model")
    params = synthetic_params(int(args.model_num)) if args.synthetic_weights else utils.restore_params(args)
    mean, std = load_normalization(args.norm if os.path.exists(args.norm) else None)
    model.restore(params, mean, std, device=int(args.gpu_num))
    return model


def encoded_frequencies(codec, patch_iter, Q):
    """Sum over batches of np.histogram(encoder(batch), range(Q+1))[0], on the GPU."""
    P = codec.patch_size
    eh, ew, ec = codec.code_shape
    d_in = codec.alloc(BATCH * P * P * 3)
    d_sym = codec.alloc(BATCH * eh * ew * ec)
    d_cnt = codec.alloc(8 * Q)
    codec.memset_device(d_cnt, 0, 8 * Q)
    for batch in patch_iter:
        x = np.ascontiguousarray(batch, np.uint8).reshape(-1, P, P, 3)
        d_in.upload(x)
        codec.encode_device(d_in, x.shape[0], d_sym)
        codec.histogram_device(d_sym, x.shape[0] * eh * ew * ec, Q, d_cnt)
    freq = d_cnt.download((Q,), np.uint64).astype(np.float64)
    for b in (d_in, d_sym, d_cnt):
        b.free()
    return freq


def patch_batches(paths, P):
    for s in range(0, len(paths), BATCH):
        batch = [utils.imread(p) for p in paths[s:s + BATCH]]
        for p, b in zip(paths[s:s + BATCH], batch):
            if b.shape != (P, P, 3):
                raise ValueError(f"{p}: expected a {P}x{P} RGB patch, got {b.shape}")
        yield np.stack(batch)


def get_distribution(model, args):
    print(args)
    config = load_config(args.model_num)
    print(config)
    P, Q = config["patch_size"], config["quan_scale"]
    codec = model.codec(P, Q)
    paths = utils.read_image_list(args.data_list.format(P))
    freq = encoded_frequencies(codec, patch_batches(paths, P), Q)
    prob = freq / sum(freq)  # get_encoded_distribution.py:129
    print(prob)
    out = args.output_file.format(args.model_num)
    os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
    np.save(out, prob)
    return prob


if __name__ == "__main__":
    a = my_parse_args()
    get_distribution(load_model(a), a)
