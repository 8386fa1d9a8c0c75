"""Image-parallel dataset run (BASELINE config 4: a synthetic image set sharded over the
GPUs of one node, RCCL all-gather of per-rank rate / distortion statistics).

Each rank takes a static contiguous slice of the image indices (dist.shard_range),
generates its images locally (seeded by global index, so the union over ranks is the
same set at any world size), encodes and decodes them in batches on its own GPU,
accumulates {SSE, dims, raw bits, images, t_start, t_end} and joins ONE all-gather; every
rank then derives the dataset PSNR the way processing_utils/evaluate.py:10-32 does
(sum of SSE / sum of dims) and the aggregate MPix/s.  No other collective exists.

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        -m tf_image_compression_amd.sharded --images 10000
"""
from __future__ import annotations

import argparse
import json
import time

import numpy as np

from . import dist
from .synthetic import structured_patches


def image_batch(lo, hi, P):
    """Images [lo, hi) of the synthetic set (each seeded by its global index)."""
    return np.concatenate([structured_patches(1, P, seed=10_000 + i) for i in range(lo, hi)])


def run_shard(codec_fn, rank, world, n_images, P, batch, code_bits_per_image):
    """codec_fn(uint8 [b,P,P,3]) -> uint8 reconstruction [b,P,P,3]."""
    lo, hi = dist.shard_range(n_images, rank, world)
    st = dist.RankStats(t_start=time.time())
    for s in range(lo, hi, batch):
        x = image_batch(s, min(hi, s + batch), P)
        y = codec_fn(x)
        st.sse += float(np.sum(np.square(y.astype(np.float64) - x.astype(np.float64))))
        st.dims += x.size
        st.bits += code_bits_per_image * x.shape[0]
        st.images += x.shape[0]
    st.t_end = time.time()
    return st


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", type=int, default=0)
    ap.add_argument("--images", type=int, default=10000)
    ap.add_argument("--patch", type=int, default=256)
    ap.add_argument("--batch", type=int, default=64)
    args = ap.parse_args(argv)
    from .codec import Codec
    from .topology import bottleneck_shape
    from .weights import synthetic_params, SYNTH_MEAN, SYNTH_STD
    rank, world, local = dist.env_rank()
    codec = Codec(args.model, synthetic_params(args.model), SYNTH_MEAN, SYNTH_STD, patch_size=args.patch,
                  device=local)
    comm = dist.make_comm(codec)
    eh, ew, ec = bottleneck_shape(args.model, args.patch)
    comm.barrier()
    st = run_shard(lambda x: codec.decode(codec.encode(x)), rank, world, args.images, args.patch, args.batch,
                   eh * ew * ec)
    summary = dist.combine(comm.allgather_stats(st))
    if rank == 0:
        print(json.dumps({"world": world, **summary}))
    comm.close()
    codec.close()


if __name__ == "__main__":
    main()
