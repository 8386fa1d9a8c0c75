"""Image-parallel dataset run (BASELINE configs[3]: a synthetic image set sharded over the
GPUs of one node, RCCL all-gather of per-rank rate / distortion statistics).

Each rank takes a static contiguous slice of the image indices (dist.shard_range) of a
synthetic set whose images are seeded by their global index (so the union over ranks is
the same set at any world size), and joins ONE all-gather of {SSE, dims, raw bits, images,
t_start, t_end}; every rank then derives the dataset PSNR the way
processing_utils/evaluate.py:10-32 does (sum of SSE / sum of dims) and the aggregate MPix/s.
No other collective exists.  The reference's loop is encode.py:152 ("To be paralleled") /
processing_utils/evaluate.py:18-32: one image after another through ``sess.run``.

Two drivers of the same orchestration:
* ``DeviceShard`` — the GPU path: the rank's images uploaded to HBM once, then a pass is
  one ``tic_codec_device`` per batch of 64 (the tuned launch sequence, the batches at
  offsets of one resident buffer) and one exact integer SSE kernel (``tic_sse_u8_device``)
  over the whole shard — no host round trip per batch, nothing but 8 bytes downloaded.
* ``run_shard`` — the same loop over host arrays with any ``codec_fn`` (the CPU gloo tests
  run it with the oracle standing in for the GPU).

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
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
    """Structured images [lo, hi) of the synthetic set (each seeded by its global index)."""
    if hi <= lo:
        return np.zeros((0, P, P, 3), np.uint8)
    return np.concatenate([structured_patches(1, P, seed=10_000 + i) for i in range(lo, hi)])


def uniform_images(lo, hi, P):
    """Uniform u8 images [lo, hi) (throughput runs: the conv cost is data-independent)."""
    out = np.empty((max(0, hi - lo), P, P, 3), np.uint8)
    for i in range(lo, hi):
        out[i - lo] = np.random.default_rng(20_000 + i).integers(0, 256, (P, P, 3), dtype=np.uint8)
    return out


def shard_images(n_images, rank, world, P, kind="structured"):
    lo, hi = dist.shard_range(n_images, rank, world)
    return (image_batch if kind == "structured" else uniform_images)(lo, hi, P)


def run_shard(codec_fn, rank, world, n_images, P, batch, code_bits_per_image):
    """Host-array driver: codec_fn(uint8 [b,P,P,3]) -> uint8 reconstruction [b,P,P,3]."""
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


class DeviceShard:
    """A rank's shard resident in HBM: uint8 images, their symbols and reconstructions,
    and one uint64 SSE accumulator."""

    def __init__(self, codec, images: np.ndarray, batch: int = 64):
        self.codec = codec
        self.n = int(images.shape[0])
        self.batch = int(batch)
        P = codec.patch_size
        eh, ew, ec = codec.code_shape
        self.pp, self.ce = P * P * 3, eh * ew * ec
        self.bits_per_symbol = max(1, (codec.quan_scale - 1).bit_length())  # raw code bits
        self.d_img = codec.alloc(max(images.nbytes, 16))
        if self.n:
            self.d_img.upload(images)
        self.d_sym = codec.alloc(max(self.n * self.ce, 16))
        self.d_rec = codec.alloc(max(images.nbytes, 16))
        self.d_acc = codec.alloc(16)

    def enqueue(self) -> None:
        """One pass over the shard, asynchronous on the codec's stream: encode -> decode of
        every batch (tic_codec_device at offsets of the resident buffers), then the exact
        SSE of reconstruction vs image (evaluate.py:10-15 summed over the shard)."""
        c = self.codec
        for s in range(0, self.n, self.batch):
            b = min(self.batch, self.n - s)
            c.codec_device(self.d_img.view(s * self.pp), b, self.d_sym.view(s * self.ce), self.d_rec.view(s * self.pp))
        c.memset_device(self.d_acc, 0, 8)
        c.sse_u8_device(self.d_img, self.d_rec, self.n * self.pp, self.d_acc)

    def sse(self) -> int:
        """SSE of the last pass (synchronises)."""
        return int(self.d_acc.download((1,), np.uint64)[0])

    def stats(self, passes: int, t_start: float, t_end: float) -> dist.RankStats:
        return dist.RankStats(sse=float(self.sse()) * passes, dims=self.n * self.pp * passes,
                              bits=self.n * self.ce * self.bits_per_symbol * passes, images=self.n * passes,
                              t_start=t_start, t_end=t_end)

    def reconstructions(self) -> np.ndarray:
        P = self.codec.patch_size
        return self.d_rec.download((self.n, P, P, 3), np.uint8)

    def free(self) -> None:
        for b in (self.d_img, self.d_sym, self.d_rec, self.d_acc):
            b.free()


def run_device_shard(codec, comm, rank, world, n_images, batch=64, kind="structured", passes=1):
    """The GPU driver end to end: build + upload the shard, barrier, `passes` timed passes,
    barrier, one all-gather; returns (combined metrics, this rank's stats)."""
    P = codec.patch_size
    shard = DeviceShard(codec, shard_images(n_images, rank, world, P, kind), batch)
    try:
        codec.synchronize()
        comm.barrier(dist.collective_timeout())  # after building this rank's shard
        t0 = time.time()
        for _ in range(passes):
            shard.enqueue()
        codec.synchronize()
        t1 = time.time()
        st = shard.stats(passes, t0, t1)
    finally:
        shard.free()
    return dist.combine(comm.allgather_stats(st, dist.collective_timeout())), st  # shards may be uneven


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", type=int, default=0)
    ap.add_argument("--images", type=int, default=10000)
    ap.add_argument("--patch", type=int, default=256)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--kind", choices=["structured", "uniform"], default="structured")
    args = ap.parse_args(argv)
    from .codec import Codec
    from .weights import synthetic_params, SYNTH_MEAN, SYNTH_STD
    rank, world, local = dist.env_rank()
    codec = Codec(args.model, synthetic_params(args.model), SYNTH_MEAN, SYNTH_STD, patch_size=args.patch,
                  device=local)
    comm = dist.make_comm(codec)
    summary, _ = run_device_shard(codec, comm, rank, world, args.images, args.batch, args.kind)
    if rank == 0:
        print(json.dumps({"world": world, **summary}))
    comm.close()
    codec.close()


if __name__ == "__main__":
    main()
