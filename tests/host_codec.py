"""A host stand-in for tf_image_compression_amd.codec.Codec with the oracle as the network:
the same device-buffer interface (alloc / upload / download / view, codec_device,
memset_device, sse_u8_device, synchronize) over numpy arrays, so the GPU orchestration
code (sharded.DeviceShard / run_device_shard) runs unchanged in CPU tests (gloo,
world size 2).  Test infrastructure only."""
import numpy as np

from oracle import tic_oracle as o


class HostBuffer:
    def __init__(self, nbytes, base=None, offset=0):
        self.base = base
        self.a = np.zeros(int(nbytes), np.uint8) if base is None else base.a[offset:]
        self.nbytes = self.a.size
        self.ptr = self

    def upload(self, arr):
        b = np.ascontiguousarray(arr).view(np.uint8).reshape(-1)
        self.a[:b.size] = b

    def download(self, shape, dtype):
        n = int(np.prod(shape)) * np.dtype(dtype).itemsize
        return self.a[:n].view(dtype).reshape(shape).copy()

    def view(self, offset):
        return HostBuffer(0, base=self, offset=int(offset))

    def free(self):
        pass


class HostCodec:
    def __init__(self, model_id, params, mean, std, patch_size, quan_scale=2):
        self.model_id, self.params, self.mean, self.std = model_id, params, mean, std
        self.patch_size, self.quan_scale = patch_size, quan_scale
        pre, _ = o.encoder(params, mean, std, np.zeros((1, patch_size, patch_size, 3), np.uint8), patch_size,
                           quan_scale, model_id)
        self.code_shape = tuple(pre.shape[1:])
        self.calls = 0

    def alloc(self, nbytes):
        return HostBuffer(nbytes)

    def codec_device(self, d_in, n, d_idx, d_rgb):
        P = self.patch_size
        x = d_in.a[:n * P * P * 3].reshape(n, P, P, 3)
        _, idx = o.encoder(self.params, self.mean, self.std, x, P, self.quan_scale, self.model_id)
        _, rgb = o.decoder(self.params, self.mean, self.std, idx, self.quan_scale, self.model_id)
        d_idx.upload(idx.astype(np.uint8))
        d_rgb.upload(rgb.astype(np.uint8))
        self.calls += 1

    def memset_device(self, d, value, nbytes):
        d.a[:nbytes] = value

    def sse_u8_device(self, d_a, d_b, n, d_acc):
        diff = d_a.a[:n].astype(np.int64) - d_b.a[:n].astype(np.int64)
        cur = d_acc.download((1,), np.uint64)[0]
        d_acc.upload(np.array([cur + np.uint64(int(np.sum(diff * diff)))], np.uint64))

    def synchronize(self):
        pass
