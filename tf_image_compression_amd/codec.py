"""Host-side codec object over libtic.so.

``Codec`` is one libtic handle: a model's weights resident on one MI355X plus the
stream its kernels run on.  It is the object behind the reference-shaped modules
``tf_image_compression_amd.model_N.model`` (``encoder`` / ``decoder``, mirroring
model_N/model.py:34 and :147) and behind ``encode.py`` / ``decode.py``.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import check, ptr, lib
from .topology import CH128_ID, RMBE_ID, param_shapes

F32 = np.float32


class DeviceBuffer:
    """Device allocation owned by a Codec handle (freed with the handle)."""

    def __init__(self, codec: "Codec", nbytes: int):
        self.codec = codec
        self.nbytes = int(nbytes)
        p = C.c_void_p()
        check(lib().tic_device_alloc(codec._h, self.nbytes, C.byref(p)), "tic_device_alloc")
        self.ptr = p

    def upload(self, arr: np.ndarray) -> None:
        arr = np.ascontiguousarray(arr)
        if arr.nbytes > self.nbytes:
            raise ValueError("array larger than device buffer")
        check(lib().tic_memcpy_h2d(self.codec._h, self.ptr, arr.ctypes.data, arr.nbytes), "tic_memcpy_h2d")

    def download(self, shape, dtype) -> np.ndarray:
        out = np.empty(shape, dtype)
        if out.nbytes > self.nbytes:
            raise ValueError("requested more bytes than the device buffer holds")
        check(lib().tic_memcpy_d2h(self.codec._h, out.ctypes.data, self.ptr, out.nbytes), "tic_memcpy_d2h")
        return out

    def view(self, offset: int) -> "DeviceView":
        """The same allocation from byte ``offset`` on (a pointer into it, as a C caller
        would pass one; not owned)."""
        if not 0 <= offset <= self.nbytes:
            raise ValueError(f"offset {offset} outside the {self.nbytes}-byte buffer")
        return DeviceView(self, int(offset))

    def free(self) -> None:
        if self.ptr is not None and self.codec._h is not None:
            check(lib().tic_device_free(self.codec._h, self.ptr), "tic_device_free")
        self.ptr = None


class DeviceView:
    """A byte offset into a DeviceBuffer, accepted wherever a DeviceBuffer is (``.ptr``)."""

    def __init__(self, buf: DeviceBuffer, offset: int):
        self.codec = buf.codec
        self.base = buf
        self.offset = offset
        self.nbytes = buf.nbytes - offset
        self.ptr = C.c_void_p(buf.ptr.value + offset)


class Codec:
    """A model_N codec on one GPU.  ``params``: TF-named float32 arrays (weights.py)."""

    def __init__(self, model_id: int, params: dict, mean, std, patch_size: int | None = None,
                 quan_scale: int = 2, device: int = 0, tuning: str = "auto"):
        """``tuning``: "auto" applies the shipped tuning database (tuning.py: the fusions,
        tilings and variants bench.py measured best for this model / patch / lanes);
        "none" keeps the runtime's built-in per-model defaults."""
        self.model_id = int(model_id)
        if patch_size is None:
            patch_size = 128 if model_id in (2, 3, CH128_ID, RMBE_ID) else 256
        self.patch_size = int(patch_size)
        self.quan_scale = int(quan_scale)
        self.device = int(device)
        h = C.c_void_p()
        check(lib().tic_create(self.model_id, self.patch_size, self.quan_scale, self.device, C.byref(h)),
              "tic_create")
        self._h = h
        try:
            mean = np.ascontiguousarray(mean, F32).reshape(3)
            std = np.ascontiguousarray(std, F32).reshape(3)
            check(lib().tic_set_normalization(h, ptr(mean, C.c_float), ptr(std, C.c_float)),
                  "tic_set_normalization")
            for name in param_shapes(self.model_id):
                if name not in params:
                    raise ValueError(f"missing variable {name!r}")
            for name, arr in params.items():
                a = np.ascontiguousarray(arr, F32)
                shape = (C.c_int64 * a.ndim)(*a.shape)
                check(lib().tic_set_param(h, name.encode(), ptr(a, C.c_float), shape, a.ndim),
                      f"tic_set_param({name})")
            check(lib().tic_finalize(h), "tic_finalize")
            self.tuning_source = "runtime defaults"
            self._auto_tuning = tuning == "auto"
            if tuning == "auto":
                from . import tuning as _tuning
                self.tuning_source = _tuning.apply(self)
            elif tuning != "none":
                raise ValueError(f"tuning must be 'auto' or 'none', got {tuning!r}")
        except Exception:
            self.close()
            raise

    # ------------------------------------------------------------------ info
    @property
    def code_shape(self) -> tuple[int, int, int]:
        eh, ew, ec = C.c_int(), C.c_int(), C.c_int()
        check(lib().tic_code_shape(self._h, C.byref(eh), C.byref(ew), C.byref(ec)), "tic_code_shape")
        return eh.value, ew.value, ec.value

    def device_info(self) -> str:
        buf = C.create_string_buffer(256)
        check(lib().tic_device_info(self._h, buf, 256), "tic_device_info")
        return buf.value.decode()

    def layers(self):
        out = []
        n = check(lib().tic_num_layers(self._h), "tic_num_layers")
        for i in range(n):
            name = C.create_string_buffer(128)
            v = [C.c_int() for _ in range(6)]
            check(lib().tic_layer_info(self._h, i, name, 128, *[C.byref(x) for x in v]), "tic_layer_info")
            out.append((name.value.decode(), *[x.value for x in v]))
        return out

    # ------------------------------------------------------------------ host entry points
    def encode(self, patches: np.ndarray, return_preact: bool = False):
        """uint8 [N,P,P,3] -> uint8 symbols [N,h,w,C] (model_N.encoder + sess.run)."""
        x = np.ascontiguousarray(patches)
        if x.dtype != np.uint8:
            raise ValueError(f"patches must be uint8, got {x.dtype}")
        P = self.patch_size
        x = x.reshape(-1, P, P, 3)  # model_0/model.py:39 reshape [-1,P,P,3]
        n = x.shape[0]
        eh, ew, ec = self.code_shape
        idx = np.empty((n, eh, ew, ec), np.uint8)
        pre = np.empty((n, eh, ew, ec), F32) if return_preact else None
        check(lib().tic_encode(self._h, ptr(x, C.c_uint8), n, ptr(idx, C.c_uint8), ptr(pre, C.c_float)),
              "tic_encode")
        return (idx, pre) if return_preact else idx

    def decode(self, symbols: np.ndarray, return_float: bool = False):
        """uint8/int symbols [N,h,w,C] -> uint8 RGB [N,P,P,3] (np.around of the clipped float)."""
        eh, ew, ec = self.code_shape
        s = np.asarray(symbols)
        if s.dtype != np.uint8:
            if np.any(s < 0) or np.any(s >= self.quan_scale):
                raise ValueError("symbols out of range [0, quan_scale)")
            s = s.astype(np.uint8)
        elif s.size and int(s.max()) >= self.quan_scale:
            raise ValueError("symbols out of range [0, quan_scale)")
        s = np.ascontiguousarray(s).reshape(-1, eh, ew, ec)
        n = s.shape[0]
        P = self.patch_size
        rgb = np.empty((n, P, P, 3), np.uint8)
        f = np.empty((n, P, P, 3), F32) if return_float else None
        check(lib().tic_decode(self._h, ptr(s, C.c_uint8), n, ptr(rgb, C.c_uint8), ptr(f, C.c_float)),
              "tic_decode")
        return (rgb, f) if return_float else rgb

    def rmbe_windows(self, windows: np.ndarray) -> np.ndarray:
        """float32 [N,128,128,3] -> float32 (submit/2/rmbe/model.py:113-197)."""
        if self.model_id != RMBE_ID:
            raise ValueError("not an rmbe codec")
        x = np.ascontiguousarray(windows, F32).reshape(-1, self.patch_size, self.patch_size, 3)
        out = np.empty_like(x)
        check(lib().tic_rmbe(self._h, ptr(x, C.c_float), x.shape[0], ptr(out, C.c_float)), "tic_rmbe")
        return out

    # ------------------------------------------------------------------ device entry points
    def alloc(self, nbytes: int) -> DeviceBuffer:
        return DeviceBuffer(self, nbytes)

    def encode_device(self, d_in: DeviceBuffer, n: int, d_idx: DeviceBuffer, d_pre: DeviceBuffer | None = None):
        check(lib().tic_encode_device(self._h, d_in.ptr, n, d_idx.ptr, d_pre.ptr if d_pre else None),
              "tic_encode_device")

    def decode_device(self, d_idx: DeviceBuffer, n: int, d_rgb: DeviceBuffer | None, d_f32: DeviceBuffer | None = None):
        check(lib().tic_decode_device(self._h, d_idx.ptr, n, d_rgb.ptr if d_rgb else None,
                                      d_f32.ptr if d_f32 else None), "tic_decode_device")

    def codec_device(self, d_in: DeviceBuffer, n: int, d_idx: DeviceBuffer, d_rgb: DeviceBuffer):
        check(lib().tic_codec_device(self._h, d_in.ptr, n, d_idx.ptr, d_rgb.ptr), "tic_codec_device")

    def rmbe_device(self, d_in: DeviceBuffer, n: int, d_out: DeviceBuffer):
        check(lib().tic_rmbe_device(self._h, d_in.ptr, n, d_out.ptr), "tic_rmbe_device")

    def set_option(self, key: str, value: int) -> None:
        check(lib().tic_set_option(self._h, key.encode(), int(value)), f"tic_set_option({key})")
        if key == "streams" and getattr(self, "_auto_tuning", False):
            # the shipped entries are keyed by per-launch batch, which the lane count changes
            from . import tuning as _tuning
            self.tuning_source = _tuning.reapply_entries(self, int(value))

    def stream_ptr(self) -> C.c_void_p:
        s = C.c_void_p()
        check(lib().tic_get_stream(self._h, C.byref(s)), "tic_get_stream")
        return s

    def stream_external(self, on: bool) -> None:
        """Whether work of the caller's own may be pending on stream_ptr() (tic_stream_external)."""
        check(lib().tic_stream_external(self._h, int(bool(on))), "tic_stream_external")

    def synchronize(self) -> None:
        check(lib().tic_synchronize(self._h), "tic_synchronize")

    def profile_layers(self, d_in: DeviceBuffer, n: int, iters: int) -> np.ndarray:
        nl = check(lib().tic_num_layers(self._h), "tic_num_layers")
        ms = np.zeros(nl, F32)
        check(lib().tic_profile_layers(self._h, d_in.ptr, n, iters, ptr(ms, C.c_float)), "tic_profile_layers")
        return ms

    def mark_durations(self, cap: int = 8192) -> np.ndarray:
        """ms of every launch recorded under option "mark_layer" since the last call (all
        lanes, in-step: tic_mark_durations)."""
        ms = np.zeros(cap, F32)
        k = check(lib().tic_mark_durations(self._h, ptr(ms, C.c_float), cap), "tic_mark_durations")
        return ms[:k]

    def autotune(self, d_in: DeviceBuffer, n: int, reps: int = 5) -> None:
        check(lib().tic_autotune(self._h, d_in.ptr, n, reps), "tic_autotune")

    def autotune_step(self, d_in: DeviceBuffer, n: int, rounds: int = 1, reps: int = 5) -> None:
        """Per-layer variants chosen by the whole dual-lane step time (tic_autotune_step)."""
        check(lib().tic_autotune_step(self._h, d_in.ptr, n, rounds, reps), "tic_autotune_step")

    def layer_variants(self, n: int):
        out = []
        for i in range(len(self.layers())):
            th, ns = C.c_int(), C.c_int()
            check(lib().tic_layer_variant(self._h, i, n, C.byref(th), C.byref(ns)), "tic_layer_variant")
            out.append((th.value, ns.value))
        return out

    def layer_kernels(self, n: int):
        """Kernel instance each layer launches for batch n ('' if fused into the previous)."""
        out = []
        for i in range(len(self.layers())):
            buf = C.create_string_buffer(160)
            check(lib().tic_layer_kernel(self._h, i, n, buf, 160), "tic_layer_kernel")
            out.append(buf.value.decode())
        return out

    def tuning_export(self) -> str:
        """Tuned tilings / variants / fusion flags as text (tic_tuning_export)."""
        n = check(lib().tic_tuning_export(self._h, None, 0), "tic_tuning_export")
        buf = C.create_string_buffer(n + 1)
        check(lib().tic_tuning_export(self._h, buf, n + 1), "tic_tuning_export")
        return buf.value.decode()

    def tuning_import(self, text: str) -> None:
        check(lib().tic_tuning_import(self._h, text.encode()), "tic_tuning_import")

    def conv3x3_device(self, kind: int, act: int, d_in: DeviceBuffer, n: int, H: int, W: int, cin: int,
                       cout: int, kernel: np.ndarray, bias: np.ndarray, d_res: DeviceBuffer | None,
                       d_out: DeviceBuffer) -> None:
        k = np.ascontiguousarray(kernel, F32)
        b = np.ascontiguousarray(bias, F32)
        check(lib().tic_conv3x3_device(self._h, kind, act, d_in.ptr, n, H, W, cin, cout, ptr(k, C.c_float),
                                       ptr(b, C.c_float), d_res.ptr if d_res else None, d_out.ptr),
              "tic_conv3x3_device")

    # ------------------------------------------------------------------ whole images (image_ops.hip)
    def image_to_patches_device(self, d_img: DeviceBuffer, H: int, W: int, P: int, d_patches: DeviceBuffer):
        check(lib().tic_image_to_patches_device(self._h, d_img.ptr, H, W, P, d_patches.ptr),
              "tic_image_to_patches_device")

    def patches_to_image_device(self, d_patches: DeviceBuffer, H: int, W: int, P: int, d_img: DeviceBuffer):
        check(lib().tic_patches_to_image_device(self._h, d_patches.ptr, H, W, P, d_img.ptr),
              "tic_patches_to_image_device")

    def rmbe_image_device(self, d_img: DeviceBuffer, H: int, W: int):
        check(lib().tic_rmbe_image_device(self._h, d_img.ptr, H, W), "tic_rmbe_image_device")

    def round_u8_device(self, d_in: DeviceBuffer, n: int, d_out: DeviceBuffer):
        check(lib().tic_round_u8_device(self._h, d_in.ptr, n, d_out.ptr), "tic_round_u8_device")

    def histogram_device(self, d_sym: DeviceBuffer, n: int, Q: int, d_counts: DeviceBuffer):
        check(lib().tic_histogram_device(self._h, d_sym.ptr, n, Q, d_counts.ptr), "tic_histogram_device")

    def sse_u8_device(self, d_a: DeviceBuffer, d_b: DeviceBuffer, n: int, d_acc: DeviceBuffer):
        check(lib().tic_sse_u8_device(self._h, d_a.ptr, d_b.ptr, n, d_acc.ptr), "tic_sse_u8_device")

    def memset_device(self, d: DeviceBuffer, value: int, nbytes: int):
        check(lib().tic_memset_device(self._h, d.ptr, value, nbytes), "tic_memset_device")

    def wait_for(self, other: "Codec") -> None:
        """Order this handle's stream after everything enqueued so far on ``other``'s."""
        check(lib().tic_stream_wait(self._h, other._h), "tic_stream_wait")

    def record(self, slot: int) -> None:
        """Mark the work enqueued so far on this handle's stream as event ``slot`` (0..7)."""
        check(lib().tic_event_record(self._h, slot), "tic_event_record")

    def wait_event(self, other: "Codec", slot: int) -> None:
        """Order this handle's stream after ``other``'s last mark of ``slot`` (if any)."""
        check(lib().tic_stream_wait_event(self._h, other._h, slot), "tic_stream_wait_event")

    # ------------------------------------------------------------------ lifetime
    def close(self) -> None:
        if getattr(self, "_h", None) is not None:
            lib().tic_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def version() -> str:
    return lib().tic_version().decode()


__all__ = ["Codec", "DeviceBuffer", "DeviceView", "version", "_lib"]
