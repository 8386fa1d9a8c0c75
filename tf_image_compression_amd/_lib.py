"""ctypes binding to libtic.so (the C-ABI declared in include/tic.h).

There is deliberately no fallback: if the HIP library is missing or fails to load,
``lib()`` raises, and every product entry point fails loudly.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TIC_LIB", os.path.join(_HERE, "libtic.so"))

TIC_OK = 0
ERRORS = {-1: "EINVAL", -2: "ENOTFOUND", -3: "ESTATE", -4: "EHIP", -5: "ENOMEM", -6: "EUNSUPPORTED",
          -7: "EOVERFLOW", -8: "EIO"}
TIC_MODEL_RMBE = 100

u8p = C.POINTER(C.c_uint8)
f32p = C.POINTER(C.c_float)
i32p = C.POINTER(C.c_int)
vp = C.c_void_p

# (name, restype, argtypes) — mirrors include/tic.h one to one
SIGNATURES = [
    ("tic_version", C.c_char_p, []),
    ("tic_last_error", C.c_char_p, []),
    ("tic_create", C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(vp)]),
    ("tic_destroy", None, [vp]),
    ("tic_set_normalization", C.c_int, [vp, f32p, f32p]),
    ("tic_set_param", C.c_int, [vp, C.c_char_p, f32p, C.POINTER(C.c_int64), C.c_int]),
    ("tic_finalize", C.c_int, [vp]),
    ("tic_code_shape", C.c_int, [vp, i32p, i32p, i32p]),
    ("tic_encode", C.c_int, [vp, u8p, C.c_int, u8p, f32p]),
    ("tic_decode", C.c_int, [vp, u8p, C.c_int, u8p, f32p]),
    ("tic_rmbe", C.c_int, [vp, f32p, C.c_int, f32p]),
    ("tic_device_alloc", C.c_int, [vp, C.c_size_t, C.POINTER(vp)]),
    ("tic_device_free", C.c_int, [vp, vp]),
    ("tic_memcpy_h2d", C.c_int, [vp, vp, vp, C.c_size_t]),
    ("tic_memcpy_d2h", C.c_int, [vp, vp, vp, C.c_size_t]),
    ("tic_synchronize", C.c_int, [vp]),
    ("tic_encode_device", C.c_int, [vp, vp, C.c_int, vp, vp]),
    ("tic_decode_device", C.c_int, [vp, vp, C.c_int, vp, vp]),
    ("tic_codec_device", C.c_int, [vp, vp, C.c_int, vp, vp]),
    ("tic_rmbe_device", C.c_int, [vp, vp, C.c_int, vp]),
    ("tic_set_option", C.c_int, [vp, C.c_char_p, C.c_int]),
    ("tic_num_layers", C.c_int, [vp]),
    ("tic_layer_info", C.c_int, [vp, C.c_int, C.c_char_p, C.c_int, i32p, i32p, i32p, i32p, i32p, i32p]),
    ("tic_model_num_layers", C.c_int, [C.c_int]),
    ("tic_model_layer", C.c_int, [C.c_int, C.c_int, C.c_char_p, C.c_int, i32p, i32p, i32p, i32p, i32p, i32p]),
    ("tic_profile_layers", C.c_int, [vp, vp, C.c_int, C.c_int, f32p]),
    ("tic_mark_durations", C.c_int, [vp, f32p, C.c_int]),
    ("tic_autotune", C.c_int, [vp, vp, C.c_int, C.c_int]),
    ("tic_layer_variant", C.c_int, [vp, C.c_int, C.c_int, i32p, i32p]),
    ("tic_autotune_step", C.c_int, [vp, vp, C.c_int, C.c_int, C.c_int]),
    ("tic_layer_kernel", C.c_int, [vp, C.c_int, C.c_int, C.c_char_p, C.c_int]),
    ("tic_tuning_export", C.c_int, [vp, C.c_char_p, C.c_int]),
    ("tic_tuning_import", C.c_int, [vp, C.c_char_p]),
    ("tic_conv3x3_device", C.c_int, [vp, C.c_int, C.c_int, vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                     f32p, f32p, vp, vp]),
    ("tic_get_stream", C.c_int, [vp, C.POINTER(vp)]),
    ("tic_stream_external", C.c_int, [vp, C.c_int]),
    ("tic_image_to_patches_device", C.c_int, [vp, vp, C.c_int, C.c_int, C.c_int, vp]),
    ("tic_patches_to_image_device", C.c_int, [vp, vp, C.c_int, C.c_int, C.c_int, vp]),
    ("tic_rmbe_image_device", C.c_int, [vp, vp, C.c_int, C.c_int]),
    ("tic_round_u8_device", C.c_int, [vp, vp, C.c_size_t, vp]),
    ("tic_histogram_device", C.c_int, [vp, vp, C.c_size_t, C.c_int, vp]),
    ("tic_sse_u8_device", C.c_int, [vp, vp, vp, C.c_size_t, vp]),
    ("tic_memset_device", C.c_int, [vp, vp, C.c_int, C.c_size_t]),
    ("tic_stream_wait", C.c_int, [vp, vp]),
    ("tic_event_record", C.c_int, [vp, C.c_int]),
    ("tic_stream_wait_event", C.c_int, [vp, vp, C.c_int]),
    ("tic_crc32c", C.c_uint32, [C.c_char_p, C.c_size_t, C.c_uint32]),
    # entropy coder (host only)
    ("tic_rc_last_error", C.c_char_p, []),
    ("tic_rc_encoder_open", C.c_int, [C.c_char_p, C.POINTER(vp)]),
    ("tic_rc_encode", C.c_int, [vp, C.POINTER(C.c_int64), C.c_size_t, C.POINTER(C.c_int64), C.c_size_t]),
    ("tic_rc_encoder_close", C.c_int, [vp]),
    ("tic_rc_encoder_free", None, [vp]),
    ("tic_rc_decoder_open", C.c_int, [C.c_char_p, C.POINTER(vp)]),
    ("tic_rc_decode", C.c_int, [vp, C.c_size_t, C.POINTER(C.c_int64), C.c_size_t, C.POINTER(C.c_int64)]),
    ("tic_rc_decoder_close", C.c_int, [vp]),
    ("tic_rc_decoder_free", None, [vp]),
    ("tic_device_info", C.c_int, [vp, C.c_char_p, C.c_int]),
]

_lock = threading.Lock()
_lib = None


class TicError(RuntimeError):
    """A libtic call failed (the message is libtic's tic_last_error())."""


def lib() -> C.CDLL:
    """Load libtic.so once; raise (no fallback) if it is missing."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise TicError(f"libtic.so not found at {LIB_PATH}: build it with `make` "
                               "(or __graft_entry__.build()); there is no CPU fallback")
            L = C.CDLL(LIB_PATH)
            for name, res, args in SIGNATURES:
                fn = getattr(L, name)
                fn.restype = res
                fn.argtypes = args
            _lib = L
    return _lib


def check(rc: int, what: str = "") -> int:
    if rc < 0:
        msg = lib().tic_last_error().decode(errors="replace")
        code = ERRORS.get(rc, str(rc))
        if rc == -1:
            raise ValueError(f"{what}: [{code}] {msg}")
        if rc == -2:
            raise KeyError(f"{what}: [{code}] {msg}")
        raise TicError(f"{what}: [{code}] {msg}")
    return rc


def source_digest() -> str:
    """SHA-256 over the device-kernel sources (csrc/*.hip, csrc/*.h: kernels, launch
    registries, argument blocks), the host runtime (csrc/tic_runtime.cpp: the tuning text's
    key and variant conventions, which candidates each form offers, the lane scheduling —
    ADVICE r03) and the HIP build flags: the stamp that ties a tuning state (tuning.py) or a
    PMC summary (tools/pmc_summary.py) to the code it measured.  The range coder and the
    checkpoint reader are not part of it."""
    import hashlib
    h = hashlib.sha256()
    csrc = os.path.join(_HERE, "csrc")
    for name in sorted(os.listdir(csrc)):
        if name.endswith((".h", ".hip")) or name == "tic_runtime.cpp":
            h.update(name.encode())
            with open(os.path.join(csrc, name), "rb") as f:
                h.update(f.read())
    mk = os.path.join(os.path.dirname(_HERE), "Makefile")
    if os.path.exists(mk):
        with open(mk, "rb") as f:
            h.update(b"".join(ln for ln in f.read().splitlines(True) if ln.startswith(b"HIPFLAGS")))
    return h.hexdigest()


def lib_digest() -> str | None:
    import hashlib
    if not os.path.exists(LIB_PATH):
        return None
    with open(LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def ptr(arr, ctype):
    """Pointer to a C-contiguous numpy array's data (or NULL for None)."""
    if arr is None:
        return None
    if not arr.flags["C_CONTIGUOUS"]:
        raise ValueError("array must be C-contiguous")
    return arr.ctypes.data_as(C.POINTER(ctype))
