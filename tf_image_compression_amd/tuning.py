"""Shipped tuning database: the measured-best launch configuration as the product default.

Each file ``tune/model{M}_p{P}_b{B}_s{S}.json`` holds the text of ``tic_tuning_export`` —
the structural fusion flags (enc01 / dec10 / chain, chain workgroup shape, stride-1 form)
and every layer's tiling and fused-kernel variant, keyed by per-launch batch — measured by
``tic_autotune`` + ``tic_autotune_step`` for model M, patch P, batch B split over S lanes,
stamped with ``_lib.source_digest()`` of the kernel sources it was measured on.

``Codec`` applies the matching entries when it is created (``apply``), so the reference's
own loops (encode.py:157-165, decode.py:212-220 through ``model_N.model``, the sharded
driver, ImageCodec) run exactly the kernels ``bench.py`` times.  Rules:

* entries for (model, P, lanes) of every batch are merged (their keys are per-launch batch
  sizes, so they do not collide; on a collision the larger batch's entry wins); the flags
  come from the largest batch's entry;
* when the stamp does not match the kernel sources (kernels edited after the tuning), only
  the flags are applied — registry indices may have moved, the flags are bit-identical
  structural choices either way;
* with no entry, the runtime's own per-model defaults stand (tic_set_option, tic.h).

Nothing here changes results: every tiling, variant and fusion is bit-identical
(tests/test_gpu_parity.py, test_gpu_chain.py), only speed.
"""
from __future__ import annotations

import json
import os
import re

TUNE_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tune")
_NAME = re.compile(r"model(\d+)_p(\d+)_b(\d+)_s(\d+)\.json$")
_digest = None


def source_digest() -> str:
    global _digest
    if _digest is None:
        from ._lib import source_digest as sd
        _digest = sd()
    return _digest


def tune_path(model: int, P: int, batch: int, streams: int) -> str:
    return os.path.join(TUNE_DIR, f"model{model}_p{P}_b{batch}_s{streams}.json")


def stamp(model: int, P: int, batch: int, streams: int, tune_step: int = 1) -> dict:
    return {"source_sha256": source_digest(), "model": model, "patch": P, "batch": batch, "streams": streams,
            "tune_step": tune_step}


def entries(model: int, P: int, streams: int):
    """[(batch, path, doc)] for (model, P, streams), largest batch first."""
    out = []
    if not os.path.isdir(TUNE_DIR):
        return out
    for name in os.listdir(TUNE_DIR):
        m = _NAME.match(name)
        if not m or (int(m[1]), int(m[2]), int(m[4])) != (model, P, streams):
            continue
        path = os.path.join(TUNE_DIR, name)
        with open(path) as f:
            doc = json.load(f)
        out.append((int(m[3]), path, doc))
    return sorted(out, key=lambda e: -e[0])


def merged_text(docs, with_entries: bool) -> str:
    """One tic-tuning text from several exported states (flags from the first)."""
    lines = ["tic-tuning 1"]
    seen = set()
    for k, doc in enumerate(docs):
        for ln in doc["tuning"].splitlines()[1:]:
            parts = ln.split()
            if not parts:
                continue
            if parts[0] == "flag":
                if k == 0:
                    lines.append(ln)
                continue
            if not with_entries:
                continue
            key = (parts[0], parts[1], parts[2])  # (conv|var, layer, batch key)
            if key not in seen:
                seen.add(key)
                lines.append(ln)
    return "\n".join(lines) + "\n"


def env_streams() -> int:
    """The lane count a new handle starts with: TIC_STREAMS clamped to 1..4 exactly as the
    runtime clamps it (tic_create), default 2."""
    try:
        v = int(os.environ.get("TIC_STREAMS", "2"))
    except ValueError:
        v = 2
    return min(4, max(1, v))


def apply(codec, streams: int | None = None) -> str:
    """Apply the shipped tuning matching the codec's (model, patch, lanes); returns a short
    description of what was applied (Codec.tuning_source)."""
    if streams is None:
        streams = env_streams()
    ents = entries(codec.model_id, codec.patch_size, streams)
    if not ents:
        return "runtime defaults (no shipped tuning for this model / patch / lanes)"
    fresh = [e for e in ents if e[2].get("_meta", {}).get("source_sha256") == source_digest()]
    if fresh:
        codec.tuning_import(merged_text([e[2] for e in fresh], True))
        return "shipped tuning: " + ", ".join(os.path.basename(e[1]) for e in fresh)
    codec.tuning_import(merged_text([e[2] for e in ents], False))
    return "shipped tuning flags only (stamp mismatch): " + os.path.basename(ents[0][1])


def reapply_entries(codec, streams: int) -> str:
    """After the lane count changed (option "streams"): the per-layer entries keyed by the
    new per-launch batches, from the shipped tuning for (model, P, streams) when its stamp
    matches — or none — and the structural flags left as they are (entries
    measured for another lane count no longer match the batches the lanes see)."""
    ents = [e for e in entries(codec.model_id, codec.patch_size, streams)
            if e[2].get("_meta", {}).get("source_sha256") == source_digest()]
    text = merged_text([e[2] for e in ents], True) if ents else "tic-tuning 1\n"
    text = "\n".join(ln for ln in text.splitlines() if not ln.startswith("flag ")) + "\n"
    codec.tuning_import(text)
    return ("shipped tuning entries: " + ", ".join(os.path.basename(e[1]) for e in ents)) if ents else \
        f"runtime defaults (no shipped tuning for {streams} lanes)"
