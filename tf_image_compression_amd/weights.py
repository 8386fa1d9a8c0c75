"""Weights in the reference's TF variable layout, and seeded synthetic weights.

The reference restores ``<scope>/kernel`` and ``<scope>/bias`` for every layer with
``tf.train.Saver`` (utils/utils.py:84-93).  Kernels are HWIO ``[3,3,Cin,Cout]`` for
convolutions (basic_block/basic_block.py:30) and ``[3,3,Cout,Cin]`` for
transposed convolutions (basic_block/basic_block.py:53); biases are ``[Cout]``.
The normalisation statistics come from ``data_info/channel_normalization_params.npz``
with keys ``mean`` and ``std`` of shape [3] (model_0/model.py:26-28).

No trained checkpoint ships with the reference (``params.*`` are git-ignored,
SURVEY.md §0.7), so benchmarks and tests use seeded He-normal weights with
non-zero biases in exactly that naming and layout.  Real weights are accepted as an
``.npz`` keyed by the same names.
"""
from __future__ import annotations

import numpy as np

from .topology import param_shapes, layer_table, RMBE_ID

# synthetic channel statistics (recorded in fixtures); the reference file is absent
SYNTH_MEAN = np.array([120.0, 115.0, 105.0], np.float32)
SYNTH_STD = np.array([65.0, 62.0, 66.0], np.float32)


def synthetic_params(model_id: int, seed: int = 0) -> dict[str, np.ndarray]:
    """He-normal kernels (std sqrt(2/(9 Cin))) and N(0, 0.05) biases, float32.

    Pre-activations stay O(1) so the binary quantiser's decisions are well away from
    the tie at 0 (SURVEY.md §7 hard part 1)."""
    rng = np.random.default_rng(np.random.PCG64(1000 + 97 * (model_id + 1) + seed))
    params = {}
    for name, shape in param_shapes(model_id).items():
        if name.endswith("/kernel"):
            cin = shape[3] if len(shape) == 4 and _is_transpose(model_id, name) else shape[2]
            std = np.sqrt(2.0 / (9.0 * cin))
            params[name] = (rng.standard_normal(shape) * std).astype(np.float32)
        else:
            params[name] = (rng.standard_normal(shape) * 0.05).astype(np.float32)
    return params


def _is_transpose(model_id: int, kernel_name: str) -> bool:
    scope = kernel_name[: -len("/kernel")]
    for lay in layer_table(model_id):
        if lay.name == scope:
            return lay.kind == "convT"
    raise KeyError(kernel_name)


def load_params(path: str, model_id: int | None = None) -> dict[str, np.ndarray]:
    """Load TF-named weights: a TF V2 checkpoint prefix (``<path>.index`` exists — the
    reference's ``model_N/params_for_test/params``, read by tf_checkpoint.py; with
    ``model_id`` only that model's variables) or an ``.npz`` keyed by the TF names (no pickle)."""
    from . import tf_checkpoint
    if tf_checkpoint.is_checkpoint(path):
        if model_id is not None:
            return tf_checkpoint.load_model_params(path, model_id)
        return {k: np.asarray(v, np.float32) for k, v in tf_checkpoint.read_checkpoint(path).items()
                if np.asarray(v).dtype.kind == "f"}
    if not path.endswith(".npz"):
        path = path + ".npz"
    with np.load(path, allow_pickle=False) as z:
        return {k: np.asarray(z[k], np.float32) for k in z.files}


def save_params(path: str, params: dict[str, np.ndarray]) -> None:
    np.savez(path, **{k: np.asarray(v, np.float32) for k, v in params.items()})


def load_normalization(path: str | None):
    """``channel_normalization_params.npz`` (mean, std) -> float32 3-vectors, the dtype TF
    casts them to when they meet the float32 input tensor (model_0/model.py:44)."""
    if path is None:
        return SYNTH_MEAN.copy(), SYNTH_STD.copy()
    with np.load(path, allow_pickle=False) as z:
        return np.asarray(z["mean"], np.float32).reshape(3), np.asarray(z["std"], np.float32).reshape(3)


def check_params(model_id: int, params: dict[str, np.ndarray]) -> None:
    """Raise ValueError on a missing variable or a shape mismatch (Saver.restore's contract)."""
    want = param_shapes(model_id)
    for name, shape in want.items():
        if name not in params:
            raise ValueError(f"missing variable {name!r} for model {model_id}")
        if tuple(params[name].shape) != tuple(shape):
            raise ValueError(f"variable {name!r}: shape {tuple(params[name].shape)} != {tuple(shape)}")


__all__ = ["synthetic_params", "load_params", "save_params", "load_normalization",
           "check_params", "SYNTH_MEAN", "SYNTH_STD", "RMBE_ID"]
