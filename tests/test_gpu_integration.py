"""INTEGRATION.md's reference-side binding, executed verbatim.

The ```python block of INTEGRATION.md is the model_0/model.py a maintainer would drop into
the reference: it is run here exactly as written — only the library path substituted —
from a directory holding synthetic ``data_info/channel_normalization_params.npz`` and
``model_0/params_for_test/params.npz`` (the reference's own paths), then driven the way
encode.py:142-182 and decode.py:159-249 drive the TF graph functions: float32 pixels in,
float32 symbols out, float32 reconstruction out.  Checked bit for bit against the
package's Codec (same kernels, same tuning) and against the oracle's bars."""
import os
import re

import numpy as np
import pytest

from conftest import ROOT, structured_patches
from oracle import tic_oracle as o

pytestmark = pytest.mark.gpu


def _snippet():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    blocks = re.findall(r"```python\n(.*?)```", text, re.S)
    assert len(blocks) == 1, "INTEGRATION.md must hold exactly one python block (the binding)"
    code = blocks[0]
    placeholder = '"/path/to/tf_image_compression_amd/libtic.so"'
    assert placeholder in code
    return code.replace(placeholder, repr(os.path.join(ROOT, "tf_image_compression_amd", "libtic.so")))


def test_integration_binding_verbatim(tmp_path, monkeypatch):
    from tf_image_compression_amd.codec import Codec
    from tf_image_compression_amd.weights import synthetic_params, SYNTH_MEAN, SYNTH_STD
    params = synthetic_params(0, seed=3)
    os.makedirs(tmp_path / "data_info")
    os.makedirs(tmp_path / "model_0" / "params_for_test")
    np.savez(tmp_path / "data_info" / "channel_normalization_params.npz", mean=SYNTH_MEAN, std=SYNTH_STD)
    np.savez(tmp_path / "model_0" / "params_for_test" / "params.npz", **params)
    monkeypatch.chdir(tmp_path)
    ns = {}
    exec(compile(_snippet(), "INTEGRATION.md", "exec"), ns)
    try:
        P = 256
        x = structured_patches(4, P, seed=1301)
        sym = ns["encoder"](x.astype(np.float32), P, 2)            # encode.py:157-165
        assert sym.dtype == np.float32 and sym.shape == (4, 16, 16, 64)
        assert set(np.unique(sym)) <= {0.0, 1.0}
        rec = ns["decoder"](sym.astype(int), 2)                      # decode.py:212-220 (ints from the file)
        assert rec.dtype == np.float32 and rec.shape == (4, P, P, 3)
        with pytest.raises(ValueError):
            ns["encoder"](x.astype(np.float32) + 0.5, P, 2)
        with Codec(0, params, SYNTH_MEAN, SYNTH_STD, patch_size=P) as c:
            idx = c.encode(x)
            _, f = c.decode(idx, return_float=True)
        assert np.array_equal(sym.astype(np.uint8), idx)
        assert np.array_equal(rec, f)
        pre, ref_idx = o.encoder(params, SYNTH_MEAN, SYNTH_STD, x, P, 2, 0)
        safe = o.decision_margin(pre, 2) > 1e-5 * max(1.0, float(np.abs(pre).max()))
        assert int(np.count_nonzero((idx != ref_idx) & safe)) == 0
        ref_f, _ = o.decoder(params, SYNTH_MEAN, SYNTH_STD, idx, 2, 0)
        assert float(np.abs(rec - ref_f).max()) <= 1e-2
    finally:
        ns["_L"].tic_destroy.argtypes = [type(ns["_h"])]
        ns["_L"].tic_destroy(ns["_h"])
