"""model_N/config.json handling (model_0/config.json:3-12).

The reference reads ``model_{N}/config.json`` relative to the working directory
(encode.py:129-131, decode.py:147-149).  ``load_config`` does the same and falls back to
the packaged copy of each model's config (same keys and values) when the file is absent.
"""
import json
import os

_HERE = os.path.dirname(os.path.abspath(__file__))


def load_config(model_num, path=None):
    candidates = [path] if path else []
    candidates += [os.path.join(f"model_{model_num}", "config.json"),
                   os.path.join(_HERE, "configs", f"model_{model_num}.json")]
    for c in candidates:
        if c and os.path.exists(c):
            with open(c) as f:
                return json.load(f)
    raise FileNotFoundError(f"no config.json for model_{model_num}")
