"""The shipped tuning states (tf_image_compression_amd/tune/*.json) are the product default
that every Codec applies and that bench.py replays (DESIGN.md §3 "Tuning state").  Each must
have been measured on exactly these kernel sources: its stamp equals the current source digest
(VERDICT r04 item 4 — two states were once carried over to a new stamp by hand), and its
tuning text parses with the runtime's own flag set.  Regenerate them with tools/gpu_tune.sh on
the final sources; never re-stamp an old measurement."""
import glob
import json
import os

import pytest

from conftest import ROOT

TUNE = sorted(glob.glob(os.path.join(ROOT, "tf_image_compression_amd", "tune", "*.json")))


def test_there_are_shipped_tunings():
    names = {os.path.basename(p) for p in TUNE}
    assert {"model0_p256_b64_s2.json", "model3_p256_b256_s2.json"} <= names, names


@pytest.mark.parametrize("path", TUNE, ids=[os.path.basename(p) for p in TUNE])
def test_tuning_stamp_matches_sources(path):
    from tf_image_compression_amd._lib import source_digest
    doc = json.load(open(path))
    meta = doc["_meta"]
    assert meta["source_sha256"] == source_digest(), (
        f"{os.path.basename(path)} was measured on other sources: re-run tools/gpu_tune.sh")
    assert "carried_over_from" not in meta
    text = doc["tuning"]
    assert text.startswith("tic-tuning 1\n")
    flags = {ln.split()[1] for ln in text.splitlines() if ln.startswith("flag ")}
    # chain_x too: tic_tuning_export always writes it, and without it a replay would fall back to
    # the runtime default
    assert {"fuse01", "fuse_tail", "s1_form", "chain", "chain_wh", "chain_x"} <= flags, flags
