"""CPU tests of the CLI host logic (no device): argument surface, .encoded naming and
parsing exactly as encode.py:102-122 / decode.py:104-140."""
import numpy as np

import decode
import encode
from tf_image_compression_amd.config import load_config


def test_flags_match_reference():
    a = encode.my_parse_args(["-m", "0", "-g", "3"])
    assert a.data_list == "data_info/tiny_valid_data_list.txt" and a.output_dir == "model_{}/encoded_data"
    b = decode.my_parse_args(["-m", "3", "-g", "-1"])
    assert b.input_dir == "model_{}/encoded_data" and b.output_dir == "model_{}/recons_data"
    assert a.debug_mode == "off" and a.params_file == ""


def test_encodepath_and_parsing_round_trip():
    cfg = load_config("0")
    args = encode.my_parse_args(["-m", "0", "-g", "0", "-o", "out_{}"])
    img = np.zeros((300, 200, 3), np.uint8)
    path = encode.get_encodepath("/data/clic/valid/foo bar.png", img, 16384, args, cfg, (16, 16, 64))
    assert path == "out_0/foo bar@_@16_16_64@_@16384_300_200.encoded"
    fname = path.split("/")[-1]
    assert decode.get_img_info(fname, cfg) == (16384, 300, 200)
    dargs = decode.my_parse_args(["-m", "0", "-g", "0", "-o", "rec_{}"])
    assert decode.get_recons_image_path(fname, dargs, cfg) == "rec_0/foo bar.png"


def test_encoded_shape_from_first_file(tmp_path):
    cfg = load_config("3")
    for n in ["b@_@8_8_80@_@5120_200_300.encoded", "a@_@8_8_80@_@5120_100_100.encoded"]:
        (tmp_path / n).write_bytes(b"")
    assert decode.get_encoded_shape(str(tmp_path), cfg) == (8, 8, 80)


def test_configs_match_reference_values():
    for m, p in [("0", 256), ("1", 256), ("2", 128), ("3", 128)]:
        c = load_config(m)
        assert c["patch_size"] == p and c["quan_scale"] == 2 and c["resolution"] == 4096
        assert c["name_sep"] == "@_@" and c["batch_size"] == 64
