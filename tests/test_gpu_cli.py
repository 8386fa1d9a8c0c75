"""End-to-end drop-in test on the GPU: encode.py -> .encoded files -> decode.py -> PNGs,
checked against the CPU oracle's pipeline on the same images and weights, plus the
rmbe post-filter pipeline (config 5's driver)."""
import os

import numpy as np
import pytest

from conftest import structured_patches
from oracle import tic_oracle as o

pytestmark = pytest.mark.gpu


def _write_images(tmp_path, sizes):
    from tf_image_compression_amd import utils
    paths = []
    for k, (h, w) in enumerate(sizes):
        big = structured_patches(1, max(h, w), seed=100 + k)[0]
        img = np.ascontiguousarray(big[:h, :w])
        p = str(tmp_path / f"img{k}.png")
        utils.imsave(p, img)
        paths.append(p)
    lst = tmp_path / "list.txt"
    lst.write_text("\n".join(paths) + "\n")
    return paths, str(lst)


@pytest.mark.parametrize("model_num,raw", [("0", False), ("3", False), ("0", True)])
def test_encode_decode_cli_round_trip(tmp_path, model_num, raw):
    import encode
    import decode
    from tf_image_compression_amd import utils
    from tf_image_compression_amd.weights import synthetic_params, SYNTH_MEAN, SYNTH_STD
    paths, lst = _write_images(tmp_path, [(300, 200), (256, 300)])
    dist = tmp_path / f"dist_{model_num}.npy"
    np.save(dist, np.array([0.6, 0.4]))
    enc_dir, rec_dir = str(tmp_path / "enc"), str(tmp_path / "rec")
    common = ["-m", model_num, "-g", "0", "--synthetic-weights", "--dist", str(tmp_path / "dist_{}.npy"),
              "--norm", "/nonexistent"] + (["--raw"] if raw else [])
    eargs = encode.my_parse_args(common + ["-v", lst, "-o", enc_dir])
    cfg = encode.load_config(model_num)
    encode.compress(encode.load_model(eargs, cfg), eargs)
    files = sorted(os.listdir(enc_dir))
    assert len(files) == 2 and all(f.endswith(".encoded") for f in files)
    dargs = decode.my_parse_args(common + ["-i", enc_dir, "-o", rec_dir])
    decode.uncompress(decode.load_model(dargs, cfg), dargs)
    P = cfg["patch_size"]
    m = int(model_num)
    params = synthetic_params(m)
    for p in paths:
        img = utils.imread(p)
        rec = utils.imread(os.path.join(rec_dir, os.path.basename(p)))
        assert rec.shape == img.shape
        patches = np.stack(o.crop_image_input_patches(img, P))
        _, idx = o.encoder(params, SYNTH_MEAN, SYNTH_STD, patches, P, 2, m)
        f, _ = o.decoder(params, SYNTH_MEAN, SYNTH_STD, idx, 2, m)
        ref = o.around_u8(o.concat_patches(f, img.shape[0], img.shape[1], P))
        d = np.abs(rec.astype(int) - ref.astype(int))
        # symbols may differ only inside the quantiser tie band; allow a tiny fraction
        assert float(np.mean(d > 1)) < 1e-3, float(np.mean(d > 1))
        assert abs(o.dataset_psnr([(img, rec)]) - o.dataset_psnr([(img, ref)])) < 0.02


def test_rmbe_postfilter_pipeline():
    from tf_image_compression_amd.rmbe import RmbeFilter
    from tf_image_compression_amd.weights import synthetic_params, SYNTH_MEAN, SYNTH_STD
    from tf_image_compression_amd.topology import RMBE_ID
    params = synthetic_params(RMBE_ID)
    r = np.random.default_rng(8)
    img = np.clip(r.normal(128, 40, (300, 330, 3)), 0, 255).astype(np.float32)
    filt = RmbeFilter(params, SYNTH_MEAN, SYNTH_STD)
    got = filt.apply(img)
    filt.close()
    ref = o.rmbe(img, params, SYNTH_MEAN, SYNTH_STD)
    assert float(np.max(np.abs(got - ref))) < 2e-2
    # edge strips outside every window are untouched
    assert np.array_equal(got[256:, 256:], img[256:, 256:])
