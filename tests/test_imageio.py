import numpy as np

from pgi_raytracing_amd.imageio import load_pfm, save_pfm, save_png, to_rgb8


def test_pfm_round_trip(tmp_path):
    rng = np.random.default_rng(0)
    img = rng.normal(size=(7, 11, 4)).astype(np.float32)
    img[2, 3, 0] = np.nan
    p = str(tmp_path / "f.pfm")
    save_pfm(p, img)
    back = load_pfm(p)
    assert back.shape == (7, 11, 3)
    same = (back == img[..., :3]) | (np.isnan(back) & np.isnan(img[..., :3]))
    assert same.all()
    assert open(p, "rb").read(3) == b"PF\n"


def test_png_encoding(tmp_path):
    img = np.array([[[0.0, 0.5, 1.0, 1.0], [np.nan, 2.0, -1.0, 1.0]]], np.float32)
    assert to_rgb8(img).tolist() == [[[0, 128, 255], [0, 255, 0]]]
    save_png(str(tmp_path / "f.png"), img)
    from PIL import Image

    assert Image.open(str(tmp_path / "f.png")).size == (2, 1)
