"""lib/preprocess.py restatement (offline, host-only).
OpenCV is absent from this image, so parity is unpinned: the checks are
known-answer values of the OpenCV operations restated (documented OpenCV
behaviour: contourArea of a filled w x h block = (w-1)(h-1), the 8-bit
bilinear ramp 0,100 -> 0,25,75,100, 14-bit gray weights) and the geometric
properties the reference pipeline relies on."""
import os

import numpy as np
import pytest

import lib.preprocess as P


def test_contrast_curve_and_gray():
    x = np.array([0, 100, 170, 200, 255], np.uint8)
    want = np.array((255 / 1.3) * (x / (255 / 1.5)) ** 2).astype(np.uint8)   # numpy cast, as the reference
    np.testing.assert_array_equal(P._increase_contrast(x), want)
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, (50, 40, 3), dtype=np.uint8)
    g = P._bgr2gray(img)
    ref = 0.114 * img[..., 0] + 0.587 * img[..., 1] + 0.299 * img[..., 2]
    assert g.dtype == np.uint8 and np.max(np.abs(g - ref)) <= 0.51
    assert P._bgr2gray(np.full((2, 2, 3), 255, np.uint8)).min() == 255


def test_external_contours_area_and_moments():
    m = np.zeros((20, 20), np.uint8)
    m[5:15, 3:13] = 7
    (c,) = P._find_external_contours(m)
    assert P._contour_area(c) == 81.0                       # (10-1) x (10-1) through pixel centres
    m00, m10, m01 = P._polygon_moments(c)
    assert (m10 / m00, m01 / m00) == (7.5, 9.5)
    one = np.zeros((5, 5), np.uint8)
    one[2, 3] = 1
    (c1,) = P._find_external_contours(one)
    assert c1.tolist() == [[3.0, 2.0]] and P._contour_area(c1) == 0
    ring = np.zeros((40, 40), np.uint8)
    ring[5:35, 5:35] = 1
    ring[10:30, 10:30] = 0
    ring[15:20, 15:20] = 1                                   # inside the hole: not external
    ring[0:3, 37:40] = 1                                     # touches the frame: still traced
    cs = P._find_external_contours(ring)
    assert sorted(P._contour_area(c) for c in cs) == [4.0, 29.0 * 29.0]
    diag = np.eye(6, dtype=np.uint8)                         # 8-connected: one component
    assert len(P._find_external_contours(diag)) == 1


def test_min_enclosing_circle():
    (cx, cy), r = P._min_enclosing_circle(np.array([[0, 0], [4, 0], [4, 4], [0, 4], [2, 2]], float))
    assert (cx, cy) == (2.0, 2.0) and abs(r - np.float32(np.sqrt(8))) == 0
    (cx, cy), r = P._min_enclosing_circle(np.array([[0, 0], [1, 0], [6, 0]], float))
    assert (cx, cy, r) == (3.0, 0.0, 3.0)


def test_bilinear_resize_known_answers():
    ramp = np.array([[0, 100]], np.uint8)
    np.testing.assert_array_equal(P.resize_linear(ramp, (4, 1)), [[0, 25, 75, 100]])
    rng = np.random.default_rng(1)
    img = rng.integers(0, 256, (13, 17, 3), dtype=np.uint8)
    np.testing.assert_array_equal(P.resize_linear(img, fx=1.0, fy=1.0), img)
    const = np.full((31, 29, 3), 173, np.uint8)
    out = P.resize_linear(const, fx=0.37, fy=0.37)
    assert out.shape == (int(np.rint(31 * 0.37)), int(np.rint(29 * 0.37)), 3) and np.all(out == 173)


def _fundus(h, w, cy, cx, r, seed=0):
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[:h, :w]
    img = np.zeros((h, w, 3), np.uint8)
    disc = (yy - cy) ** 2 + (xx - cx) ** 2 <= r * r
    base = np.array([40, 85, 180], np.float64)               # BGR
    img[disc] = np.clip(base + rng.normal(0, 8, (disc.sum(), 3)), 1, 255).astype(np.uint8)
    return img


def test_find_contours_locates_the_disc():
    img = _fundus(600, 700, 290, 360, 240)
    (cx, cy), r = P._find_contours(img)
    assert abs(cx - 360) <= 1 and abs(cy - 290) <= 1 and abs(r - 240) <= 1
    assert P._find_contours(_fundus(300, 300, 150, 150, 90)) is None        # radius <= 100 rejected
    assert P._find_contours(np.zeros((50, 50, 3), np.uint8)) is None


def test_scale_normalize_files_and_resize(tmp_path):
    from PIL import Image
    src = tmp_path / "src"
    dst = tmp_path / "dst"
    src.mkdir()
    dst.mkdir()
    img = _fundus(560, 640, 300, 330, 230, seed=3)
    Image.fromarray(img[..., ::-1]).save(src / "10_left.png")            # stored RGB, like a fundus photo
    Image.fromarray(np.zeros((200, 200, 3), np.uint8)).save(src / "blank.png")
    n = P.scale_normalize(save_path=str(dst), images_path=str(src), diameter=299, verbosity=0)
    assert n == 1 and os.listdir(dst) == ["10_left.jpg"]
    out = np.asarray(Image.open(dst / "10_left.jpg"))
    assert out.shape == (299, 299, 3)
    assert out[:3, :3].max() < 16 and out[-3:, -3:].max() < 16              # black outside the disc
    lum = out.astype(np.float64).mean(axis=2) > 30
    ys, xs = np.nonzero(lum)
    assert abs(ys.mean() - 149) < 2 and abs(xs.mean() - 149) < 2          # disc centred
    assert 290 <= ys.max() - ys.min() + 1 <= 299                           # diameter ~ 299
    assert abs(out[149, 149].astype(int) - img[300, 330, ::-1]).max() < 40  # colours kept (RGB on disk)
    with pytest.raises(ValueError):
        P.scale_normalize(images_path=str(src))
    big = tmp_path / "big.jpg"
    Image.fromarray(np.zeros((400, 500, 3), np.uint8)).save(big)
    P.resize([str(big)], size=299)
    assert Image.open(big).size == (299, 299)
