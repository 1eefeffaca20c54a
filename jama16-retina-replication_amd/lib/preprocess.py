"""Drop-in for the reference's lib/preprocess.py, no OpenCV.

Same public entry points and arguments:
    scale_normalize(save_path=None, images_path=None, image_paths=None,
                    image_path=None, diameter=299, verbosity=1)  -> #written
    resize(images_paths, size=299)
and the same per-image algorithm (lib/preprocess.py:17-130):
  1. contrast curve  (255/1.3) * (x / (255/1.5))**2, cast to uint8 the numpy
     way (:17-37);
  2. BGR -> gray, then the external contours of the non-zero pixels; the
     largest by polygon area; its minimum enclosing circle; accepted only
     when radius > 100; centre = the contour polygon's centroid m10/m00,
     truncated to int (:40-70);
  3. crop the 2r square at (centre - r) (clipped at 0 on the low side only,
     numpy slicing on the high side), bilinear resize by (diameter/2)/r,
     zero-pad to diameter x diameter with the odd pixel on top/left
     (:81-126); JPEG q=100 out, named <stem>.jpg (:137-173).

OpenCV pieces restated [cv2-3P, version unpinned; parity unpinned — no cv2 in
this image, see DESIGN.md §4]:
  * cvtColor BGR2GRAY, 8-bit: (1868 B + 9617 G + 4899 R + 2^13) >> 14;
  * findContours(RETR_EXTERNAL): outer borders of the 8-connected components
    of non-zero pixels that are not inside a hole of another component, image
    frame padded with zeros (OpenCV >= 3.2 behaviour); traced with Moore
    neighbour tracing from the first pixel in raster order;
  * contourArea / moments: Green's-theorem polygon sums over the border
    pixel centres (collinear points do not change them, so
    CHAIN_APPROX_SIMPLE's compression is immaterial);
  * minEnclosingCircle: the exact minimal circle of the border points
    (float64), reported as float32 like cv::Point2f / float;
  * resize INTER_LINEAR, 8-bit: src = (d + 0.5) / f - 0.5 in float, edge
    clamped, 11-bit fixed-point weights, (sum + 2^21) >> 22 (the scalar
    path of OpenCV's fixed-point bilinear);
  * imread(-1) / imwrite(JPEG, 100): Pillow, channels kept in BGR order
    inside like cv2.
"""
from __future__ import annotations

import os
import sys
from typing import List, Optional, Tuple

import numpy as np

try:
    from PIL import Image
except ImportError:  # pragma: no cover
    Image = None

try:
    from scipy import ndimage
except ImportError:  # pragma: no cover
    ndimage = None


# ------------------------------------------------------------- pixel ops
def _increase_contrast(image: np.ndarray) -> np.ndarray:
    """lib/preprocess.py:17-37: dark pixels much darker, bright slightly."""
    top = 255.0
    out = (top / 1.3) * (image / (top / 1.5)) ** 2
    return np.array(out, dtype=np.uint8)


def _bgr2gray(image: np.ndarray) -> np.ndarray:
    """cv2.cvtColor(COLOR_BGR2GRAY) for uint8 (14-bit fixed point)."""
    if image.ndim == 2:
        return image
    b = image[..., 0].astype(np.int32)
    g = image[..., 1].astype(np.int32)
    r = image[..., 2].astype(np.int32)
    return ((b * 1868 + g * 9617 + r * 4899 + (1 << 13)) >> 14).astype(np.uint8)


# --------------------------------------------------------------- contours
# clockwise in image coordinates (y down), starting east
_DY = (0, 1, 1, 1, 0, -1, -1, -1)
_DX = (1, 1, 0, -1, -1, -1, 0, 1)
_DIR = {(dy, dx): k for k, (dy, dx) in enumerate(zip(_DY, _DX))}


def _trace_outer(mask: np.ndarray, sy: int, sx: int) -> np.ndarray:
    """Moore-neighbour trace of the outer border through (sy, sx), the first
    pixel of its component in raster order.  Returns [n, 2] (x, y) points."""
    h, w = mask.shape
    pts = [(sx, sy)]
    cy, cx, back = sy, sx, 4            # the west neighbour of the first pixel is background
    first = None
    while True:
        for k in range(1, 9):
            d = (back + k) % 8
            ny, nx = cy + _DY[d], cx + _DX[d]
            if 0 <= ny < h and 0 <= nx < w and mask[ny, nx]:
                p = (back + k - 1) % 8
                by, bx = cy + _DY[p], cx + _DX[p]
                cy, cx = ny, nx
                back = _DIR[(by - cy, bx - cx)]
                break
        else:
            return np.array(pts, np.float64)        # isolated pixel
        state = (cy, cx, back)
        if first is None:
            first = state
        elif state == first:                         # Jacob's stopping criterion
            break
        pts.append((cx, cy))
    return np.array(pts[:-1] if len(pts) > 1 else pts, np.float64)


def _find_external_contours(gray: np.ndarray) -> List[np.ndarray]:
    """cv2.findContours(gray, RETR_EXTERNAL, CHAIN_APPROX_SIMPLE)[-2] (as
    point sets; see the module docstring)."""
    if ndimage is None:
        raise RuntimeError("scipy is required for contour detection")
    fg = gray != 0
    # components inside a hole of another component are not external: fill
    # the holes (background 4-connected, as the dual of 8-connected
    # foreground), then every 8-connected component has one outer border
    filled = ndimage.binary_fill_holes(fg)
    lab, n = ndimage.label(filled, structure=np.ones((3, 3), bool))
    out = []
    for sl, k in zip(ndimage.find_objects(lab), range(1, n + 1)):
        sub = lab[sl] == k
        ys, xs = np.nonzero(sub[:1])                 # first row of the box holds the raster-first pixel
        c = _trace_outer(sub, 0, int(xs[0]))
        c[:, 0] += sl[1].start
        c[:, 1] += sl[0].start
        out.append(c)
    return out


def _polygon_moments(c: np.ndarray) -> Tuple[float, float, float]:
    """m00, m10, m01 of the closed polygon (cv2.moments of a contour)."""
    x, y = c[:, 0], c[:, 1]
    xn, yn = np.roll(x, -1), np.roll(y, -1)
    cr = x * yn - xn * y
    m00 = cr.sum() / 2.0
    m10 = ((x + xn) * cr).sum() / 6.0
    m01 = ((y + yn) * cr).sum() / 6.0
    if m00 < 0:
        m00, m10, m01 = -m00, -m10, -m01
    return m00, m10, m01


def _contour_area(c: np.ndarray) -> float:
    return abs(_polygon_moments(c)[0])


def _circle2(a, b):
    cx, cy = (a[0] + b[0]) / 2, (a[1] + b[1]) / 2
    return cx, cy, np.hypot(a[0] - cx, a[1] - cy)


def _circle3(a, b, c):
    ax, ay = a
    bx, by = b
    cx, cy = c
    d = 2 * (ax * (by - cy) + bx * (cy - ay) + cx * (ay - by))
    if abs(d) < 1e-12:                                # collinear: widest pair
        return max((_circle2(a, b), _circle2(a, c), _circle2(b, c)), key=lambda t: t[2])
    ux = ((ax * ax + ay * ay) * (by - cy) + (bx * bx + by * by) * (cy - ay) + (cx * cx + cy * cy) * (ay - by)) / d
    uy = ((ax * ax + ay * ay) * (cx - bx) + (bx * bx + by * by) * (ax - cx) + (cx * cx + cy * cy) * (bx - ax)) / d
    return ux, uy, np.hypot(ax - ux, ay - uy)


def _min_enclosing_circle(pts: np.ndarray) -> Tuple[Tuple[float, float], float]:
    """Exact minimal enclosing circle (incremental Welzl, fixed shuffle)."""
    p = [tuple(v) for v in np.unique(pts, axis=0)]
    np.random.default_rng(0).shuffle(p)
    eps = 1e-9

    def inside(c, q):
        return np.hypot(q[0] - c[0], q[1] - c[1]) <= c[2] + eps

    c = (p[0][0], p[0][1], 0.0)
    for i in range(1, len(p)):
        if inside(c, p[i]):
            continue
        c = (p[i][0], p[i][1], 0.0)
        for j in range(i):
            if inside(c, p[j]):
                continue
            c = _circle2(p[i], p[j])
            for k in range(j):
                if not inside(c, p[k]):
                    c = _circle3(p[i], p[j], p[k])
    f = np.float32
    return (float(f(c[0])), float(f(c[1]))), float(f(c[2]))


def _find_contours(image: np.ndarray):
    """lib/preprocess.py:40-70: ((cx, cy), radius) of the fundus, or None."""
    gray = _bgr2gray(_increase_contrast(image))
    cnts = _find_external_contours(gray)
    if not cnts:
        return None
    c = max(cnts, key=_contour_area)
    _, radius = _min_enclosing_circle(c)
    if radius > 100:
        m00, m10, m01 = _polygon_moments(c)
        return (int(m10 / m00), int(m01 / m00)), radius
    return None


# ----------------------------------------------------------------- resize
def _linear_taps(n_src: int, n_dst: int, scale: float):
    """Per destination index: (i0, i1, w0, w1) with 11-bit weights."""
    d = np.arange(n_dst, dtype=np.float64)
    f = ((d + 0.5) * scale - 0.5).astype(np.float32)
    i0 = np.floor(f).astype(np.int64)
    f = (f - i0).astype(np.float32)
    low = i0 < 0
    f[low], i0[low] = 0, 0
    high = i0 >= n_src - 1
    f[high], i0[high] = 0, n_src - 1
    w0 = np.round((np.float32(1) - f) * np.float32(2048)).astype(np.int64)   # saturate_cast<short>
    i1 = np.minimum(i0 + 1, n_src - 1)
    return i0, i1, w0, 2048 - w0


def resize_linear(image: np.ndarray, dsize: Optional[Tuple[int, int]] = None,
                  fx: float = 0.0, fy: float = 0.0) -> np.ndarray:
    """cv2.resize(image, dsize, fx=fx, fy=fy) with INTER_LINEAR, uint8."""
    h, w = image.shape[:2]
    if dsize is None or dsize == (0, 0):
        dw, dh = int(np.rint(w * fx)), int(np.rint(h * fy))
    else:
        dw, dh = dsize
        fx, fy = dw / w, dh / h
    if dw <= 0 or dh <= 0:
        raise ValueError("resize: empty destination")
    x0, x1, a0, a1 = _linear_taps(w, dw, 1.0 / fx)
    y0, y1, b0, b1 = _linear_taps(h, dh, 1.0 / fy)
    src = image.astype(np.int64)
    shp = (1, -1) + (1,) * (image.ndim - 2)
    rows0 = src[y0][:, x0] * a0.reshape(shp) + src[y0][:, x1] * a1.reshape(shp)
    rows1 = src[y1][:, x0] * a0.reshape(shp) + src[y1][:, x1] * a1.reshape(shp)
    colshp = (-1, 1) + (1,) * (image.ndim - 2)
    acc = rows0 * b0.reshape(colshp) + rows1 * b1.reshape(colshp)
    return np.clip((acc + (1 << 21)) >> 22, 0, 255).astype(np.uint8)


# ------------------------------------------------------------ scale norm
def _scale_normalize(image: np.ndarray, diameter: int) -> Optional[np.ndarray]:
    """lib/preprocess.py:81-126."""
    found = _find_contours(image)
    if found is None:
        return None
    (cx, cy), radius = found
    x_min = max(0, int(cx - radius))
    y_min = max(0, int(cy - radius))
    z = int(radius * 2)
    crop = image[y_min:y_min + z, x_min:x_min + z]
    f = (diameter / 2) / radius
    out = resize_linear(crop, fx=f, fy=f)
    top = bottom = int((diameter - out.shape[0]) / 2)
    left = right = int((diameter - out.shape[1]) / 2)
    if out.shape[0] + top + bottom == diameter - 1:
        top += 1
    if out.shape[1] + left + right == diameter - 1:
        left += 1
    pad = [(top, bottom), (left, right)] + [(0, 0)] * (out.ndim - 2)
    return np.pad(out, pad, mode="constant", constant_values=0)


def _imread(path: str) -> np.ndarray:
    """cv2.imread(path, -1): uint8, colour channels in BGR(A) order."""
    if Image is None:
        raise RuntimeError("Pillow is required to read images")
    with Image.open(path) as im:
        im.load()
        a = np.asarray(im)
    if a.ndim == 3 and a.shape[2] >= 3:
        a = np.concatenate([a[..., 2::-1], a[..., 3:]], axis=2)
    return np.ascontiguousarray(a)


def _imwrite_jpeg(path: str, image: np.ndarray) -> None:
    """cv2.imwrite(path, image, [IMWRITE_JPEG_QUALITY, 100])."""
    rgb = image[..., 2::-1] if image.ndim == 3 else image
    Image.fromarray(np.ascontiguousarray(rgb)).save(path, format="JPEG", quality=100)


def _get_filename(file_path: str) -> str:
    return file_path.split("/")[-1]


def _get_image_paths(images_path: str) -> List[str]:
    return [os.path.join(images_path, fn) for fn in os.listdir(images_path)]


def _scale_normalize_all(image_paths, save_path, diameter, verbosity) -> int:
    """lib/preprocess.py:137-180: returns the number of images written."""
    total = len(image_paths)
    ok = 0
    for i, path in enumerate(image_paths):
        if verbosity > 0:
            sys.stdout.write("\r- Preprocessing image: {0:>6} / {1}".format(i + 1, total))
            sys.stdout.flush()
        try:
            image = _imread(os.path.abspath(path))
        except (OSError, ValueError) as e:      # cv2.imread returns None -> AttributeError in the reference
            print(e)
            print("Could not preprocess {}...".format(path))
            continue
        out = _scale_normalize(image, diameter=diameter)
        if out is None:
            print("Could not preprocess {}...".format(path))
            continue
        stem = os.path.splitext(os.path.basename(_get_filename(path)))[0]
        _imwrite_jpeg(os.path.join(save_path, "{0}.jpg".format(stem)), out)
        ok += 1
    return ok


def scale_normalize(save_path=None, images_path=None, image_paths=None,
                    image_path=None, diameter=299, verbosity=1):
    """lib/preprocess.py:183-228 (same argument precedence)."""
    if save_path is None:
        raise ValueError("Save path not specified!")
    save_path = os.path.abspath(save_path)
    if image_paths is not None:
        paths = image_paths
    elif images_path is not None:
        paths = _get_image_paths(images_path)
    elif image_path is not None:
        paths = [image_path]
    else:
        return None
    return _scale_normalize_all(paths, save_path, diameter, verbosity)


def resize(images_paths, size=299):
    """lib/preprocess.py:231-254: in-place resize to size x size, JPEG q=100."""
    for path in images_paths:
        image = _imread(path)[..., :3]
        _imwrite_jpeg(path, resize_linear(image, (size, size)))
