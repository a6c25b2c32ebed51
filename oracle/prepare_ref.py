"""CPU oracle of the training-batch preparation -- TEST INFRASTRUCTURE ONLY (tests/ only).

numpy restatement of STCGAN/utils.py:58-60 (uint2float: float32 u / 255), the normalisation
(v - 0.5) * 2 of STCGAN/dataset.py:122-124, RandomHorizontalFlip (np.fliplr,
transform.py:103-116) and RandomCrop (cv.copyMakeBorder BORDER_CONSTANT 0 + slice,
transform.py:119-156; the zero border is a plain np.pad here -- cv2 is absent, the border
semantics are the documented constant fill), Resize (cv.resize INTER_AREA when shrinking in both
axes, INTER_LINEAR otherwise, transform.py:159-181) and RandomScale / RandomRotate
(getRotationMatrix2D + cv.warpAffine INTER_LINEAR, BORDER_CONSTANT 0, transform.py:59-100), each
restated from OpenCV's algorithm (float32 generic resize; warpAffine's inversion, 10-bit fixed-point
coordinates, 1/32-pixel bilinear table).  PARITY VS OPENCV UNPINNED (cv2 is not importable here).
"""
import math
import numpy as np


def prepare_one(img_u8, flip, oy, ox, pad_h, pad_w, oh, ow):
    x = np.asarray(img_u8)
    if x.ndim == 2:
        x = x[:, :, None]
    v = x.astype(np.float32) / np.float32(255)
    v = (v - np.float32(0.5)) * np.float32(2)
    if flip:
        v = np.fliplr(v).copy()
    if pad_h or pad_w:
        v = np.pad(v, ((pad_h, pad_h), (pad_w, pad_w), (0, 0)), constant_values=0)
    return v[oy:oy + oh, ox:ox + ow].transpose(2, 0, 1).astype(np.float32)


def _area_tab(dsize, ssize, scale):
    """OpenCV computeResizeAreaTab: per output index, [(source index, float32 weight), ...]."""
    tabs = []
    for d in range(dsize):
        fsx1 = d * scale
        fsx2 = fsx1 + scale
        cell = min(scale, ssize - fsx1)
        sx1, sx2 = int(np.ceil(fsx1)), int(np.floor(fsx2))
        sx2 = min(sx2, ssize - 1)
        sx1 = min(sx1, sx2)
        t = []
        if sx1 - fsx1 > 1e-3:
            t.append((sx1 - 1, np.float32((sx1 - fsx1) / cell)))
        for s in range(sx1, sx2):
            t.append((s, np.float32(1.0 / cell)))
        if fsx2 - sx2 > 1e-3:
            t.append((sx2, np.float32(min(min(fsx2 - sx2, 1.0), cell) / cell)))
        tabs.append(t)
    return tabs


def resize_area_one(img_u8, oh, ow):
    """cv.resize(normalised image, (ow, oh), INTER_AREA) restated (loops; small images only):
    generic cells (ResizeArea_Invoker order) or, for integer scales, the row-major block mean."""
    x = np.asarray(img_u8)
    if x.ndim == 2:
        x = x[:, :, None]
    v = (x.astype(np.float32) / np.float32(255) - np.float32(0.5)) * np.float32(2)
    h, w, c = v.shape
    sx, sy = 1.0 / (ow / w), 1.0 / (oh / h)
    out = np.zeros((oh, ow, c), np.float32)
    ix, iy = int(round(sx)), int(round(sy))
    if abs(sx - ix) < np.finfo(float).eps and abs(sy - iy) < np.finfo(float).eps:
        inv = np.float32(1.0) / np.float32(ix * iy)
        for dy in range(oh):
            for dx in range(ow):
                s = np.zeros(c, np.float32)
                for yy in range(iy):
                    for xx in range(ix):
                        s = (s + v[dy * iy + yy, dx * ix + xx]).astype(np.float32)
                out[dy, dx] = s * inv
        return out
    xt, yt = _area_tab(ow, w, sx), _area_tab(oh, h, sy)
    for dy in range(oh):
        for dx in range(ow):
            s = np.zeros(c, np.float32)
            for (yy, by) in yt[dy]:
                buf = np.zeros(c, np.float32)
                for (xx, ax) in xt[dx]:
                    buf = (buf + (v[yy, xx] * ax).astype(np.float32)).astype(np.float32)
                s = (s + (by * buf).astype(np.float32)).astype(np.float32)
            out[dy, dx] = s
    return out


def normalise(img_u8):
    x = np.asarray(img_u8)
    if x.ndim == 2:
        x = x[:, :, None]
    return (x.astype(np.float32) / np.float32(255) - np.float32(0.5)) * np.float32(2)


def resize_linear_one(v, oh, ow):
    """cv.resize(v (float32 HWC), (ow, oh), INTER_LINEAR), OpenCV's generic float path (loops)."""
    v = np.asarray(v, np.float32)
    h, w, c = v.shape
    sx, sy = 1.0 / (ow / w), 1.0 / (oh / h)
    out = np.zeros((oh, ow, c), np.float32)
    f32 = np.float32
    for dy in range(oh):
        fy = f32((dy + 0.5) * sy - 0.5)
        y0i = int(np.floor(fy))
        fy = f32(fy - f32(y0i))
        b0, b1 = f32(f32(1) - fy), fy
        ya, yb = min(max(y0i, 0), h - 1), min(max(y0i + 1, 0), h - 1)
        for dx in range(ow):
            fx = f32((dx + 0.5) * sx - 0.5)
            x0 = int(np.floor(fx))
            fx = f32(fx - f32(x0))
            two = x0 + 1 < w
            if x0 < 0:
                fx, x0 = f32(0), 0
            if x0 >= w - 1:
                fx, x0 = f32(0), w - 1
            a0, a1 = f32(f32(1) - fx), fx
            x1 = x0 + 1 if two else x0
            hh = []
            for yy in (ya, yb):
                t0 = (v[yy, x0] * a0).astype(np.float32)
                hh.append((t0 + (v[yy, x1] * a1).astype(np.float32)).astype(np.float32) if two else t0)
            out[dy, dx] = ((hh[0] * b0).astype(np.float32) + (hh[1] * b1).astype(np.float32)).astype(np.float32)
    return out


def rotation_matrix(cols, rows, angle, scale):
    """cv.getRotationMatrix2D(((cols - 1) / 2, (rows - 1) / 2), angle, scale) (float64 2x3)."""
    cx, cy = float(np.float32((cols - 1) / 2.0)), float(np.float32((rows - 1) / 2.0))  # Point2f centre
    a = angle * (math.pi / 180)
    alpha, beta = math.cos(a) * scale, math.sin(a) * scale
    return np.array([[alpha, beta, (1 - alpha) * cx - beta * cy],
                     [-beta, alpha, beta * cx + (1 - alpha) * cy]], np.float64)


def _cv_round(v):
    return int(np.rint(v))  # cvRound: nearest, ties to even


def warp_affine_one(v, M):
    """cv.warpAffine(v (float32 HWC), M, (W, H), INTER_LINEAR, BORDER_CONSTANT 0) (loops)."""
    v = np.asarray(v, np.float32)
    h, w, c = v.shape
    M = [float(t) for t in np.asarray(M, np.float64).reshape(-1)]
    D = M[0] * M[4] - M[1] * M[3]
    D = 1. / D if D != 0 else 0.
    A11, A22 = M[4] * D, M[0] * D
    M[0] = A11
    M[1] *= -D
    M[3] *= -D
    M[4] = A22
    b1 = -M[0] * M[2] - M[1] * M[5]
    b2 = -M[3] * M[2] - M[4] * M[5]
    M[2], M[5] = b1, b2
    f32 = np.float32
    out = np.zeros((h, w, c), np.float32)
    for y in range(h):
        X0 = _cv_round((M[1] * y + M[2]) * 1024) + 16
        Y0 = _cv_round((M[4] * y + M[5]) * 1024) + 16
        for x in range(w):
            X = (X0 + _cv_round(M[0] * x * 1024)) >> 5
            Y = (Y0 + _cv_round(M[3] * x * 1024)) >> 5
            sx, sy = X >> 5, Y >> 5
            fx, fy = f32(X & 31) * f32(1 / 32), f32(Y & 31) * f32(1 / 32)
            vx0, vy0 = f32(1) - fx, f32(1) - fy
            wts = (vy0 * vx0, vy0 * fx, fy * vx0, fy * fx)

            def tap(yy, xx):
                return v[yy, xx] if 0 <= yy < h and 0 <= xx < w else np.zeros(c, np.float32)

            t = (tap(sy, sx) * wts[0]).astype(f32)
            t = (t + (tap(sy, sx + 1) * wts[1]).astype(f32)).astype(f32)
            t = (t + (tap(sy + 1, sx) * wts[2]).astype(f32)).astype(f32)
            t = (t + (tap(sy + 1, sx + 1) * wts[3]).astype(f32)).astype(f32)
            out[y, x] = t
    return out
