"""CPU oracle of the training-batch preparation -- TEST INFRASTRUCTURE ONLY (tests/ only).

numpy restatement of STCGAN/utils.py:58-60 (uint2float: float32 u / 255), the normalisation
(v - 0.5) * 2 of STCGAN/dataset.py:122-124, RandomHorizontalFlip (np.fliplr,
transform.py:103-116) and RandomCrop (cv.copyMakeBorder BORDER_CONSTANT 0 + slice,
transform.py:119-156; the zero border is a plain np.pad here -- cv2 is absent, the border
semantics are the documented constant fill).
"""
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
