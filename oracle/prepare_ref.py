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
