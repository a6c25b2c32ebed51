"""Training-batch preparation on the GPU (STCGAN/dataset.py:89-147 and
STCGAN/transform.py:103-156).

The reference's ``ISTDDataset.__getitem__`` reads each image with cv2 (BGR), converts it with
``uint2float`` (u / 255), normalises ``(v - 0.5) * 2`` (the intent of dataset.py:122-124, which
references undefined names and raises NameError as written), then applies the transforms of
``transform.transforms(...)`` to (img, mask, target) with shared random draws.  Here the decoded
uint8 batch goes to the device once and ``stc_prepare_batch`` does normalisation, the horizontal
flip and the (zero-padded) random crop in one pass.  The random parameters are drawn on the host
in the reference's order per sample: ``np.random.rand() > flip_prob`` (no flip), then
``randint(0, rows - crop_rows)`` and ``randint(0, cols - crop_cols)``.  The whole composition of
``transform.transforms`` runs on the device in the reference's order -- Resize (cv.INTER_AREA when
shrinking in both axes, ``resize_area``; cv.INTER_LINEAR otherwise, ``resize_linear``),
RandomScale and RandomRotate (cv.warpAffine about the image centre, ``warp_affine``), then flip
and crop -- with the draws of each sample in that order: ``uniform(1 - scale, 1 + scale)``,
``uniform(-angle, angle)``, the flip, the two crop offsets.  ``ISTDLoader`` replaces the
reference's ``DataLoader(ISTDDataset(...))`` (STCGAN/stcgan.py:73-100) on top of it.
"""
import math
import os

import numpy as np
import torch

from ._lib import check, lib, ptr, stream


def augment_params(n, H, W, flip_prob=None, crop_size=None, rng=np.random):
    """Per-sample {flip, row_offset, col_offset} and the crop geometry (pad_h, pad_w, OH, OW)."""
    if crop_size is None:
        OH, OW = H, W
    elif isinstance(crop_size, (int, np.integer)):
        OH, OW = int(crop_size), int(crop_size)
    else:
        OH, OW = (int(v) for v in crop_size)
    pad_h, pad_w = (max(OH - H, 0), max(OW - W, 0)) if (OH > H or OW > W) else (0, 0)
    rows, cols = H + 2 * pad_h, W + 2 * pad_w
    params = np.zeros((n, 3), np.int32)
    for i in range(n):
        if flip_prob is not None:
            params[i, 0] = 0 if rng.rand() > flip_prob else 1
        if crop_size is not None:
            params[i, 1] = rng.randint(low=0, high=rows - OH)
            params[i, 2] = rng.randint(low=0, high=cols - OW)
    return params, (pad_h, pad_w, OH, OW)


def rotation_matrix(cols, rows, angle, scale):
    """cv.getRotationMatrix2D(((cols - 1) / 2, (rows - 1) / 2), angle, scale): float64 [2, 3]."""
    cx, cy = float(np.float32((cols - 1) / 2.0)), float(np.float32((rows - 1) / 2.0))  # Point2f centre
    a = angle * (math.pi / 180)
    alpha, beta = math.cos(a) * scale, math.sin(a) * scale
    return np.array([[alpha, beta, (1 - alpha) * cx - beta * cy],
                     [-beta, alpha, beta * cx + (1 - alpha) * cy]], np.float64)


def _nhwc(t):
    return t.unsqueeze(-1) if t.dim() == 3 else t


def warp_affine(images, mats):
    """cv.warpAffine(img_b, M_b, (W, H), INTER_LINEAR, BORDER_CONSTANT 0) for every image of a batch;
    images: uint8 (normalised on the fly) or fp32 NHWC CUDA tensor; mats: [B, 2, 3] float64."""
    src = _nhwc(images).contiguous()
    B, H, W, C = src.shape
    M = torch.as_tensor(np.ascontiguousarray(mats, np.float64).reshape(B, 6)).pin_memory().to(src.device, non_blocking=True)
    out = torch.empty((B, H, W, C), dtype=torch.float32, device=src.device)
    check(lib().stc_warp_affine(ptr(src), int(src.dtype == torch.uint8), B, H, W, C, ptr(M), ptr(out), stream()),
          "stc_warp_affine")
    return out


def resize_linear(images, size):
    """cv.resize INTER_LINEAR of the normalised images (the Resize of transform.py:173-178 when it
    does not shrink both axes): uint8 or fp32 NHWC -> fp32 NHWC [B, rows, cols, C]."""
    src = _nhwc(images).contiguous()
    B, H, W, C = src.shape
    rows, cols = (size, size) if isinstance(size, (int, np.integer)) else size
    out = torch.empty((B, rows, cols, C), dtype=torch.float32, device=src.device)
    check(lib().stc_resize_linear(ptr(src), int(src.dtype == torch.uint8), B, H, W, C, rows, cols, ptr(out),
                                  stream()), "stc_resize_linear")
    return out


def resize(images_u8, size):
    """Resize (transform.py:159-181): INTER_AREA when both axes shrink, INTER_LINEAR otherwise."""
    H, W = images_u8.shape[1:3]
    rows, cols = (size, size) if isinstance(size, (int, np.integer)) else size
    if rows < H and cols < W:
        return resize_area(images_u8, size)
    return resize_linear(images_u8, size)


def resize_area(images_u8, size):
    """Resize (transform.py:159-181) of the normalised images when they shrink in both dimensions
    (cv.INTER_AREA): uint8 [B, H, W, C] -> fp32 NHWC [B, rows, cols, C]."""
    if images_u8.dim() == 3:
        images_u8 = images_u8.unsqueeze(-1)
    src = images_u8.contiguous()
    B, H, W, C = src.shape
    rows, cols = (size, size) if isinstance(size, (int, np.integer)) else size
    if not (rows < H and cols < W):
        raise NotImplementedError("stcgan_amd.data: Resize is restated for shrinking (INTER_AREA) only")
    out = torch.empty((B, rows, cols, C), dtype=torch.float32, device=src.device)
    check(lib().stc_resize_area(ptr(src), B, H, W, C, rows, cols, ptr(out), stream()), "stc_resize_area")
    return out


def prepare(images, params, geom):
    """[B, H, W, C] CUDA tensor -> fp32 [B, C, OH, OW] = crop(flip(v)), v = (u / 255 - 0.5) * 2 for a
    uint8 source, or the fp32 source as is (already normalised, e.g. by resize_area)."""
    if not images.is_cuda:
        raise RuntimeError("stcgan_amd.data: CUDA (HIP) tensors only")
    if images.dim() == 3:
        images = images.unsqueeze(-1)
    src = images.contiguous()
    B, H, W, C = src.shape
    pad_h, pad_w, OH, OW = geom
    p = torch.as_tensor(np.ascontiguousarray(params, np.int32)).pin_memory().to(src.device, non_blocking=True)
    out = torch.empty((B, C, OH, OW), dtype=torch.float32, device=src.device)
    if src.dtype == torch.uint8:
        check(lib().stc_prepare_batch(ptr(src), B, H, W, C, ptr(p), pad_h, pad_w, OH, OW, ptr(out), stream()),
              "stc_prepare_batch")
    elif src.dtype == torch.float32:
        check(lib().stc_prepare_batch_f32(ptr(src), B, H, W, C, ptr(p), pad_h, pad_w, OH, OW, ptr(out), stream()),
              "stc_prepare_batch_f32")
    else:
        raise TypeError(f"stcgan_amd.data: uint8 or fp32 images, got {src.dtype}")
    return out


def draw_params(n, H, W, scale=None, angle=None, flip_prob=None, crop_size=None, rng=np.random):
    """The random draws of transform.transforms(scale, angle, flip_prob, crop_size) for n samples,
    per sample in the reference's order (RandomScale, RandomRotate, RandomHorizontalFlip,
    RandomCrop): ([n] scales or None, [n] angles or None, [n, 3] flip/crop params, crop geometry)."""
    if crop_size is None:
        OH, OW = H, W
    elif isinstance(crop_size, (int, np.integer)):
        OH, OW = int(crop_size), int(crop_size)
    else:
        OH, OW = (int(v) for v in crop_size)
    pad_h, pad_w = (max(OH - H, 0), max(OW - W, 0)) if (OH > H or OW > W) else (0, 0)
    rows, cols = H + 2 * pad_h, W + 2 * pad_w
    scales = np.zeros(n) if scale is not None else None
    angles = np.zeros(n) if angle is not None else None
    params = np.zeros((n, 3), np.int32)
    for i in range(n):
        if scale is not None:
            scales[i] = rng.uniform(low=1.0 - scale, high=1.0 + scale)
        if angle is not None:
            angles[i] = rng.uniform(low=-angle, high=angle)
        if flip_prob is not None:
            params[i, 0] = 0 if rng.rand() > flip_prob else 1
        if crop_size is not None:
            params[i, 1] = rng.randint(low=0, high=rows - OH)
            params[i, 2] = rng.randint(low=0, high=cols - OW)
    return scales, angles, params, (pad_h, pad_w, OH, OW)


def apply_draws(tensors, scales, angles, params, geom):
    """The transforms after Resize for drawn parameters: RandomScale / RandomRotate warps (one
    launch per tensor and transform), then flip + crop + NCHW (``prepare``)."""
    B, H, W = tensors[0].shape[:3]
    if scales is not None:
        mats = np.stack([rotation_matrix(W, H, 0, s) for s in scales])
        tensors = [warp_affine(t, mats) for t in tensors]
    if angles is not None:
        mats = np.stack([rotation_matrix(W, H, a, 1) for a in angles])
        tensors = [warp_affine(t, mats) for t in tensors]
    return [prepare(t, params, geom) for t in tensors]


def prepare_samples(tensors, flip_prob=None, crop_size=None, rng=np.random, resize=None, scale=None, angle=None):
    """(img, mask, target, ...) uint8 batches [B, H, W(, C)] sharing one draw per sample -> fp32 NCHW
    batches: transform.transforms(resize, scale, angle, flip_prob, crop_size) on the device."""
    assert scale is None or 0 <= scale <= 0.5  # RandomScale's own check (transform.py:61-62)
    if resize is not None:
        tensors = [globals()["resize"](t, resize) for t in tensors]
    B, H, W = tensors[0].shape[:3]
    scales, angles, params, geom = draw_params(B, H, W, scale, angle, flip_prob, crop_size, rng)
    return apply_draws(tensors, scales, angles, params, geom), params


def shard_bounds(n, rank, world):
    """Rank ``rank``'s slice of a global batch of n: equal shards; a ragged final batch is split
    as evenly as possible (sizes differ by at most one)."""
    q, r = divmod(n, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


class ISTDLoader:
    """The reference's ``DataLoader(ISTDDataset(root, subset, datas, transforms), batch_size, shuffle,
    drop_last, num_workers, worker_init_fn=np.random.seed(42 + id))`` (STCGAN/dataset.py:17-151,
    STCGAN/stcgan.py:73-104) with the decode on the host and everything after it on the device.

    Yields (names, *tensors) with the tensors in sorted ``datas`` order (img, mask, matte, target as
    the reference's ``sorted(sample.keys())``), fp32 NCHW CUDA batches.  Files:
    {root}/{subset}/{subset}_A (img), _B (mask), _matte, _C_fixed (target), each sorted by stem; the
    four directories must hold as many files (the reference's assertions).  Decode: PIL, colour
    images reordered to BGR (cv.IMREAD_COLOR), masks/mattes as 8-bit grey (cv.IMREAD_GRAYSCALE) --
    identical pixels for ISTD's lossless PNGs.

    Random streams, as the reference's DataLoader consumes them: every epoch draws the iterator's
    base seed and, with ``shuffle``, RandomSampler's seed from torch's global generator and permutes
    with ``torch.randperm``; the transform draws of batch s come from worker ``s % workers``'s numpy
    stream, seeded 42 + id at every epoch start (non-persistent workers), or from the global
    ``np.random`` when ``workers == 0``.  With ``world > 1`` every rank draws the same global batch
    and decodes and prepares only its shard (``shard_bounds``), as nn.DataParallel scatters it; a
    final batch smaller than ``world`` is skipped on every rank (no rank may sit out a step's
    collectives), and the trainer weights each rank's loss means of a ragged final batch by its share
    (``last_global``: the global size of the batch last yielded; stcgan.batch_weight)."""

    DIRS = {"img": "A", "mask": "B", "matte": "matte", "target": "C_fixed"}

    def __init__(self, root, subset, batch_size, datas=("img", "mask", "target"), resize=None, scale=None,
                 angle=None, flip_prob=None, crop_size=None, shuffle=False, drop_last=False, workers=0,
                 rank=0, world=1, device="cuda"):
        assert subset in ("train", "test")
        assert scale is None or 0 <= scale <= 0.5
        d = os.path.join(root, subset)
        stem = lambda f: os.path.splitext(f)[0]  # noqa: E731
        listing = {k: sorted(os.listdir(os.path.join(d, f"{subset}_{v}")), key=stem) for k, v in self.DIRS.items()}
        n = len(listing["img"])
        assert all(len(f) == n for f in listing.values())
        self.datas = sorted(datas)
        self.dirs = {k: os.path.join(d, f"{subset}_{self.DIRS[k]}") for k in self.datas}
        self.files = {k: listing[k] for k in self.datas}
        self.names = [stem(f) for f in listing["img"]]
        self.batch_size, self.shuffle, self.drop_last, self.workers = batch_size, shuffle, drop_last, workers
        self.resize = resize
        self.aug = dict(scale=scale, angle=angle, flip_prob=flip_prob, crop_size=crop_size)
        self.rank, self.world, self.device = rank, world, device
        self.last_global = None  # global size of the batch last yielded

    def __len__(self):
        n = len(self.names)
        return n // self.batch_size if self.drop_last else (n + self.batch_size - 1) // self.batch_size

    def _read(self, k, i):
        from PIL import Image
        with Image.open(os.path.join(self.dirs[k], self.files[k][i])) as im:
            if k in ("mask", "matte"):
                return np.asarray(im.convert("L"))
            return np.ascontiguousarray(np.asarray(im.convert("RGB"))[:, :, ::-1])

    def epoch_order(self):
        """The sample order of one epoch, consuming torch's global generator as DataLoader does."""
        torch.empty((), dtype=torch.int64).random_()  # _BaseDataLoaderIter._base_seed
        n = len(self.names)
        if not self.shuffle:
            return list(range(n))
        seed = int(torch.empty((), dtype=torch.int64).random_().item())
        g = torch.Generator()
        g.manual_seed(seed)
        return torch.randperm(n, generator=g).tolist()

    def schedule(self):
        """One epoch's host plan: (global sample indices, numpy stream of its transform draws) per batch."""
        order = self.epoch_order()
        streams = [np.random.RandomState(42 + w) for w in range(self.workers)]
        for s in range(len(self)):
            yield order[s * self.batch_size:(s + 1) * self.batch_size], (streams[s % self.workers] if self.workers
                                                                         else np.random)

    def __iter__(self):
        for sel, rng in self.schedule():
            lo, hi = shard_bounds(len(sel), self.rank, self.world)
            mine = sel[lo:hi]
            if len(sel) < self.world:  # some rank would get no sample: every rank skips the batch
                draw_params(len(sel), *self._shape(), rng=rng, **self.aug)  # keep the stream in step
                continue
            tensors = [torch.from_numpy(np.stack([self._read(k, i) for i in mine])).to(self.device)
                       for k in self.datas]
            if self.resize is not None:
                tensors = [resize(t, self.resize) for t in tensors]
            H, W = tensors[0].shape[1:3]
            scales, angles, params, geom = draw_params(len(sel), H, W, rng=rng, **self.aug)
            self.last_global = len(sel)  # (the trainer's batch_weight)
            sl = slice(lo, hi)
            out = apply_draws(tensors, None if scales is None else scales[sl], None if angles is None else angles[sl],
                              params[sl], geom)
            yield ([self.names[i] for i in mine], *out)

    def _shape(self):
        if self.resize is not None:
            return (self.resize, self.resize) if isinstance(self.resize, (int, np.integer)) else tuple(self.resize)
        return self._read(self.datas[0], 0).shape[:2]
