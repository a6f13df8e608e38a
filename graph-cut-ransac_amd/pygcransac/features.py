"""Feature front-end and output warp of the example notebook flow
(examples/utils.py:5-49 and :92-123 of the reference).

The reference takes cv2.KeyPoint lists.  cv2 is optional here: any object
with .pt, .size and .angle works, and so does an (N, 4) array of
(x, y, size, angle_degrees) rows (angle -1 = none, OpenCV's convention).
`perspective_warp` rectifies an image with the estimated homography on the
GPU (a HIP resampling kernel behind gcr_warp_perspective), cv2-free.
"""
from __future__ import annotations

import numpy as np

__all__ = ["scale_features_from_sift", "orientation_features_from_sift", "keypoints_to_array", "perspective_warp",
           "warp_geometry", "BORDER_CONSTANT", "BORDER_REPLICATE"]

# OpenCV's border codes (cv2.BORDER_CONSTANT = 0, cv2.BORDER_REPLICATE = 1)
BORDER_CONSTANT, BORDER_REPLICATE = 0, 1


def keypoints_to_array(keypoints) -> np.ndarray:
    """(N, 4) float64 rows (x, y, size, angle_deg) from cv2-style keypoints or an array."""
    if isinstance(keypoints, np.ndarray):
        a = np.asarray(keypoints, dtype=np.float64)
        if a.ndim != 2 or a.shape[1] < 4:
            raise ValueError("keypoint array must have shape (N, 4): x, y, size, angle (degrees)")
        return a[:, :4]
    rows = [(float(kp.pt[0]), float(kp.pt[1]), float(kp.size), float(kp.angle)) for kp in keypoints]
    return np.array(rows, dtype=np.float64).reshape(-1, 4)


def scale_features_from_sift(keypoints) -> np.ndarray:
    """One (x, y, size) row per distinct integer pixel, first keypoint wins,
    in first-seen order (utils.py:5-26: dict keyed by (int(x), int(y)))."""
    kp = keypoints_to_array(keypoints)
    unique = {}
    for row in kp:
        key = (int(row[0]), int(row[1]))          # int() truncates toward zero, as in Python
        if key not in unique:
            unique[key] = row
    if not unique:
        return np.array([])
    return np.array([[r[0], r[1], r[2]] for r in unique.values()])


def orientation_features_from_sift(keypoints):
    """(x, y, angle in radians) for every keypoint with an angle (!= -1) and the
    matching sizes 0.5 * size (utils.py:29-49)."""
    kp = keypoints_to_array(keypoints)
    feats, sizes = [], []
    for row in kp:
        if row[3] != -1:
            feats.append([row[0], row[1], np.deg2rad(row[3])])
            sizes.append(0.5 * row[2])
    return np.array(feats), np.array(sizes)


def warp_geometry(h: int, w: int, H):
    """Output frame of perspective_warp (utils.py:107-118): the image corners
    (0,0), (w,0), (w,h), (0,h) through H, their bounding box, the output size
    (ceil of its extent) and the translated homography T @ H that moves the
    box's minimum corner to the origin.

    Returns (H_translated (3, 3), (out_w, out_h), (min_x, min_y))."""
    H = np.asarray(H, dtype=np.float64).reshape(3, 3)
    corners = np.array([[0, 0, 1], [w, 0, 1], [w, h, 1], [0, h, 1]]).T
    wc = H @ corners
    wc = wc[:2] / wc[2]
    min_x, min_y = wc.min(axis=1)
    max_x, max_y = wc.max(axis=1)
    size = (int(np.ceil(max_x - min_x)), int(np.ceil(max_y - min_y)))
    translation = np.array([[1, 0, -min_x], [0, 1, -min_y], [0, 0, 1]])
    return translation @ H, size, (min_x, min_y)


def perspective_warp(img, H, border_mode=BORDER_CONSTANT, border_value=(255, 255, 255), device=None):
    """Warp `img` with homography H into an automatically sized frame
    (utils.py:92-123).  img: (h, w) or (h, w, c) uint8 / float32 array, c <= 4.

    Returns (warped_img, H_translated, (min_x, min_y)) like the reference.
    Resampling as cv2.warpPerspective's INTER_LINEAR: every output pixel takes
    the bilinear sample at inv(H_translated) (x, y, 1); neighbours outside the
    image take `border_value` (BORDER_CONSTANT) or the nearest edge pixel
    (BORDER_REPLICATE).  cv2 blends in fixed point (5-bit sub-pixel
    positions), this kernel in float32: uint8 outputs can differ from cv2's by
    one grey level at sub-pixel positions."""
    import ctypes as C

    from . import _native as N

    a = np.asarray(img)
    if a.ndim not in (2, 3) or (a.ndim == 3 and not 1 <= a.shape[2] <= 4):
        raise ValueError("img must have shape (h, w) or (h, w, c) with 1 <= c <= 4")
    if a.dtype == np.uint8:
        dtype = 0
    elif a.dtype in (np.float32, np.float64):
        a, dtype = a.astype(np.float32), 1
    else:
        raise ValueError(f"unsupported image dtype {a.dtype} (uint8 or float32)")
    if border_mode not in (BORDER_CONSTANT, BORDER_REPLICATE):
        raise ValueError("border_mode must be BORDER_CONSTANT (0) or BORDER_REPLICATE (1)")
    h, w = a.shape[:2]
    ch = 1 if a.ndim == 2 else a.shape[2]
    Ht, (ow, oh), mins = warp_geometry(h, w, H)
    M = np.ascontiguousarray(np.linalg.inv(Ht), dtype=np.float64)
    bv = np.zeros(4)
    vals = np.atleast_1d(np.asarray(border_value, dtype=np.float64))
    bv[:min(4, vals.size)] = vals[:4]
    if vals.size == 1:
        bv[:] = vals[0]
    src = np.ascontiguousarray(a)
    out = np.empty((oh, ow) if a.ndim == 2 else (oh, ow, ch), dtype=src.dtype)
    dp = C.POINTER(C.c_double)
    N.check(N.lib.gcr_warp_perspective(N.context(device), src.ctypes.data, h, w, ch, dtype, M.ctypes.data_as(dp),
                                       int(border_mode), bv.ctypes.data_as(dp), out.ctypes.data, oh, ow))
    return out, Ht, mins
