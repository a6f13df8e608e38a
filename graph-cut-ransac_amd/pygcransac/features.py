"""Feature front-end: SIFT keypoints -> the estimator's input arrays
(examples/utils.py:5-49 of the reference).

The reference takes cv2.KeyPoint lists.  cv2 is optional here: any object
with .pt, .size and .angle works, and so does an (N, 4) array of
(x, y, size, angle_degrees) rows (angle -1 = none, OpenCV's convention).
"""
from __future__ import annotations

import numpy as np

__all__ = ["scale_features_from_sift", "orientation_features_from_sift", "keypoints_to_array"]


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
