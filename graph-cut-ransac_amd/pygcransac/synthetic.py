"""Synthetic rectification problems (inputs M1 / M2).

The reference's example notebook and its SIFT features are not in the snapshot
(``.MISSING_LARGE_BLOBS:1``) and cv2 is absent, so benchmarks and tests use
seeded synthetic features with a known rectifying homography instead.

Feature conventions follow ``examples/utils.py:5-49`` of the reference:
scale features are rows ``(x, y, size)``, orientation features rows
``(x, y, angle_rad)``.  Ground truth uses the reference's own model maths
(``model.h:122-204``): an inlier scale feature satisfies
``alpha^3 * s * (1 - h7 x - h8 y)^-3 = exp(eps)``; an inlier orientation
feature rectifies (``rectifiedAngle``) to ``phi`` or ``phi + pi/2`` plus noise.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

WIDTH, HEIGHT = 1368.0, 1824.0          # examples/img/tiled_floor_001.jpg
DEFAULT_SEED = 20251121


@dataclass
class GroundTruth:
    h7: float = 2.0e-4
    h8: float = -1.5e-4
    alpha: float = 0.5
    phi: float = 0.35


def _unrectified_angle(h7, h8, x, y, angle):
    # model.h:167-174 (glibc cos/sin/atan2 via Python's math module)
    ct, st = math.cos(angle), math.sin(angle)
    numer = (x * st - y * ct) * h7 + st
    denom = (-x * st + y * ct) * h8 + ct
    a = math.fmod(math.atan2(numer, denom), 2.0 * math.pi)
    return a + 2.0 * math.pi if a < 0.0 else a


def scale_features(n: int, outlier_ratio: float = 0.5, seed: int = DEFAULT_SEED,
                   gt: GroundTruth = GroundTruth(), noise: float = 0.02, width: float = WIDTH,
                   height: float = HEIGHT):
    """M1: n scale features (x, y, s); returns (features[n,3], inlier_mask)."""
    rng = np.random.default_rng(seed)
    n_out = int(round(n * outlier_ratio))
    n_in = n - n_out
    x = rng.uniform(0.0, width, n)
    y = rng.uniform(0.0, height, n)
    t = 1.0 - gt.h7 * x[:n_in] - gt.h8 * y[:n_in]
    s_in = (t / gt.alpha) ** 3 * np.exp(rng.normal(0.0, noise, n_in))
    s_out = np.exp(rng.uniform(math.log(2.0), math.log(64.0), n_out))
    s = np.concatenate([s_in, s_out])
    truth = np.zeros(n, dtype=bool)
    truth[:n_in] = True
    perm = rng.permutation(n)
    feats = np.stack([x, y, s], axis=1)[perm]
    return np.ascontiguousarray(feats), truth[perm]


def orientation_features(n: int, outlier_ratio: float = 0.5, seed: int = DEFAULT_SEED + 1,
                         gt: GroundTruth = GroundTruth(), noise_deg: float = 0.5, width: float = WIDTH,
                         height: float = HEIGHT):
    """M2 orientation part: n features (x, y, angle); returns (features, inlier_mask)."""
    rng = np.random.default_rng(seed)
    n_out = int(round(n * outlier_ratio))
    n_in = n - n_out
    x = rng.uniform(0.0, width, n)
    y = rng.uniform(0.0, height, n)
    theta = np.empty(n)
    which = rng.integers(0, 2, n_in)
    noise = np.deg2rad(rng.normal(0.0, noise_deg, n_in))
    for i in range(n_in):
        w = 1.0 - gt.h7 * x[i] - gt.h8 * y[i]          # rectifyPoint
        u, v = x[i] / w, y[i] / w
        tr = gt.phi + (math.pi / 2.0) * which[i] + noise[i]
        theta[i] = _unrectified_angle(gt.h7, gt.h8, u, v, tr)
    theta[n_in:] = rng.uniform(0.0, 2.0 * math.pi, n_out)
    truth = np.zeros(n, dtype=bool)
    truth[:n_in] = True
    perm = rng.permutation(n)
    feats = np.stack([x, y, theta], axis=1)[perm]
    return np.ascontiguousarray(feats), truth[perm]


def problem_m1(n: int = 10_000, outlier_ratio: float = 0.5, seed: int = DEFAULT_SEED):
    """Scale-only problem (3-SIFT): features, truth mask, thresholds."""
    f, t = scale_features(n, outlier_ratio, seed)
    return f, t, 0.05


def problem_m2(n_scale: int = 5_000, n_orient: int = 5_000, outlier_ratio: float = 0.5,
               seed: int = DEFAULT_SEED):
    """Hybrid problem (2+2 SIFT): scale feats, orientation feats, truths, thresholds."""
    fs, ts = scale_features(n_scale, outlier_ratio, seed)
    fo, to = orientation_features(n_orient, outlier_ratio, seed + 1)
    return fs, fo, ts, to, 0.05, math.radians(1.0)


# ------------------------------------------------------------ homography ----
# BASELINE configs[2]: N = 5 000 correspondences, 50 % outliers.  Two views of
# a plane: inliers are image-1 points mapped by a ground-truth homography plus
# Gaussian pixel noise; outliers are independent uniform pairs.
H_GT = np.array([[0.92, -0.08, 35.0],
                 [0.06, 0.97, -18.0],
                 [4.0e-5, -3.0e-5, 1.0]])
IMG_W, IMG_H = 1280.0, 960.0


def problem_h(n: int = 5_000, outlier_ratio: float = 0.5, seed: int = DEFAULT_SEED, noise: float = 0.5,
              H: np.ndarray = H_GT):
    """Homography problem: correspondences (n, 4) = (x1, y1, x2, y2), inlier
    truth mask, ground-truth H and the inlier threshold (px)."""
    rng = np.random.default_rng(seed)
    n_out = int(round(n * outlier_ratio))
    n_in = n - n_out
    x1 = rng.uniform(0, IMG_W, n_in)
    y1 = rng.uniform(0, IMG_H, n_in)
    w = H[2, 0] * x1 + H[2, 1] * y1 + H[2, 2]
    x2 = (H[0, 0] * x1 + H[0, 1] * y1 + H[0, 2]) / w + rng.normal(0, noise, n_in)
    y2 = (H[1, 0] * x1 + H[1, 1] * y1 + H[1, 2]) / w + rng.normal(0, noise, n_in)
    inl = np.stack([x1, y1, x2, y2], axis=1)
    out = np.stack([rng.uniform(0, IMG_W, n_out), rng.uniform(0, IMG_H, n_out),
                    rng.uniform(0, IMG_W, n_out), rng.uniform(0, IMG_H, n_out)], axis=1)
    corr = np.concatenate([inl, out])
    truth = np.concatenate([np.ones(n_in, bool), np.zeros(n_out, bool)])
    perm = rng.permutation(n)
    return np.ascontiguousarray(corr[perm]), truth[perm], H.copy(), 2.0


def _rot(yaw, pitch, roll):
    cy, sy, cp, sp, cr, sr = (math.cos(yaw), math.sin(yaw), math.cos(pitch), math.sin(pitch), math.cos(roll),
                              math.sin(roll))
    Ry = np.array([[cy, 0, sy], [0, 1, 0], [-sy, 0, cy]])
    Rx = np.array([[1, 0, 0], [0, cp, -sp], [0, sp, cp]])
    Rz = np.array([[cr, -sr, 0], [sr, cr, 0], [0, 0, 1]])
    return Rz @ Rx @ Ry


def two_view_geometry(focal: float = 1000.0, yaw: float = 0.12, pitch: float = 0.03, roll: float = 0.02,
                      t=(1.0, 0.1, 0.15)):
    """Calibration, relative pose and F_gt (x2^T F x1 = 0, unit Frobenius norm)."""
    K = np.array([[focal, 0, IMG_W / 2], [0, focal, IMG_H / 2], [0, 0, 1.0]])
    R = _rot(yaw, pitch, roll)
    t = np.asarray(t, dtype=float)
    tx = np.array([[0, -t[2], t[1]], [t[2], 0, -t[0]], [-t[1], t[0], 0]])
    Ki = np.linalg.inv(K)
    F = Ki.T @ tx @ R @ Ki
    return K, R, t, F / np.linalg.norm(F)


def problem_f(n: int = 10_000, outlier_ratio: float = 0.8, seed: int = DEFAULT_SEED, noise: float = 0.5):
    """Fundamental-matrix problem (BASELINE configs[3]): a random 3-D scene seen
    by two calibrated cameras.  Returns correspondences (n, 4) = (x1, y1, x2,
    y2), inlier truth mask, F_gt and the inlier threshold (px, Sampson)."""
    rng = np.random.default_rng(seed)
    K, R, t, F = two_view_geometry()
    n_out = int(round(n * outlier_ratio))
    n_in = n - n_out
    pts = []
    while sum(len(p) for p in pts) < n_in:
        m = 2 * n_in
        X = np.stack([rng.uniform(-5, 5, m), rng.uniform(-4, 4, m), rng.uniform(6, 16, m)], axis=1)
        p1 = X @ K.T
        X2 = X @ R.T + t
        p2 = X2 @ K.T
        ok = (X2[:, 2] > 0.1)
        u1, v1 = p1[:, 0] / p1[:, 2], p1[:, 1] / p1[:, 2]
        u2, v2 = p2[:, 0] / p2[:, 2], p2[:, 1] / p2[:, 2]
        ok &= (u1 >= 0) & (u1 < IMG_W) & (v1 >= 0) & (v1 < IMG_H) & (u2 >= 0) & (u2 < IMG_W) & (v2 >= 0) & (v2 < IMG_H)
        pts.append(np.stack([u1, v1, u2, v2], axis=1)[ok])
    inl = np.concatenate(pts)[:n_in]
    inl = inl + rng.normal(0, noise, inl.shape)
    out = np.stack([rng.uniform(0, IMG_W, n_out), rng.uniform(0, IMG_H, n_out),
                    rng.uniform(0, IMG_W, n_out), rng.uniform(0, IMG_H, n_out)], axis=1)
    corr = np.concatenate([inl, out])
    truth = np.concatenate([np.ones(n_in, bool), np.zeros(n_out, bool)])
    perm = rng.permutation(n)
    return np.ascontiguousarray(corr[perm]), truth[perm], F, 1.0
