"""Feature front-end (pygcransac.features) against the reference's
examples/utils.py:5-49 semantics, restated literally here on cv2-style
keypoint objects."""
import numpy as np

from pygcransac import features as F


class KP:
    def __init__(self, x, y, size, angle):
        self.pt, self.size, self.angle = (x, y), size, angle


def _ref_scale(keypoints):                       # utils.py:5-26, verbatim logic
    unique_xys = {}
    for kp in keypoints:
        key = (int(kp.pt[0]), int(kp.pt[1]))
        if key not in unique_xys:
            unique_xys[key] = kp
    return np.array([[kp.pt[0], kp.pt[1], kp.size] for kp in unique_xys.values()])


def _ref_orient(keypoints):                      # utils.py:29-49, verbatim logic
    feats, sizes = [], []
    for kp in keypoints:
        if kp.angle != -1:
            feats.append([kp.pt[0], kp.pt[1], np.deg2rad(kp.angle)])
            sizes.append(0.5 * kp.size)
    return np.array(feats), np.array(sizes)


def _keypoints(seed=0, n=3000):
    rng = np.random.default_rng(seed)
    kps = []
    for _ in range(n):
        x, y = rng.uniform(-3, 400, size=2)
        if rng.random() < 0.3 and kps:           # SIFT repeats a location with other angles
            x, y = kps[int(rng.integers(len(kps)))].pt
        angle = -1.0 if rng.random() < 0.1 else float(rng.uniform(0, 360))
        kps.append(KP(float(x), float(y), float(rng.uniform(1, 30)), angle))
    return kps


def test_scale_features_match_reference_bitwise():
    kps = _keypoints()
    exp = _ref_scale(kps)
    assert np.array_equal(F.scale_features_from_sift(kps), exp)
    arr = np.array([[k.pt[0], k.pt[1], k.size, k.angle] for k in kps])
    assert np.array_equal(F.scale_features_from_sift(arr), exp)
    assert len(exp) < len(kps)                   # duplicates were removed


def test_orientation_features_match_reference_bitwise():
    kps = _keypoints(1)
    ef, es = _ref_orient(kps)
    gf, gs = F.orientation_features_from_sift(kps)
    assert np.array_equal(gf, ef) and np.array_equal(gs, es)
    assert len(ef) < len(kps)                    # angle == -1 dropped


def test_negative_coordinates_truncate_toward_zero():
    kps = [KP(-0.5, 2.2, 3.0, 10.0), KP(0.4, 2.9, 5.0, 20.0), KP(-1.2, 2.0, 7.0, 30.0)]
    out = F.scale_features_from_sift(kps)
    assert out.shape == (2, 3) and out[0, 2] == 3.0 and out[1, 2] == 7.0
