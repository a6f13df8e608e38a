"""Feature front-end (pygcransac.features) against the reference's
examples/utils.py:5-49 semantics, restated literally here on cv2-style
keypoint objects."""
import numpy as np
import pytest

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


# ------------------------------------------------------ perspective_warp ----
# examples/utils.py:92-123.  The frame geometry is host numpy (CPU tests); the
# resampling is the HIP kernel behind gcr_warp_perspective (GPU tests), checked
# against an analytic warp and a numpy bilinear restatement.
def test_warp_geometry_translation_and_scale():
    from pygcransac.features import warp_geometry

    Ht, size, mins = warp_geometry(40, 60, [[1, 0, 5.5], [0, 1, -7], [0, 0, 1]])
    assert size == (60, 40) and mins == (5.5, -7.0)
    assert np.allclose(Ht, np.eye(3))
    Ht, size, mins = warp_geometry(40, 60, np.diag([2.0, 0.5, 1.0]))
    assert size == (120, 20) and mins == (0.0, 0.0)
    # a projective warp: every corner lands inside the translated frame
    H = np.array([[1.0, 0.1, 3.0], [0.05, 0.9, 2.0], [1e-3, 2e-4, 1.0]])
    Ht, (ow, oh), (mx, my) = warp_geometry(100, 150, H)
    c = Ht @ np.array([[0, 0, 1], [150, 0, 1], [150, 100, 1], [0, 100, 1]]).T
    c = c[:2] / c[2]
    assert np.all(c > -1e-9) and np.all(c[0] <= ow + 1e-9) and np.all(c[1] <= oh + 1e-9)
    assert np.isclose(c[0].min(), 0.0, atol=1e-9) and np.isclose(c[1].min(), 0.0, atol=1e-9)


def _bilinear_ref(img, M, oh, ow, border_mode, border):
    """numpy restatement of the kernel's sampling rule (float64)."""
    img = np.asarray(img, dtype=np.float64)
    if img.ndim == 2:
        img = img[:, :, None]
    h, w, ch = img.shape
    ys, xs = np.mgrid[0:oh, 0:ow].astype(np.float64)
    wz = M[2, 0] * xs + M[2, 1] * ys + M[2, 2]
    sx = (M[0, 0] * xs + M[0, 1] * ys + M[0, 2]) / wz
    sy = (M[1, 0] * xs + M[1, 1] * ys + M[1, 2]) / wz
    x0, y0 = np.floor(sx).astype(np.int64), np.floor(sy).astype(np.int64)
    ax, ay = (sx - x0)[..., None], (sy - y0)[..., None]

    def tex(x, y):
        inside = (x >= 0) & (y >= 0) & (x < w) & (y < h)
        v = img[np.clip(y, 0, h - 1), np.clip(x, 0, w - 1)]
        if border_mode == 0:
            v = np.where(inside[..., None], v, np.asarray(border[:ch], dtype=np.float64))
        return v

    p00, p01, p10, p11 = tex(x0, y0), tex(x0 + 1, y0), tex(x0, y0 + 1), tex(x0 + 1, y0 + 1)
    top = p00 + ax * (p01 - p00)
    bot = p10 + ax * (p11 - p10)
    return top + ay * (bot - top)


@pytest.mark.gpu
def test_perspective_warp_integer_shift_is_exact():
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (37, 53, 3), dtype=np.uint8)
    out, Ht, mins = F.perspective_warp(img, [[1, 0, 4], [0, 1, -9], [0, 0, 1]])
    assert out.shape == img.shape and mins == (4.0, -9.0) and np.allclose(Ht, np.eye(3))
    assert np.array_equal(out, img)          # zero bilinear weights on every neighbour but the pixel


@pytest.mark.gpu
def test_perspective_warp_reproduces_an_analytic_linear_image():
    h, w = 90, 120
    ys, xs = np.mgrid[0:h, 0:w].astype(np.float64)
    img = (0.75 * xs - 0.5 * ys + 3.0).astype(np.float32)
    H = np.array([[0.9, 0.2, 10.0], [-0.1, 1.1, 5.0], [2e-4, -1e-4, 1.0]])
    out, Ht, _ = F.perspective_warp(img, H, border_mode=F.BORDER_REPLICATE)
    M = np.linalg.inv(Ht)
    oh, ow = out.shape
    yy, xx = np.mgrid[0:oh, 0:ow].astype(np.float64)
    wz = M[2, 0] * xx + M[2, 1] * yy + M[2, 2]
    sx = (M[0, 0] * xx + M[0, 1] * yy + M[0, 2]) / wz
    sy = (M[1, 0] * xx + M[1, 1] * yy + M[1, 2]) / wz
    interior = (sx >= 0) & (sy >= 0) & (sx <= w - 1) & (sy <= h - 1)
    assert interior.mean() > 0.5
    expect = 0.75 * sx - 0.5 * sy + 3.0          # bilinear sampling of a linear image is exact
    assert np.max(np.abs(out[interior] - expect[interior])) < 1e-3


@pytest.mark.gpu
@pytest.mark.parametrize("border_mode", [0, 1])
def test_perspective_warp_matches_bilinear_restatement(border_mode):
    rng = np.random.default_rng(11 + border_mode)
    img = rng.integers(0, 256, (64, 80, 3), dtype=np.uint8)
    H = np.array([[1.05, 0.12, -4.0], [-0.08, 0.97, 6.0], [3e-4, 1e-4, 1.0]])
    border = (255, 128, 7)
    out, Ht, _ = F.perspective_warp(img, H, border_mode=border_mode, border_value=border)
    ref = _bilinear_ref(img, np.linalg.inv(Ht), out.shape[0], out.shape[1], border_mode, border)
    diff = np.abs(out.astype(np.int64) - np.clip(np.rint(ref), 0, 255).astype(np.int64))
    assert diff.max() <= 1 and (diff == 0).mean() > 0.99       # float32 blend vs float64 restatement
    gray = rng.random((30, 40)).astype(np.float32)
    outg, Htg, _ = F.perspective_warp(gray, H, border_mode=border_mode, border_value=0.5)
    refg = _bilinear_ref(gray, np.linalg.inv(Htg), outg.shape[0], outg.shape[1], border_mode, (0.5,) * 4)[..., 0]
    assert outg.dtype == np.float32 and np.max(np.abs(outg - refg)) < 1e-5


def test_perspective_warp_rejects_bad_inputs():
    with pytest.raises(ValueError):
        F.perspective_warp(np.zeros((4, 4, 5), np.uint8), np.eye(3))
    with pytest.raises(ValueError):
        F.perspective_warp(np.zeros((4, 4), np.int32), np.eye(3))
    with pytest.raises(ValueError):
        F.perspective_warp(np.zeros((4, 4), np.uint8), np.eye(3), border_mode=4)
