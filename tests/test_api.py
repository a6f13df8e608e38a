"""The Python surface of pygcransac mirrors bindings.cpp (no GPU needed: every
check here fires before the engine is called).

bindings.cpp:35-51 / 199-224 (ValueError texts), :315-399 (names, defaults),
:329-364 (model classes); pybind11 raises TypeError for arguments it cannot
convert."""
import inspect

import numpy as np
import pytest

import pygcransac as P

FUNCS = ("findRectifyingHomographyScaleOnly", "findRectifyingHomographyScaleOnlyOriginal",
         "findRectifyingHomographySIFT")


def test_module_exports_the_reference_surface():
    for name in FUNCS + ("NormalizingTransform", "RectifyingHomography", "ScaleBasedRectifyingHomography",
                         "OrientationBasedRectifyingHomography", "SIFTRectifyingHomography"):
        assert hasattr(P, name), name


@pytest.mark.parametrize("name", FUNCS)
def test_positional_signature_and_defaults(name):
    sig = inspect.signature(getattr(P, name))
    pos = [p for p in sig.parameters.values() if p.kind == p.POSITIONAL_OR_KEYWORD]
    tail = [(p.name, p.default) for p in pos[-4:]]
    assert tail == [("spatial_coherence_weight", 0.0), ("min_iteration_number", 10000),
                    ("max_iteration_number", 10000), ("max_local_optimization_number", 50)]
    # extensions are keyword-only, so positional calls mean what they meant
    kw = {p.name for p in sig.parameters.values() if p.kind == p.KEYWORD_ONLY}
    assert {"seed", "confidence", "device", "batch_slots", "return_stats"} <= kw


@pytest.mark.parametrize("original", [False, True])
def test_scale_only_shape_errors(original):
    fn = P.findRectifyingHomographyScaleOnlyOriginal if original else P.findRectifyingHomographyScaleOnly
    with pytest.raises(ValueError, match=r"^Number of dimensions must be 2\.$"):
        fn(np.zeros(9), 0.05)
    with pytest.raises(ValueError) as e:
        fn(np.zeros((2, 3)), 0.05)
    assert str(e.value) == ("Features should be an array with 3 columns and at least 3 rows. "
                            "It has 3 columns and 2 rows.")
    with pytest.raises(ValueError) as e:
        fn(np.zeros((10, 4)), 0.05)
    assert str(e.value) == ("Features should be an array with 3 columns and at least 3 rows. "
                            "It has 4 columns and 10 rows.")


def test_sift_shape_errors():
    ok = np.zeros((5, 3))
    with pytest.raises(ValueError, match=r"^Number of dimensions must be 2\.$"):
        P.findRectifyingHomographySIFT(ok, np.zeros(3), 0.05, 0.01)
    with pytest.raises(ValueError) as e:
        P.findRectifyingHomographySIFT(np.zeros((1, 3)), ok, 0.05, 0.01)
    assert str(e.value) == ("Scale features should be an array with 3 columns and at least 2 rows. "
                            "It has 3 columns and 1 rows.")
    with pytest.raises(ValueError) as e:
        P.findRectifyingHomographySIFT(ok, np.zeros((4, 2)), 0.05, 0.01)
    assert str(e.value) == ("Orientation features should be an array with 3 columns and at least 2 rows. "
                            "It has 2 columns and 4 rows.")


def test_unconvertible_arguments_raise_type_error():
    f = np.zeros((5, 3))
    with pytest.raises(TypeError):
        P.findRectifyingHomographyScaleOnly([["a", "b", "c"]] * 4, 0.05)
    with pytest.raises(TypeError):
        P.findRectifyingHomographyScaleOnly(f, "0.05")
    with pytest.raises(TypeError):
        P.findRectifyingHomographyScaleOnly(f, 0.05, 0.0, -1)          # size_t
    with pytest.raises(TypeError):
        P.findRectifyingHomographyScaleOnly(f, 0.05, 0.0, 10, 2.5)     # size_t


def test_model_classes_mirror_bindings():
    m = P.SIFTRectifyingHomography()
    assert isinstance(m, P.ScaleBasedRectifyingHomography)
    assert isinstance(m, P.OrientationBasedRectifyingHomography)
    assert isinstance(m, P.RectifyingHomography) and isinstance(m, P.NormalizingTransform)
    # default-constructible with read-write attributes (bindings.cpp:329-364)
    assert (m.x0, m.y0, m.s, m.h7, m.h8) == (0.0, 0.0, 1.0, 0.0, 0.0)
    m.h7, m.alpha, m.phi = 1e-4, 0.5, 0.25
    assert (m.h7, m.alpha, m.phi) == (1e-4, 0.5, 0.25)
    H = m.getHomography()
    assert H.shape == (3, 3) and H[2, 2] == 1.0 and H[2, 0] == 1e-4
    for meth in ("rectifiedScale", "unrectifiedScale", "rectifiedAngle", "unrectifiedAngle",
                 "rectifiedPoint", "unrectifiedPoint"):
        assert callable(getattr(m, meth))
