"""The C-ABI library loads and exports every entry point include/gcr.h declares
(no GPU compute is invoked here)."""
import ctypes as C
import os
import re

import numpy as np

from pygcransac import _native as N

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(REPO, "include", "gcr.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"\b(gcr_[a-z0-9_]+)\s*\(", src)
    return sorted(set(names))


def test_header_declares_the_drop_in_entry_points():
    names = _declared()
    for n in ("gcr_rect_scale_only", "gcr_rect_sift", "gcr_create", "gcr_destroy", "gcr_last_error",
              "gcr_problem_create", "gcr_problem_run", "gcr_problem_verify_batch"):
        assert n in names


def test_library_exports_every_declared_symbol():
    lib = C.CDLL(N.LIB_PATH)
    missing = [n for n in _declared() if not hasattr(lib, n)]
    assert not missing, missing


def test_abi_version_and_defaults():
    assert N.lib.gcr_abi_version() == 5          # 5: gcr_stats.chunk_msac_lists
    p = N.default_params()
    assert (p.min_iteration_number, p.max_iteration_number, p.max_local_optimization_number) == (10000, 10000, 50)
    assert p.spatial_coherence_weight == 0.0 and p.confidence == 0.95
    assert p.cell_number == 0 and list(p.cell_size) == [0.0] * 4      # the reference's empty grid
    # the ctypes mirror has the C struct's size (no silently misaligned fields)
    import re
    hdr = open(os.path.join(os.path.dirname(N.LIB_PATH), "..", "..", "include", "gcr.h")).read()
    body = hdr[hdr.index("typedef struct gcr_params {"):hdr.index("} gcr_params;")]
    fields = re.findall(r"^\s+(double|uint64_t|uint32_t) ([a-z_]+)(\[4\])?;", body, re.M)
    assert [f[1] for f in fields] == [f[0] for f in N.Params._fields_]


def test_errors_cross_the_abi_as_codes_not_exceptions():
    out = C.c_void_p()
    rc = N.lib.gcr_create(-1, C.byref(out))
    assert rc < 0 and N.last_error()
    p = N.default_params()
    rc = N.lib.gcr_problem_run(None, C.byref(p), None, None, None, None, None)
    assert rc == N.GCR_EINVAL


def test_kernel_build_id_is_the_source_hash():
    bid = N.lib.gcr_kernel_build_id().decode()
    assert len(bid) == 16 and int(bid, 16) >= 0


def test_host_hooks_need_no_gpu():
    assert N.lib.gcr_host_log(1.0) == 0.0
    assert N.lib.gcr_host_pow_m3(2.0) == 0.125
    out = (C.c_uint32 * 3)()
    assert N.lib.gcr_host_sample(1, 2, 3, 0, 0, 100, 3, out) == 0
    assert len(set(out)) == 3 and max(out) < 100
    H = np.zeros(9)
    m = N.RectModel(0.0, 0.0, 1.0, 1e-4, -2e-4, 0.5, 0.0)
    N.lib.gcr_host_homography(C.byref(m), H.ctypes.data_as(C.POINTER(C.c_double)))
    assert np.array_equal(H.reshape(3, 3), [[1, 0, 0], [0, 1, 0], [1e-4, -2e-4, 1]])
