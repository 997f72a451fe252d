"""The C ABI library: loads without a GPU, exports every symbol the header
declares, and its host-side validation returns the documented status codes
(no compute calls here -- those are the -m gpu tests)."""
import ctypes

import pytest

from bpc_baseline_amd import _native


@pytest.fixture(scope="module")
def lib():
    return _native.load()


def test_header_symbols_exported(lib):
    names = _native.header_symbols()
    assert len(names) >= 8
    for n in names:
        assert hasattr(lib, n), f"{n} declared in include/mvmatch.h but not exported"
    assert set(names) == set(_native.SIGNATURES), "ctypes signature table out of sync with header"


def test_version_and_status_strings(lib):
    assert _native.version().startswith("mvmatch ")
    assert "gfx950" in _native.version()
    assert lib.mvm_status_string(0) == b"ok"
    assert lib.mvm_status_string(3) == b"workspace too small"


def _pairs(*ab):
    n = len(ab)
    return (ctypes.c_int32 * n)(*[a for a, _ in ab]), (ctypes.c_int32 * n)(*[b for _, b in ab])


FAKE = ctypes.c_void_p(0x1000)   # never dereferenced: validation fails first


def test_unsupported_camera_count(lib):
    pa, pb = _pairs((0, 1))
    st = lib.mvm_pairwise_residual_argmin(FAKE, FAKE, FAKE, pa, pb, 1, 99, 1, 4,
                                          FAKE, FAKE, FAKE, FAKE, FAKE, None)
    assert st == 2
    assert b"n_cams" in lib.mvm_last_error_string()


def test_bad_pair_index(lib):
    pa, pb = _pairs((0, 3))
    st = lib.mvm_pairwise_residual_argmin(FAKE, FAKE, FAKE, pa, pb, 1, 3, 1, 4,
                                          FAKE, FAKE, FAKE, FAKE, FAKE, None)
    assert st == 1
    pa, pb = _pairs((1, 1))
    assert lib.mvm_pairwise_residual_argmin(FAKE, FAKE, FAKE, pa, pb, 1, 3, 1, 4,
                                            FAKE, FAKE, FAKE, FAKE, FAKE, None) == 1


def test_outputs_need_offsets(lib):
    pa, pb = _pairs((0, 1))
    st = lib.mvm_pairwise_residual_argmin(FAKE, FAKE, FAKE, pa, pb, 1, 2, 1, 4,
                                          None, FAKE, FAKE, None, None, None)
    assert st == 1 and b"dist_offs" in lib.mvm_last_error_string()
    st = lib.mvm_pairwise_residual_argmin(FAKE, FAKE, FAKE, pa, pb, 1, 2, 1, 4,
                                          FAKE, None, None, FAKE, None, None)
    assert st == 1 and b"row_offs" in lib.mvm_last_error_string()


def test_empty_batch_is_a_noop(lib):
    pa, pb = _pairs((0, 1))
    # zero scenes / zero detections: nothing is launched, status ok
    assert lib.mvm_pairwise_residual_argmin(None, None, None, pa, pb, 0, 2, 1, 0,
                                            None, None, None, None, None, None) == 0
    assert lib.mvm_triplet_cost_argmin(None, None, None, 0, 0, None, None, None, None, None,
                                       None, 0, None) == 0


def test_triplet_workspace_contract(lib):
    need = lib.mvm_triplet_workspace_bytes(10, 30)
    assert need == 10 * 3 * 30 * 32 * 8          # ld rounded up to a multiple of 4
    assert lib.mvm_triplet_workspace_bytes(0, 30) == 0
    st = lib.mvm_triplet_cost_argmin(FAKE, FAKE, FAKE, 10, 30, FAKE, FAKE, FAKE, FAKE, FAKE,
                                     FAKE, need - 16, None)
    assert st == 3
    st = lib.mvm_triplet_cost_argmin(FAKE, FAKE, FAKE, 10, 30, FAKE, FAKE, FAKE, FAKE, FAKE,
                                     ctypes.c_void_p(0x1004), need, None)
    assert st == 1   # misaligned workspace


def test_write_probe_validation(lib):
    assert lib.mvm_hbm_write_probe(None, 1024, None) == 1
    assert lib.mvm_hbm_write_probe(FAKE, 1000, None) == 1


def test_check_raises(lib):
    with pytest.raises(_native.MvmError):
        pa, pb = _pairs((0, 1))
        st = lib.mvm_pairwise_residual_argmin(FAKE, FAKE, FAKE, pa, pb, 1, 99, 1, 4,
                                              FAKE, FAKE, FAKE, FAKE, FAKE, None)
        _native.check("mvm_pairwise_residual_argmin", st)


def test_pack_detections_validation(lib):
    f = ctypes.c_float
    # no images: nothing launched; negative count and missing offsets refused
    assert lib.mvm_pack_detections(None, None, None, None, 0, f(0.1), f(0.0), None, None, None,
                                   None, None, None) == 0
    assert lib.mvm_pack_detections(None, None, None, FAKE, -1, f(0.1), f(0.0), FAKE, FAKE, None,
                                   None, FAKE, None) == 1
    assert lib.mvm_pack_detections(FAKE, FAKE, FAKE, None, 3, f(0.1), f(0.0), FAKE, FAKE, FAKE,
                                   FAKE, FAKE, None) == 1


def test_triangulate_dlt_validation(lib):
    assert lib.mvm_triangulate_dlt(None, None, None, 0, 3, None, None) == 0
    assert lib.mvm_triangulate_dlt(FAKE, None, FAKE, 5, 1, FAKE, None) == 1      # one view
    assert lib.mvm_triangulate_dlt(FAKE, None, FAKE, 5, 9, FAKE, None) == 1      # > MVM_MAX_CAMS
    assert b"n_views" in lib.mvm_last_error_string()
    assert lib.mvm_triangulate_dlt(None, None, FAKE, 5, 3, FAKE, None) == 1


def test_library_reads_no_environment():
    """The ABI has no hidden global state: kernel-path choices come only from
    mvm_options (include/mvmatch.h), so the library imports no getenv."""
    with open(_native.LIB_PATH, "rb") as fh:
        blob = fh.read()
    assert b"getenv\x00" not in blob      # no imported getenv / secure_getenv symbol name


def test_grid_beyond_the_dispatch_limit(lib):
    """A dispatch packet counts work-items in 32 bits: a pairwise batch of
    more than 2^32 / 256 workgroups is refused, not launched truncated
    (2,000,000 scenes x 28 pairs x 4 row blocks = 224M workgroups)."""
    pa, pb = _pairs(*[(a, b) for a in range(8) for b in range(a + 1, 8)])
    st = lib.mvm_pairwise_residual_argmin_ex(FAKE, FAKE, FAKE, pa, pb, 2_000_000, 8, 28, 1024, FAKE,
                                             FAKE, FAKE, FAKE, FAKE, None, None)
    assert st == 2 and b"split the scenes" in lib.mvm_last_error_string()
    st = lib.mvm_lsap_solve_ex(FAKE, 0, FAKE, FAKE, 5_000_000, FAKE, FAKE, FAKE, 1 << 20, FAKE, FAKE,
                               FAKE, 1, 1, None, None)
    assert st == 2 and b"split it" in lib.mvm_last_error_string()


def test_options_init_and_validation(lib):
    o = _native.MvmOptions()
    lib.mvm_options_init(ctypes.byref(o))
    assert o.size == ctypes.sizeof(_native.MvmOptions)
    assert all(getattr(o, n) == 0 for n in _native.OPTION_FIELDS)
    pa, pb = _pairs((0, 1))
    bad = _native.make_options(pairwise_rows_per_wave=5)
    st = lib.mvm_pairwise_residual_argmin_ex(FAKE, FAKE, FAKE, pa, pb, 1, 2, 1, 4, FAKE, FAKE,
                                             FAKE, FAKE, FAKE, ctypes.byref(bad), None)
    assert st == 1 and b"rows_per_wave" in lib.mvm_last_error_string()
    bad = _native.make_options(pairwise_xcd_fronts=17)
    st = lib.mvm_pairwise_residual_argmin_ex(FAKE, FAKE, FAKE, pa, pb, 1, 2, 1, 4, FAKE, FAKE,
                                             FAKE, FAKE, FAKE, ctypes.byref(bad), None)
    assert st == 1 and b"pairwise_xcd_fronts" in lib.mvm_last_error_string()
    bad = _native.make_options(cube_kernel=9)
    st = lib.mvm_triplet_cost_argmin_ex(FAKE, FAKE, FAKE, 1, 4, FAKE, FAKE, FAKE, FAKE, FAKE,
                                        FAKE, 1 << 20, ctypes.byref(bad), None)
    assert st == 1 and b"cube_kernel" in lib.mvm_last_error_string()
    bad = _native.make_options(cube_cols_per_lane=9)
    st = lib.mvm_triplet_cost_argmin_ex(FAKE, FAKE, FAKE, 1, 4, FAKE, FAKE, FAKE, FAKE, FAKE,
                                        FAKE, 1 << 20, ctypes.byref(bad), None)
    assert st == 1 and b"cube_cols_per_lane" in lib.mvm_last_error_string()
    # 3 k per lane forced on a view wider than 3 x 64 at one row per instruction
    bad = _native.make_options(cube_kernel="fused", cube_rows_per_instr=1, cube_cols_per_lane=3)
    st = lib.mvm_triplet_cost_argmin_ex(FAKE, FAKE, FAKE, 1, 200, FAKE, FAKE, FAKE, FAKE, FAKE,
                                        FAKE, 1 << 20, ctypes.byref(bad), None)
    assert st == 1 and b"exceed 192" in lib.mvm_last_error_string()
    # ... with four rows per instruction forced on a view of 60 (> 48), and on
    # the k-chunked kernel's views (> 256)
    bad = _native.make_options(cube_kernel="fused", cube_rows_per_instr=4, cube_cols_per_lane=3)
    st = lib.mvm_triplet_cost_argmin_ex(FAKE, FAKE, FAKE, 1, 60, FAKE, FAKE, FAKE, FAKE, FAKE,
                                        FAKE, 1 << 20, ctypes.byref(bad), None)
    assert st == 1 and b"exceed 48" in lib.mvm_last_error_string()
    bad = _native.make_options(cube_cols_per_lane=3)
    st = lib.mvm_triplet_cost_argmin_ex(FAKE, FAKE, FAKE, 1, 300, FAKE, FAKE, FAKE, FAKE, FAKE,
                                        FAKE, 1 << 30, ctypes.byref(bad), None)
    assert st == 1 and b"k-chunked" in lib.mvm_last_error_string()
    bad = _native.make_options(cube_cols_per_lane=5)        # 5 k x 32 lanes < 200
    st = lib.mvm_triplet_cost_argmin_ex(FAKE, FAKE, FAKE, 1, 200, FAKE, FAKE, FAKE, FAKE, FAKE,
                                        FAKE, 1 << 20, ctypes.byref(bad), None)
    assert st == 1 and b"no 2 or 4 rows" in lib.mvm_last_error_string()
    bad = _native.make_options(cube_tile_rows=24)
    st = lib.mvm_triplet_cost_argmin_ex(FAKE, FAKE, FAKE, 1, 4, FAKE, FAKE, FAKE, FAKE, FAKE,
                                        FAKE, 1 << 20, ctypes.byref(bad), None)
    assert st == 1 and b"cube_tile_rows" in lib.mvm_last_error_string()
    o.size = 3                                      # not a struct size
    st = lib.mvm_triplet_cost_argmin_ex(FAKE, FAKE, FAKE, 1, 4, FAKE, FAKE, FAKE, FAKE, FAKE,
                                        FAKE, 1 << 20, ctypes.byref(o), None)
    assert st == 1 and b"size" in lib.mvm_last_error_string()
    with pytest.raises(ValueError):
        _native.make_options(no_such_field=1)


def test_lsap_plan_dtype(lib):
    import numpy as np
    rows, cols = np.array([300, 4], np.int64), np.array([20, 9], np.int64)
    w32, w64 = np.zeros(3, np.int64), np.zeros(3, np.int64)
    o = np.zeros(3, np.int64)
    t32 = lib.mvm_lsap_plan_ex(2, rows.ctypes.data, cols.ctypes.data, _native.MVM_F32,
                               w32.ctypes.data, o.ctypes.data)
    t64 = lib.mvm_lsap_plan_ex(2, rows.ctypes.data, cols.ctypes.data, _native.MVM_F64,
                               w64.ctypes.data, o.ctypes.data)
    # the tall 300 x 20 problem keeps a transposed copy of its costs: 4 more bytes each
    assert t64 - t32 >= 300 * 20 * 4
    assert lib.mvm_lsap_plan_ex(2, rows.ctypes.data, cols.ctypes.data, 7, w32.ctypes.data,
                                o.ctypes.data) == -1


# ---- the cube-free association (ABI 7) ----------------------------------------
def test_cube_free_class_bounds_and_scenes(lib):
    import numpy as np
    from bpc_baseline_amd import ops
    assert ops.sparse_class_bounds() == (4096, 65536, 1024)
    counts = np.array([[256, 256, 256],    # 65536 x 256: the class
                       [64, 64, 64],       # 4096 x 64: its lower edge
                       [63, 64, 64],       # 4032: below it (the dense classes read a cube)
                       [0, 100, 100],      # empty: nothing to read
                       [100, 100, 0],
                       [300, 20, 40],      # a view of more than 256: no minima kernel
                       [256, 256, 1]])     # one column
    assert ops.cube_free_scenes(counts).tolist() == [True, True, False, True, True, False, True]
    assert ops.cube_free_scenes(counts, min_cols=2048).tolist() == [True, True, True, True, True,
                                                                     False, True]


def test_lsap_plan_resid_sizes(lib):
    import numpy as np
    rows = np.array([65536, 4096, 600, 0, 24], np.int64)
    cols = np.array([256, 64, 40, 10, 576], np.int64)
    ws = np.zeros(6, np.int64)
    out = np.zeros(6, np.int64)
    total = lib.mvm_lsap_plan_resid(5, rows.ctypes.data, cols.ctypes.data, ws.ctypes.data, out.ctypes.data)
    assert total == ws[-1] > 0
    assert out.tolist() == [0, 256, 320, 360, 360, 384]
    sizes = np.diff(ws)
    assert sizes[3] == 0                              # an empty problem reserves nothing
    # a 256^3 scene: its candidate lists only (the block minima come from
    # mvm_triplet_minima; no transposed cost)
    assert 2e5 < sizes[0] < 4e5
    # the dense plan reserves the transposed cost for the same problem
    ws2 = np.zeros(6, np.int64)
    lib.mvm_lsap_plan_ex(5, rows.ctypes.data, cols.ctypes.data, 0, ws2.ctypes.data, out.ctypes.data)
    assert np.diff(ws2)[0] > 60e6
    # a wide problem reserves ceil(L/32) block keys per row, not L
    assert sizes[4] < 24 * 576 * 4
    assert lib.mvm_lsap_plan_resid(-1, None, None, None, None) == -1
    assert lib.mvm_lsap_sparse_stats_offset(65536, 256) == 0


def test_lsap_solve_resid_validation(lib):
    """Host bounds that are not all of the candidate-list class are refused
    before anything is launched (there is no cost for another class to read)."""
    def call(long_min, long_max, short_max, max_n=256, n=3):
        return lib.mvm_lsap_solve_resid(FAKE, n, FAKE, FAKE, FAKE, 1 << 20, FAKE, FAKE, FAKE,
                                        long_min, long_max, short_max, FAKE, FAKE, FAKE, FAKE, FAKE, FAKE,
                                        max_n, None, None)
    assert call(600, 65536, 256) == 1
    assert b"candidate-list class" in lib.mvm_last_error_string()
    assert call(4096, 70000, 256) == 1
    assert call(4096, 65536, 2000) == 1
    assert call(4096, 65536, 256, max_n=300) == 2          # views of more than 256
    assert call(4096, 65536, 256, n=0) == 0                # nothing to solve
    assert lib.mvm_lsap_solve_resid(None, 3, FAKE, FAKE, FAKE, 0, FAKE, FAKE, FAKE, 4096, 65536, 256,
                                    FAKE, FAKE, FAKE, FAKE, FAKE, FAKE, 256, None, None) == 1


def test_triplet_minima_validation(lib):
    need = lib.mvm_triplet_workspace_bytes(10, 200)
    args = lambda max_n, nbytes, resid=FAKE: (FAKE, FAKE, FAKE, 10, max_n, FAKE, FAKE, FAKE, FAKE, resid,
                                              nbytes, None, None)
    assert lib.mvm_triplet_minima(*args(300, 1 << 40)) == 2          # views of more than 256
    assert lib.mvm_triplet_minima(*args(200, need - 8)) == 3         # workspace too small
    assert lib.mvm_triplet_minima(*args(200, need, ctypes.c_void_p(0x1008))) == 1   # misaligned
    assert lib.mvm_triplet_minima(*args(200, need, None)) == 1       # null pointer
    assert lib.mvm_triplet_minima(None, None, None, 0, 0, None, None, None, None, None, 0, None, None) == 0
    assert lib.mvm_triplet_minima(FAKE, FAKE, FAKE, 10, 200, FAKE, FAKE, ctypes.c_void_p(0x1004), FAKE,
                                  FAKE, need, None, None) == 1      # misaligned block minima
    assert lib.mvm_triplet_minima(FAKE, FAKE, FAKE, 10, 200, FAKE, None, FAKE, FAKE,
                                  FAKE, need, None, None) == 1      # 8-row minima without offsets
    assert lib.mvm_select_triangulate_resid(None, 10, FAKE, FAKE, FAKE, FAKE, FAKE, FAKE, 3, 30.0,
                                            FAKE, FAKE, FAKE, FAKE, None) == 1
