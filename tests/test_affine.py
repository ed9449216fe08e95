"""extract_affine_square_region (row f4; AKB_raytrace_20250312.py:1047-1119). PARITY UNPINNED: the
reference calls OpenCV, which is absent here and holds no recorded output of this function. The
product (host C + device warp) is checked bit for bit against the oracle's independent
restatement (oracle/affine.py) and both against closed-form cases."""
import numpy as np
import pytest
import torch

import oracle.affine as OA


def _blobs(seed, shape=(48, 56)):
    """masks with several components, holes, components inside holes, edge-touching regions,
    single pixels and one-pixel-wide lines"""
    rng = np.random.default_rng(seed)
    m = np.zeros(shape, np.uint8)
    for _ in range(6):
        y0, x0 = rng.integers(0, shape[0] - 4), rng.integers(0, shape[1] - 4)
        h, w = rng.integers(1, 20), rng.integers(1, 20)
        m[y0:y0 + h, x0:x0 + w] = 255
    for _ in range(3):  # holes
        y0, x0 = rng.integers(0, shape[0] - 2), rng.integers(0, shape[1] - 2)
        m[y0:y0 + rng.integers(1, 6), x0:x0 + rng.integers(1, 6)] = 0
    m[rng.integers(0, shape[0]), rng.integers(0, shape[1])] = 255  # maybe a lone pixel
    return m


def _parallelogram(n, angle_deg, shear=0.0, pad=6, seed=0):
    """a NaN-surrounded map whose valid region is a rotated / sheared square (the pupil shapes the
    reference cuts out), values smooth with noise"""
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:n, 0:n].astype(np.float64)
    c = (n - 1) / 2
    t = np.radians(angle_deg)
    u = (xx - c) * np.cos(t) + (yy - c) * np.sin(t)
    v = -(xx - c) * np.sin(t) + (yy - c) * np.cos(t)
    u = u + shear * v
    half = (c - pad) / (abs(np.cos(t)) + abs(np.sin(t))) / (1 + abs(shear))  # inside the frame
    img = 0.3 * u / n - 0.2 * (v / n) ** 2 + 1e-3 * rng.standard_normal((n, n))
    img[(np.abs(u) > half) | (np.abs(v) > half)] = np.nan
    return img


@pytest.mark.parametrize("seed", range(12))
def test_contours_equal_the_oracle(seed):
    from akbraytracing_amd.affine import find_external_contours
    m = _blobs(seed)
    got = find_external_contours(m)
    want = OA.find_contours_external(m)
    assert len(got) == len(want)
    for g, w in zip(got, want):
        assert np.array_equal(g.reshape(-1, 2), w)


def test_contours_of_a_rectangle_and_nested_regions():
    from akbraytracing_amd.affine import find_external_contours
    m = np.zeros((20, 30), np.uint8)
    m[3:12, 5:25] = 1
    got = find_external_contours(m)
    # cv2's known answer for a filled rectangle: top-left, bottom-left, bottom-right, top-right
    assert len(got) == 1 and np.array_equal(got[0].reshape(-1, 2), [[5, 3], [5, 11], [24, 11], [24, 3]])
    # a ring with a blob inside its hole: RETR_EXTERNAL keeps the ring only
    m[:] = 0
    m[2:18, 2:18] = 1
    m[5:15, 5:15] = 0
    m[8:11, 8:11] = 1
    assert len(find_external_contours(m)) == 1
    # a region touching every edge: the frame makes its border the image's
    m[:] = 1
    assert np.array_equal(find_external_contours(m)[0].reshape(-1, 2), [[0, 0], [0, 19], [29, 19], [29, 0]])
    m[:] = 0
    assert find_external_contours(m) == []


@pytest.mark.parametrize("seed", range(8))
def test_area_length_and_polygon_equal_the_oracle(seed):
    from akbraytracing_amd import affine as A
    m = (~np.isnan(_parallelogram(97, 7 + 9 * seed, shear=0.05 * (seed % 3), seed=seed))).astype(np.uint8)
    m |= _blobs(seed, (97, 97)) & 1
    for c in A.find_external_contours(m):
        assert A.contour_area(c) == OA.contour_area(c.reshape(-1, 2))
        assert A.arc_length(c) == OA.arc_length(c.reshape(-1, 2))
        for frac in (0.003, 0.01, 0.05):
            eps = frac * A.arc_length(c)
            assert np.array_equal(A.approx_poly_dp(c, eps).reshape(-1, 2), OA.approx_poly_dp_closed(c, eps))


def test_affine_solve_and_inverse_equal_the_oracle():
    from akbraytracing_amd import _lib
    from akbraytracing_amd.affine import get_affine_transform
    rng = np.random.default_rng(3)
    for _ in range(200):
        src = rng.uniform(-50, 300, (3, 2)).astype(np.float32)
        dst = rng.uniform(-10, 260, (3, 2)).astype(np.float32)
        M = get_affine_transform(src, dst)
        assert np.array_equal(M, OA.affine_from_points(src, dst))
        iM = np.empty(6)
        _lib.check(_lib.lib().akb_affine_invert(M.ravel().ctypes.data_as(_lib.c_vp), iM.ctypes.data_as(_lib.c_vp)))
        assert np.array_equal(iM, OA.invert_affine(M))
    # the three points map onto their targets
    src = np.array([[10, 5], [90, 20], [0, 70]], np.float32)
    dst = np.array([[0, 0], [63, 0], [0, 63]], np.float32)
    M = get_affine_transform(src, dst)
    np.testing.assert_allclose(M[:, :2] @ src.T.astype(np.float64) + M[:, 2:], dst.T, atol=1e-9)
    with pytest.raises(_lib.AKBError):
        get_affine_transform(np.array([[0, 0], [1, 1], [2, 2]], np.float32), dst)


@pytest.mark.gpu
@pytest.mark.parametrize("case", range(6))
def test_warp_bitwise_vs_oracle(gpu, case):
    from akbraytracing_amd.affine import warp_square
    rng = np.random.default_rng(10 + case)
    ny, nx = 61 + 7 * case, 53 + 11 * case
    img = rng.standard_normal((ny, nx))
    img[rng.random((ny, nx)) < 0.1] = np.nan
    t = rng.uniform(-0.6, 0.6)
    s = rng.uniform(0.6, 1.7)
    M = np.array([[s * np.cos(t), -s * np.sin(t) + 0.1 * case, rng.uniform(-20, 20)],
                  [s * np.sin(t), s * np.cos(t), rng.uniform(-20, 20)]])
    side = 40 + 13 * case
    got = warp_square(torch.from_numpy(img).cuda(), M, side).cpu().numpy()
    want = OA.warp(img, M, side)
    assert np.array_equal(got, want, equal_nan=True)


@pytest.mark.gpu
@pytest.mark.parametrize("n,angle,shear,target", [(65, 8.0, 0.0, 65), (65, -13.0, 0.04, None), (128, 21.0, 0.0, 256),
                                                  (257, 3.5, 0.02, 256)])
def test_extract_affine_square_region_bitwise_vs_oracle(gpu, n, angle, shear, target):
    from akbraytracing_amd.affine import extract_affine_square_region
    img = _parallelogram(n, angle, shear)
    got = extract_affine_square_region(img, target_size=target)
    want = OA.extract_affine_square_region(img, target_size=target)
    assert isinstance(got, np.ndarray) and got.shape == want.shape
    assert np.array_equal(got, want, equal_nan=True)
    # the device-tensor form gives the same bits
    dev = extract_affine_square_region(torch.from_numpy(img).cuda(), target_size=target)
    assert np.array_equal(dev.cpu().numpy(), want, equal_nan=True)


@pytest.mark.gpu
def test_extract_affine_square_region_closed_forms(gpu):
    """An axis-aligned valid block of 41 x 41 pixels: its corner pixels are 40 apart, so the
    reference's default side is int(40.0) = 40 (a 39/40 scaling), and target_size=41 is an exact
    translation that returns the block itself. Fewer or more than 4 corners and an all-NaN map
    raise the reference's ValueErrors."""
    from akbraytracing_amd.affine import extract_affine_square_region
    rng = np.random.default_rng(0)
    img = np.full((70, 80), np.nan)
    blk = rng.standard_normal((41, 41))
    img[11:52, 17:58] = blk
    out = extract_affine_square_region(img)
    assert out.shape == (40, 40) and not np.isnan(out).any()
    assert np.array_equal(out, OA.extract_affine_square_region(img))
    assert out[0, 0] == blk[0, 0] and out[39, 39] == blk[40, 40]  # corners map onto corners
    out = extract_affine_square_region(img, target_size=41)
    assert np.array_equal(out, blk)
    tri = np.full((60, 60), np.nan)
    yy, xx = np.mgrid[0:60, 0:60]
    tri[(xx > 5) & (yy > 5) & (xx + yy < 100)] = 1.0
    with pytest.raises(ValueError, match="4"):
        extract_affine_square_region(tri)
    with pytest.raises(ValueError):
        extract_affine_square_region(np.full((10, 10), np.nan))
    with pytest.raises(AssertionError):
        extract_affine_square_region(np.zeros(5))


@pytest.mark.gpu
def test_install_rebinds_extract_affine_square_region(gpu):
    import types
    from akbraytracing_amd.install import install, uninstall
    mod = types.ModuleType("fake_akb")
    mod.extract_affine_square_region = lambda img, target_size=None: "reference"
    assert "extract_affine_square_region" in install(mod)
    img = _parallelogram(65, 10.0)
    assert np.array_equal(mod.extract_affine_square_region(img, target_size=65),
                          OA.extract_affine_square_region(img, 65), equal_nan=True)
    uninstall(mod)
    assert mod.extract_affine_square_region(img) == "reference"
