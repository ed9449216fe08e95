"""extract_affine_square_region (AKB_raytrace_20250312.py:1047-1119) on the
device.

The reference cuts the valid (non-NaN) parallelogram out of a pupil map and warps it onto a square
with OpenCV: findContours (RETR_EXTERNAL, CHAIN_APPROX_SIMPLE) of the valid mask, the largest
contour by contourArea, approxPolyDP at 1 % of its arcLength, three corners ordered by x + y and
y - x, getAffineTransform onto the square's corners, warpAffine of nan_to_num(img) (INTER_LINEAR)
and of the mask (INTER_NEAREST), NaN where the warped mask is 0.

Here the mask and the two warps are device kernels (akb_valid_mask_u8, akb_warp_affine_f64: one
pass over the output, both warps fused), the contour, polygon and 6 x 6 solve are host C
(akb_affine_host.cpp) and the small float32 steps numpy, as the reference forms them. OpenCV is not
in this image: the restated algorithms (OpenCV 4.x's raster scanner and border following, its
Douglas-Peucker, its LU solve and its fixed-point warp) are checked against the oracle's
independent restatement (oracle/affine.py) and against closed-form cases, but parity with cv2
itself is unpinned.
"""
import numpy as np
import torch

from . import _lib
from . import device as D


def _hp(a):
    return a.ctypes.data_as(_lib.c_vp)


def find_external_contours(mask):
    """cv2.findContours(mask, RETR_EXTERNAL, CHAIN_APPROX_SIMPLE)[0] for a 2-D uint8 mask: a list of
    (k, 1, 2) int32 arrays in cv2's order."""
    m = np.ascontiguousarray(np.asarray(mask, dtype=np.uint8))
    if m.ndim != 2:
        raise ValueError("mask must be 2-D")
    rows, cols = m.shape
    L = _lib.lib()
    cap, ocap = 4 * (rows + cols) + 64, 64
    for _ in range(2):
        xy = np.empty((cap, 2), np.int32)
        offs = np.empty(ocap, np.int32)
        nxy = np.zeros(1, np.int64)
        nc = np.zeros(1, np.int32)
        st = L.akb_external_contours(_hp(m), rows, cols, cap, _hp(xy), _hp(nxy), ocap, _hp(offs), _hp(nc))
        if st == 0:
            return [xy[offs[c]:offs[c + 1]].reshape(-1, 1, 2).copy() for c in range(int(nc[0]))]
        cap, ocap = int(nxy[0]) + 1, int(nc[0]) + 2  # exact sizes for the second call
    _lib.check(st)


def contour_area(c):
    """cv2.contourArea(c) (not oriented): the shoelace sum over float32-converted points in double."""
    p = np.asarray(c, dtype=np.float32).reshape(-1, 2)
    if p.shape[0] == 0:
        return 0.0
    a = 0.0
    px, py = float(p[-1, 0]), float(p[-1, 1])
    for x, y in p.astype(np.float64):
        a += px * y - py * x
        px, py = x, y
    return abs(a * 0.5)


def arc_length(c, closed=True):
    """cv2.arcLength: float32 segment components and square roots, summed in double."""
    p = np.asarray(c, dtype=np.float32).reshape(-1, 2)
    n = p.shape[0]
    if n == 0:
        return 0.0
    per = 0.0
    prev = p[n - 1] if closed else p[0]
    for i in range(n):
        d = p[i] - prev  # float32
        per += float(np.sqrt(d[0] * d[0] + d[1] * d[1], dtype=np.float32))
        prev = p[i]
    return per


def approx_poly_dp(c, eps, closed=True):
    """cv2.approxPolyDP(c, eps, closed) for int32 points: (k, 1, 2) int32."""
    p = np.ascontiguousarray(np.asarray(c, dtype=np.int32).reshape(-1, 2))
    out = np.empty_like(p) if p.size else np.empty((1, 2), np.int32)
    n = np.zeros(1, np.int32)
    _lib.check(_lib.lib().akb_approx_poly_dp(_hp(p), p.shape[0], float(eps), int(bool(closed)), _hp(out), _hp(n)))
    return out[:int(n[0])].reshape(-1, 1, 2).copy()


def get_affine_transform(src, dst):
    """cv2.getAffineTransform(src (3, 2) float32, dst (3, 2) float32) -> (2, 3) float64"""
    s = np.ascontiguousarray(np.asarray(src, dtype=np.float32).reshape(3, 2))
    d = np.ascontiguousarray(np.asarray(dst, dtype=np.float32).reshape(3, 2))
    M = np.empty(6, np.float64)
    _lib.check(_lib.lib().akb_affine_from_points(_hp(s), _hp(d), _hp(M)))
    return M.reshape(2, 3)


def order_points_affine(pts):
    """the reference's inner helper (:1080-1086): top-left, top-right, bottom-left (float32)"""
    s = pts.sum(axis=1)
    diff = np.diff(pts, axis=1)
    return np.array([pts[np.argmin(s)], pts[np.argmin(diff)], pts[np.argmax(diff)]], dtype=np.float32)


def warp_square(img, M, side):
    """warpAffine(nan_to_num(img), M, (side, side), INTER_LINEAR), NaN where the INTER_NEAREST warp
    of the valid mask is 0 - one device pass (img: 2-D float64 device tensor)."""
    iM = np.empty(6, np.float64)
    _lib.check(_lib.lib().akb_affine_invert(_hp(np.ascontiguousarray(M, dtype=np.float64).ravel()), _hp(iM)))
    out = torch.empty((side, side), dtype=D.F64, device=img.device)
    _lib.check(_lib.lib().akb_warp_affine_f64(D.ptr(img), int(img.shape[0]), int(img.shape[1]), _hp(iM), side,
                                              D.ptr(out), D.stream_handle()))
    return out


def extract_affine_square_region(img, target_size=None):
    """Drop-in for the reference function (same arguments, value rules and exceptions). A numpy
    input returns numpy (as the reference), a torch input a device tensor."""
    as_torch = isinstance(img, torch.Tensor)
    if as_torch:
        assert img.dim() == 2, "2次元配列を入力してください"
        x = img.to(device=D.device(), dtype=D.F64).contiguous()
    else:
        a = np.asarray(img)
        assert a.ndim == 2, "2次元配列を入力してください"
        x = D.to_dev(np.ascontiguousarray(a, dtype=np.float64))
    ny, nx = int(x.shape[0]), int(x.shape[1])
    mask = torch.empty((ny, nx), dtype=torch.uint8, device=x.device)
    _lib.check(_lib.lib().akb_valid_mask_u8(D.ptr(x), ny, nx, D.ptr(mask), D.stream_handle()))
    contours = find_external_contours(mask.cpu().numpy())
    if not contours:
        raise ValueError("有効領域が見つかりませんでした")
    contour = max(contours, key=contour_area)
    approx = approx_poly_dp(contour, 0.01 * arc_length(contour, True), True)
    if len(approx) != 4:
        raise ValueError(f"矩形が4点で検出できませんでした（点数: {len(approx)}）")
    src = order_points_affine(approx[:, 0, :].astype(np.float32))
    if target_size is None:
        width = np.linalg.norm(src[0] - src[1])
        height = np.linalg.norm(src[0] - src[2])
        side = int(max(width, height))
    else:
        side = int(target_size)
    dst = np.array([[0, 0], [side - 1, 0], [0, side - 1]], dtype=np.float32)
    M = get_affine_transform(src, dst)
    out = warp_square(x, M, side)
    return out if as_torch else out.cpu().numpy()
