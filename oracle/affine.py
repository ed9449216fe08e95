"""extract_affine_square_region of AKB_raytrace_20250312.py (:1047-1119), restated. TEST
INFRASTRUCTURE ONLY. PARITY UNPINNED: the reference calls OpenCV (cv2: findContours,
contourArea, arcLength, approxPolyDP, getAffineTransform, warpAffine), which is not installed in
this image, and the reference holds no recorded output of this function. The algorithms are
restated here from OpenCV 4.x's published implementation, independently of the product's C / HIP
code (akbraytracing_amd/csrc/akb_affine_host.cpp, akb_psfcalc.hip), so the tests check the product
against this module bit for bit and both against closed-form cases (axis-aligned regions, exact
translations) - not against cv2.

* findContours(RETR_EXTERNAL, CHAIN_APPROX_SIMPLE): the image framed by one zero pixel; a raster
  scan that starts an outer border where a 1 follows a 0 unless the last border pixel seen to the
  left on the row carries a positive mark (the start is inside a traced region); Suzuki-Abe
  border following (chain codes 0..7 counter-clockwise from +x, y down; the first neighbour
  searched clockwise from the left, then counter-clockwise from the previous direction + 1),
  marking right-bound pixels -126 and others 2, keeping a point where the direction changes; the
  list is returned last-found first.
* contourArea: shoelace over float32 points in double; arcLength: float32 steps and square roots
  summed in double.
* approxPolyDP(closed): three rounds of "farthest point from the current start", the two slices
  between the last pair on a stack, each split at its farthest point from the chord while
  dist^2 > eps^2 |chord|^2, then the pass dropping nearly collinear points.
* getAffineTransform: the 6 x 6 system solved by Gaussian elimination with partial pivoting.
* warpAffine: M inverted (D = 1 / det), source coordinates in fixed point - the affine terms times
  1024 rounded to nearest even, + 16 and >> 5 for INTER_LINEAR (5 fractional bits, weights
  products of (1 - f, f) with f = k / 32), + 512 and >> 10 for INTER_NEAREST; BORDER_CONSTANT 0.
"""
import numpy as np

_DX = [1, 1, 0, -1, -1, -1, 0, 1]
_DY = [0, -1, -1, -1, 0, 1, 1, 1]


def _follow(img, y, x):
    """outer border from (y, x) of the framed image; marks it; points in unframed coordinates"""
    out = []
    s = s_end = 4
    while True:
        s = (s - 1) & 7
        y1, x1 = y + _DY[s], x + _DX[s]
        if img[y1, x1] != 0 or s == s_end:
            break
    if s == s_end and img[y1, x1] == 0:
        img[y, x] = -126
        return [(x - 1, y - 1)]
    cy, cx = y, x  # i3
    py, px = y - 1, x - 1  # the point written
    prev_s = s ^ 4
    while True:
        s_end = s
        ny = nx = None
        for k in range(s + 1, s + 9):
            d = k & 7
            ty, tx = cy + _DY[d], cx + _DX[d]
            if img[ty, tx] != 0:
                s, ny, nx = d, ty, tx
                break
        else:  # cannot happen for a region of more than one pixel
            raise AssertionError("border following lost the region")
        if 0 <= s - 1 < s_end:
            img[cy, cx] = -126
        elif img[cy, cx] == 1:
            img[cy, cx] = 2
        if s != prev_s:
            out.append((px, py))
            prev_s = s
        px += _DX[s]
        py += _DY[s]
        if (ny, nx) == (y, x) and (cy, cx) == (y1, x1):
            break
        cy, cx = ny, nx
        s = (s + 4) & 7
    return out


def find_contours_external(mask):
    """cv2.findContours(mask, RETR_EXTERNAL, CHAIN_APPROX_SIMPLE)[0] as a list of (k, 2) int arrays"""
    m = np.asarray(mask)
    rows, cols = m.shape
    img = np.zeros((rows + 2, cols + 2), np.int16)
    img[1:-1, 1:-1] = m != 0
    found = []
    for y in range(1, rows + 1):
        prev, lnbd = 0, 0
        for x in range(1, cols + 1):
            p = int(img[y, x])
            if p == prev:
                continue
            if prev == 0 and p == 1 and img[y, lnbd] <= 0:
                found.append(np.array(_follow(img, y, x), dtype=np.int64).reshape(-1, 2))
                prev = int(img[y, x])
                continue
            if p == 0 and prev >= 1 and (prev & -2):
                lnbd = x - 1
            prev = p
            if prev & -2:
                lnbd = x
    return found[::-1]


def contour_area(c):
    p = np.asarray(c, np.float32).reshape(-1, 2).astype(np.float64)
    if len(p) == 0:
        return 0.0
    q = np.roll(p, 1, axis=0)
    a = 0.0
    for (x0, y0), (x1, y1) in zip(q, p):
        a += x0 * y1 - y0 * x1
    return abs(0.5 * a)


def arc_length(c):
    p = np.asarray(c, np.float32).reshape(-1, 2)
    per = 0.0
    for a, b in zip(np.roll(p, 1, axis=0), p):
        d = (b - a).astype(np.float32)
        per += float(np.float32(np.sqrt(np.float32(d[0] * d[0] + d[1] * d[1]))))
    return per


def approx_poly_dp_closed(c, eps):
    src = [tuple(int(v) for v in r) for r in np.asarray(c).reshape(-1, 2)]
    n = len(src)
    if n == 0:
        return np.zeros((0, 2), np.int64)
    e2 = eps * eps
    # 1. two approximately farthest points (three rounds from the running start)
    start, pos, far = 0, 0, 0
    le = False
    for _ in range(3):
        start = (start + far) % n
        sx, sy = src[start]
        best, far = 0.0, 0
        for j in range(1, n):
            x, y = src[(start + j) % n]
            d = float(x - sx) ** 2 + float(y - sy) ** 2
            if d > best:
                best, far = d, j
        le = best <= e2
    out = []
    if le:
        out.append(src[start])
        stack = []
    else:
        a, b = start, (start + far) % n
        stack = [(b, a), (a, b)]  # (start, end) slices; the last one is processed first
    # 2. split slices at their farthest point from the chord
    while stack:
        s0, s1 = stack.pop()
        (sx, sy), (ex, ey) = src[s0], src[s1]
        nxt = (s0 + 1) % n
        if nxt == s1:
            out.append((sx, sy))
            continue
        dx, dy = float(ex - sx), float(ey - sy)
        best, at = 0.0, None
        i = nxt
        while i != s1:
            x, y = src[i]
            d = abs((y - sy) * dx - (x - sx) * dy)
            if d > best:
                best, at = d, i
            i = (i + 1) % n
        if best * best <= e2 * (dx * dx + dy * dy):
            out.append((sx, sy))
        else:
            stack.append((at, s1))
            stack.append((s0, at))
    # 3. drop nearly collinear points (closed curve: starts from the last point)
    cnt = len(out)
    res = list(out)
    new = cnt
    st = res[cnt - 1]
    wpos = 0
    rpos = 0
    pt = res[rpos]
    rpos = (rpos + 1) % cnt
    i = 0
    while i < cnt and new > 2:
        en = res[rpos]
        rpos = (rpos + 1) % cnt
        dx, dy = float(en[0] - st[0]), float(en[1] - st[1])
        dist = abs((pt[0] - st[0]) * dy - (pt[1] - st[1]) * dx)
        sip = (pt[0] - st[0]) * (en[0] - pt[0]) + (pt[1] - st[1]) * (en[1] - pt[1])
        if dist * dist <= 0.5 * e2 * (dx * dx + dy * dy) and dx != 0 and dy != 0 and sip >= 0:
            new -= 1
            res[wpos] = st = en
            wpos = (wpos + 1) % cnt
            pt = res[rpos]
            rpos = (rpos + 1) % cnt
            i += 2
            continue
        res[wpos] = st = pt
        wpos = (wpos + 1) % cnt
        pt = en
        i += 1
    return np.array(res[:new], dtype=np.int64).reshape(-1, 2)


def affine_from_points(src, dst):
    s = np.asarray(src, np.float32).astype(np.float64)
    d = np.asarray(dst, np.float32).astype(np.float64)
    A = np.zeros((6, 6))
    b = np.zeros(6)
    for i in range(3):
        A[2 * i, 0:3] = (s[i, 0], s[i, 1], 1.0)
        A[2 * i + 1, 3:6] = (s[i, 0], s[i, 1], 1.0)
        b[2 * i], b[2 * i + 1] = d[i]
    for i in range(6):
        k = i
        for j in range(i + 1, 6):
            if abs(A[j, i]) > abs(A[k, i]):
                k = j
        if k != i:
            A[[i, k], i:] = A[[k, i], i:]
            b[[i, k]] = b[[k, i]]
        f = -1.0 / A[i, i]
        for j in range(i + 1, 6):
            al = A[j, i] * f
            for c in range(i + 1, 6):
                A[j, c] = A[j, c] + al * A[i, c]
            b[j] = b[j] + al * b[i]
    for i in range(5, -1, -1):
        t = b[i]
        for c in range(i + 1, 6):
            t = t - A[i, c] * b[c]
        b[i] = t / A[i, i]
    return b.reshape(2, 3)


def invert_affine(M):
    m = [float(v) for v in np.asarray(M, np.float64).ravel()]
    D = m[0] * m[4] - m[1] * m[3]
    D = 1.0 / D if D != 0 else 0.0
    a11, a22 = m[4] * D, m[0] * D
    m[0], m[1], m[3], m[4] = a11, m[1] * -D, m[3] * -D, a22
    b1 = -m[0] * m[2] - m[1] * m[5]
    b2 = -m[3] * m[2] - m[4] * m[5]
    m[2], m[5] = b1, b2
    return m


def warp(img, M, side):
    """warpAffine(nan_to_num(img), INTER_LINEAR) with NaN where the INTER_NEAREST warp of the
    valid mask is 0 (BORDER_CONSTANT 0)"""
    img = np.asarray(img, np.float64)
    ny, nx = img.shape
    f = np.nan_to_num(img)
    valid = ~np.isnan(img)
    m0, m1, m2, m3, m4, m5 = invert_affine(M)
    ys = np.arange(side, dtype=np.float64)[:, None]
    xs = np.arange(side, dtype=np.float64)[None, :]
    xr = np.rint((m1 * ys + m2) * 1024).astype(np.int64)
    yr = np.rint((m4 * ys + m5) * 1024).astype(np.int64)
    ad = np.rint(m0 * xs * 1024).astype(np.int64)
    bd = np.rint(m3 * xs * 1024).astype(np.int64)
    clip = lambda v: np.clip(v, -32768, 32767)  # noqa: E731
    xn, yn = clip((xr + 512 + ad) >> 10), clip((yr + 512 + bd) >> 10)
    inn = (xn >= 0) & (xn < nx) & (yn >= 0) & (yn < ny)
    mk = np.zeros((side, side), bool)
    mk[inn] = valid[yn[inn], xn[inn]]
    X, Y = (xr + 16 + ad) >> 5, (yr + 16 + bd) >> 5
    sx, sy = clip(X >> 5), clip(Y >> 5)
    ax, ay = (X & 31) / 32.0, (Y & 31) / 32.0
    w = [(1 - ay) * (1 - ax), (1 - ay) * ax, ay * (1 - ax), ay * ax]

    def at(yy, xx):
        ok = (xx >= 0) & (xx < nx) & (yy >= 0) & (yy < ny)
        v = np.zeros((side, side))
        v[ok] = f[yy[ok], xx[ok]]
        return v

    v = [at(sy, sx), at(sy, sx + 1), at(sy + 1, sx), at(sy + 1, sx + 1)]
    out = v[0] * w[0] + v[1] * w[1]
    out = out + v[2] * w[2]
    out = out + v[3] * w[3]
    out[~mk] = np.nan
    return out


def extract_affine_square_region(img, target_size=None):
    a = np.asarray(img, np.float64)
    assert a.ndim == 2
    cs = find_contours_external((~np.isnan(a)).astype(np.uint8) * 255)
    if not cs:
        raise ValueError("no valid region")
    c = cs[0]
    for k in cs[1:]:
        if contour_area(k) > contour_area(c):
            c = k
    ap = approx_poly_dp_closed(c, 0.01 * arc_length(c))
    if len(ap) != 4:
        raise ValueError(f"not 4 points: {len(ap)}")
    p = ap.astype(np.float32)
    s, dd = p.sum(axis=1), np.diff(p, axis=1)
    src = np.array([p[np.argmin(s)], p[np.argmin(dd)], p[np.argmax(dd)]], np.float32)
    if target_size is None:
        side = int(max(np.linalg.norm(src[0] - src[1]), np.linalg.norm(src[0] - src[2])))
    else:
        side = int(target_size)
    dst = np.array([[0, 0], [side - 1, 0], [0, side - 1]], np.float32)
    return warp(a, affine_from_points(src, dst), side)
