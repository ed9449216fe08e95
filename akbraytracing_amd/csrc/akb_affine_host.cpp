// Host half of extract_affine_square_region (AKB_raytrace_20250312.py:1047-1119, row f4 of SURVEY.md
// §8). The reference finds the valid (non-NaN) region of a pupil map with OpenCV and warps it onto a
// square:
//
//   contours = cv2.findContours(mask, RETR_EXTERNAL, CHAIN_APPROX_SIMPLE)   (:1066)
//   contour  = max(contours, key=cv2.contourArea)                            (:1070)
//   approx   = cv2.approxPolyDP(contour, 0.01 * cv2.arcLength(contour, True), True)   (:1073-1074)
//   M        = cv2.getAffineTransform(3 ordered corners, square corners)    (:1106)
//   warped   = cv2.warpAffine(nan_to_num(img), M, INTER_LINEAR); mask by INTER_NEAREST  (:1109-1115)
//
// OpenCV is not part of this image (cv2 does not import here), so these are restatements of the
// published algorithms as OpenCV 4.x implements them - Suzuki-Abe border following with OpenCV's
// raster scanner and chain compression, OpenCV's closed Douglas-Peucker (two farthest points, an
// explicit slice stack, the final collinear clean-up), LU with partial pivoting for the 6 x 6
// affine system, and warpAffine's inversion of M - and their parity with cv2 is unpinned. The warp
// itself is the device kernel akb_warp_affine_f64 (akb_psfcalc.hip).
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <vector>

#include "akb_common.h"

namespace {

// OpenCV's chain-code directions: 0 = +x, then counter-clockwise on screen (y grows downwards)
const int kCodeDx[8] = {1, 1, 0, -1, -1, -1, 0, 1};
const int kCodeDy[8] = {0, -1, -1, -1, 0, 1, 1, 1};

// One outer border from pixel i0 of the framed image (values 0 / 1, traced pixels marked 2, or
// -126 where the border is "right bound"), CHAIN_APPROX_SIMPLE: a point is kept where the chain
// direction changes. Points are in the unframed image's coordinates.
void fetch_contour(int8_t* img, int64_t step, int64_t i0, int px, int py, std::vector<int32_t>& out) {
    const int8_t nbd = 2;
    int64_t deltas[16];
    for (int s = 0; s < 8; ++s) deltas[s] = deltas[s + 8] = kCodeDx[s] + (int64_t)kCodeDy[s] * step;
    int s = 4, s_end = 4;  // an outer border: the pixel to the left is background
    int64_t i1;
    do {
        s = (s - 1) & 7;
        i1 = i0 + deltas[s];
    } while (img[i1] == 0 && s != s_end);
    if (s == s_end) {  // a single-pixel region
        img[i0] = (int8_t)(nbd | -128);
        out.push_back(px);
        out.push_back(py);
        return;
    }
    int64_t i3 = i0, i4 = i0;
    int prev_s = s ^ 4;
    for (;;) {
        s_end = s;
        while (s < 15) {
            i4 = i3 + deltas[++s];
            if (img[i4] != 0) break;
        }
        s &= 7;
        if ((unsigned)(s - 1) < (unsigned)s_end)
            img[i3] = (int8_t)(nbd | -128);
        else if (img[i3] == 1)
            img[i3] = nbd;
        if (s != prev_s) {
            out.push_back(px);
            out.push_back(py);
            prev_s = s;
        }
        px += kCodeDx[s];
        py += kCodeDy[s];
        if (i4 == i0 && i3 == i1) break;
        i3 = i4;
        s = (s + 4) & 7;
    }
}

}  // namespace

extern "C" {

int akb_external_contours(const uint8_t* mask, int rows, int cols, int64_t cap, int32_t* xy, int64_t* n_xy,
                          int32_t ocap, int32_t* offsets, int32_t* n_contours) {
    AKB_REQUIRE(mask && xy && n_xy && offsets && n_contours, "null pointer");
    AKB_REQUIRE(rows > 0 && cols > 0 && cap >= 0 && ocap >= 0, "sizes");
    // the framed binary image (findContours works on a copy with a one-pixel zero border)
    const int W = cols + 2, H = rows + 2;
    std::vector<int8_t> img((size_t)W * H, 0);
    for (int y = 0; y < rows; ++y)
        for (int x = 0; x < cols; ++x) img[(size_t)(y + 1) * W + x + 1] = mask[(size_t)y * cols + x] != 0;
    std::vector<int32_t> pts;
    std::vector<int32_t> offs{0};
    // OpenCV's raster scanner in RETR_EXTERNAL mode: an outer border starts where a 1 follows a 0;
    // it is traced unless the last border pixel met on this row to the left (lnbd) is positive,
    // i.e. the start lies inside a region already traced (holes are never traced in this mode)
    for (int y = 1; y < H - 1; ++y) {
        int8_t* row = img.data() + (size_t)y * W;
        int lnbd = 0, prev = 0;
        for (int x = 1; x < W - 1; ++x) {
            const int p = row[x];
            if (p == prev) continue;
            bool skip = false;
            if (!(prev == 0 && p == 1)) {
                if (p != 0 || prev < 1) {
                    skip = true;
                } else {  // a hole border: not traced in this mode
                    if (prev & -2) lnbd = x - 1;
                    skip = true;
                }
            } else if (row[lnbd] > 0) {
                skip = true;
            }
            if (skip) {
                prev = p;
                if (prev & -2) lnbd = x;
                continue;
            }
            fetch_contour(img.data(), W, (int64_t)y * W + x, x - 1, y - 1, pts);
            offs.push_back((int32_t)(pts.size() / 2));
            prev = row[x];  // the scan resumes after the (now marked) start pixel
        }
    }
    // cv2 lists the contours last-found first
    const int nc = (int)offs.size() - 1;
    *n_contours = nc;
    *n_xy = (int64_t)pts.size() / 2;
    if ((int64_t)pts.size() / 2 > cap || nc + 1 > ocap) {
        ::akb::set_error("akb_external_contours: %lld points / %d contours exceed the caller's capacity",
                         (long long)(pts.size() / 2), nc);
        return AKB_E_INVALID;
    }
    int64_t w = 0;
    offsets[0] = 0;
    for (int c = nc - 1, k = 1; c >= 0; --c, ++k) {
        for (int32_t i = offs[c]; i < offs[c + 1]; ++i) {
            xy[2 * w] = pts[2 * (size_t)i];
            xy[2 * w + 1] = pts[2 * (size_t)i + 1];
            ++w;
        }
        offsets[k] = (int32_t)w;
    }
    return AKB_OK;
}

int akb_approx_poly_dp(const int32_t* src, int32_t count0, double eps, int closed, int32_t* dst, int32_t* n_out) {
    AKB_REQUIRE(src && dst && n_out && count0 >= 0, "arguments");
    *n_out = 0;
    if (count0 == 0) return AKB_OK;
    struct Range {
        int32_t start, end;
    };
    std::vector<Range> stack;
    const int32_t count = count0;
    int32_t new_count = 0;
    auto X = [&](int32_t i) { return src[2 * (int64_t)i]; };
    auto Y = [&](int32_t i) { return src[2 * (int64_t)i + 1]; };
    auto write_pt = [&](int32_t x, int32_t y) {
        dst[2 * (int64_t)new_count] = x;
        dst[2 * (int64_t)new_count + 1] = y;
        ++new_count;
    };
    int init_iters = 3;
    Range slice{0, 0}, right{0, 0};
    int32_t pos = 0;
    int32_t sx = -1000000, sy = -1000000;  // start point
    bool is_closed = closed != 0, le_eps = false;
    eps *= eps;
    if (!is_closed) {
        right.start = count;
        if (X(count - 1) != X(0) || Y(count - 1) != Y(0)) {
            slice = Range{0, count - 1};
            stack.push_back(slice);
        } else {
            is_closed = true;
            init_iters = 1;
        }
    }
    if (is_closed) {
        // 1. two approximately farthest points
        right.start = 0;
        for (int it = 0; it < init_iters; ++it) {
            double max_dist = 0;
            pos = (pos + right.start) % count;
            sx = X(pos);
            sy = Y(pos);
            if (++pos >= count) pos = 0;
            for (int32_t j = 1; j < count; ++j) {
                const double dx = (double)X(pos) - sx, dy = (double)Y(pos) - sy;
                if (++pos >= count) pos = 0;
                const double dist = dx * dx + dy * dy;
                if (dist > max_dist) {
                    max_dist = dist;
                    right.start = j;
                }
            }
            le_eps = max_dist <= eps;
        }
        // 2. the initial two slices
        if (!le_eps) {
            right.end = slice.start = pos % count;
            slice.end = right.start = (right.start + slice.start) % count;
            stack.push_back(right);
            stack.push_back(slice);
        } else {
            write_pt(sx, sy);
        }
    }
    // 3. split each slice at its farthest point until every point lies within eps of its chord
    while (!stack.empty()) {
        slice = stack.back();
        stack.pop_back();
        const int32_t ex = X(slice.end), ey = Y(slice.end);
        pos = slice.start;
        sx = X(pos);
        sy = Y(pos);
        if (++pos >= count) pos = 0;
        if (pos != slice.end) {
            double max_dist = 0;
            const double dx = (double)ex - sx, dy = (double)ey - sy;
            if (dx == 0 && dy == 0) {
                ::akb::set_error("akb_approx_poly_dp: a slice with coincident ends");
                return AKB_E_INVALID;
            }
            while (pos != slice.end) {
                const double px = X(pos), py = Y(pos);
                if (++pos >= count) pos = 0;
                const double dist = fabs((py - sy) * dx - (px - sx) * dy);
                if (dist > max_dist) {
                    max_dist = dist;
                    right.start = (pos + count - 1) % count;
                }
            }
            le_eps = max_dist * max_dist <= eps * (dx * dx + dy * dy);
        } else {
            le_eps = true;
            sx = X(slice.start);
            sy = Y(slice.start);
        }
        if (le_eps) {
            write_pt(sx, sy);
        } else {
            right.end = slice.end;
            slice.end = right.start;
            stack.push_back(right);
            stack.push_back(slice);
        }
    }
    if (!is_closed) write_pt(X(count - 1), Y(count - 1));
    // 4. clean-up: drop points on [almost] straight runs of the result
    is_closed = closed != 0;
    const int32_t cnt = new_count;
    int32_t dpos = is_closed ? cnt - 1 : 0;
    auto DX = [&](int32_t i) { return dst[2 * (int64_t)i]; };
    auto DY = [&](int32_t i) { return dst[2 * (int64_t)i + 1]; };
    int32_t s0x = DX(dpos), s0y = DY(dpos);
    if (++dpos >= cnt) dpos = 0;
    int32_t wpos = dpos;  // the slot after the start point
    int32_t ptx = DX(dpos), pty = DY(dpos);
    if (++dpos >= cnt) dpos = 0;
    for (int32_t i = !is_closed; i < cnt - !is_closed && new_count > 2; ++i) {
        const int32_t e_x = DX(dpos), e_y = DY(dpos);
        if (++dpos >= cnt) dpos = 0;
        const double dx = (double)e_x - s0x, dy = (double)e_y - s0y;
        const double dist = fabs(((double)ptx - s0x) * dy - ((double)pty - s0y) * dx);
        const double sip = ((double)ptx - s0x) * ((double)e_x - ptx) + ((double)pty - s0y) * ((double)e_y - pty);
        if (dist * dist <= 0.5 * eps * (dx * dx + dy * dy) && dx != 0 && dy != 0 && sip >= 0) {
            --new_count;
            dst[2 * (int64_t)wpos] = s0x = e_x;
            dst[2 * (int64_t)wpos + 1] = s0y = e_y;
            if (++wpos >= cnt) wpos = 0;
            ptx = DX(dpos);
            pty = DY(dpos);
            if (++dpos >= cnt) dpos = 0;
            ++i;
            continue;
        }
        dst[2 * (int64_t)wpos] = s0x = ptx;
        dst[2 * (int64_t)wpos + 1] = s0y = pty;
        if (++wpos >= cnt) wpos = 0;
        ptx = e_x;
        pty = e_y;
    }
    if (!is_closed) {
        dst[2 * (int64_t)wpos] = ptx;
        dst[2 * (int64_t)wpos + 1] = pty;
    }
    *n_out = new_count;
    return AKB_OK;
}

int akb_affine_from_points(const float* src, const float* dst, double* M) {
    AKB_REQUIRE(src && dst && M, "null pointer");
    // the 6 x 6 system of getAffineTransform: rows (x, y, 1, 0, 0, 0) -> u, (0, 0, 0, x, y, 1) -> v
    double a[36], b[6];
    for (int i = 0; i < 3; ++i) {
        const int j = i * 12, k = i * 12 + 6;
        a[j] = a[k + 3] = src[2 * i];
        a[j + 1] = a[k + 4] = src[2 * i + 1];
        a[j + 2] = a[k + 5] = 1;
        a[j + 3] = a[j + 4] = a[j + 5] = 0;
        a[k] = a[k + 1] = a[k + 2] = 0;
        b[2 * i] = dst[2 * i];
        b[2 * i + 1] = dst[2 * i + 1];
    }
    // Gaussian elimination with partial pivoting (the first largest pivot), then back substitution
    const int m = 6;
    const double eps = 2.220446049250313e-16 * 100;
    for (int i = 0; i < m; ++i) {
        int k = i;
        for (int j = i + 1; j < m; ++j)
            if (fabs(a[j * m + i]) > fabs(a[k * m + i])) k = j;
        if (fabs(a[k * m + i]) < eps) {
            ::akb::set_error("akb_affine_from_points: the three points are collinear");
            return AKB_E_INVALID;
        }
        if (k != i) {
            for (int j = i; j < m; ++j) {
                const double t = a[i * m + j];
                a[i * m + j] = a[k * m + j];
                a[k * m + j] = t;
            }
            const double t = b[i];
            b[i] = b[k];
            b[k] = t;
        }
        const double d = -1 / a[i * m + i];
        for (int j = i + 1; j < m; ++j) {
            const double alpha = a[j * m + i] * d;
            for (int c = i + 1; c < m; ++c) a[j * m + c] += alpha * a[i * m + c];
            b[j] += alpha * b[i];
        }
    }
    for (int i = m - 1; i >= 0; --i) {
        double s = b[i];
        for (int c = i + 1; c < m; ++c) s -= a[i * m + c] * b[c];
        b[i] = s / a[i * m + i];
    }
    for (int i = 0; i < 6; ++i) M[i] = b[i];
    return AKB_OK;
}

int akb_affine_invert(const double* M, double* iM) {
    AKB_REQUIRE(M && iM, "null pointer");
    double m[6];
    memcpy(m, M, sizeof m);
    double D = m[0] * m[4] - m[1] * m[3];
    D = D != 0 ? 1. / D : 0;
    const double A11 = m[4] * D, A22 = m[0] * D;
    m[0] = A11;
    m[1] *= -D;
    m[3] *= -D;
    m[4] = A22;
    const double b1 = -m[0] * m[2] - m[1] * m[5];
    const double b2 = -m[3] * m[2] - m[4] * m[5];
    m[2] = b1;
    m[5] = b2;
    memcpy(iM, m, sizeof m);
    return AKB_OK;
}

}  // extern "C"
