"""System construction of the AKB driver: params[26] -> the four quadrics.

plot_result_debug (AKB_raytrace_20250312.py:1326) starts every call by building its Wolter III+I
system from design constants and the 26 alignment parameters; the ray trace proper only sees the
resulting 10-coefficient quadrics, the detector plane and the launch-angle ranges. This module
restates that construction for the live configuration (Setting12 vertical / setting11
horizontal, :1706-1755; option_axial, option_alignment, optin_axialrotation, option_rotateLocal
all True as the driver hard-codes them, :1897-1900) and returns the SystemGeometry that
wavefront.RayWave and autofocus.TestTrace trace.

Scalar arithmetic stays numpy float64 on the host in the reference's own expression order
(coefficient shifts and rotations are ten-number transforms, negligible work); the few centre
traces it needs (2-3 rays per mirror, :2252-2391) go through the drop-in primitives, which run
on the device (`prims`, default akbraytracing_amd.primitives; the CPU tests pass the oracle's
restatement to check the host logic alone). The coefficients come out bit-identical to the
reference's (tests/golden/akb_autofocus.npz, recorded from plot_result_debug itself).

Coefficient transforms (the reference's module functions, restated):
  shift_x / shift_y / shift_z   :645-667  (EllipseRaytrace3D.py:73-95)
  rotation_matrix               :747-762  (Rodrigues, EllipseRaytrace3D.py:97-112)
  rotate_general_axis           :764-793  (EllipseRaytrace3D.py:114-143)
  rotatematrix                  :980-984
"""
import numpy as np

from .trace import Mirror


# ---------------------------------------------------------------- coefficient transforms

def shift_x(coeffs, s):
    """Translate the quadric by s along x (:645-651): returns a list, as the reference."""
    a, b, c, d, e, f, g, h, i, j = coeffs
    return [a, b, c, d, e, f, g - 2 * a * s, h - d * s, i - e * s, j + a * s**2 - g * s]


def shift_y(coeffs, s):
    """:653-659"""
    a, b, c, d, e, f, g, h, i, j = coeffs
    return [a, b, c, d, e, f, g - d * s, h - 2 * b * s, i - f * s, j + b * s**2 - h * s]


def shift_z(coeffs, s):
    """:661-667"""
    a, b, c, d, e, f, g, h, i, j = coeffs
    return [a, b, c, d, e, f, g - e * s, h, i - 2 * c * s, j + c * s**2 - i * s]


def rotation_matrix(axis, theta):
    """Rodrigues' rotation about `axis` (normalised first), :747-762."""
    axis = axis / np.linalg.norm(axis)
    ct, st = np.cos(theta), np.sin(theta)
    ux, uy, uz = axis
    k = np.array([[0, -uz, uy], [uz, 0, -ux], [-uy, ux, 0]])
    return np.eye(3) * ct + (1 - ct) * np.outer(axis, axis) + k * st


def rotate_general_axis(coeffs, axis, theta, center):
    """Rotate the quadric by theta about `axis` through `center` (:764-793): (coeffs, R)."""
    coeffs = shift_z(shift_y(shift_x(coeffs, -center[0]), -center[1]), -center[2])
    a, b, c, d, e, f, g, h, i, j = coeffs
    R = rotation_matrix(axis, theta).T
    r = R  # the substituted coordinates: x = R[0,0] x' + R[0,1] y' + ...
    a1 = a * r[0, 0]**2 + b * r[1, 0]**2 + c * r[2, 0]**2 + d * r[0, 0] * r[1, 0] + e * r[2, 0] * r[0, 0] \
        + f * r[1, 0] * r[2, 0]
    b1 = a * r[0, 1]**2 + b * r[1, 1]**2 + c * r[2, 1]**2 + d * r[0, 1] * r[1, 1] + e * r[2, 1] * r[0, 1] \
        + f * r[1, 1] * r[2, 1]
    c1 = a * r[0, 2]**2 + b * r[1, 2]**2 + c * r[2, 2]**2 + d * r[0, 2] * r[1, 2] + e * r[2, 2] * r[0, 2] \
        + f * r[1, 2] * r[2, 2]
    d1 = 2 * a * r[0, 0] * r[0, 1] + 2 * b * r[1, 0] * r[1, 1] + 2 * c * r[2, 0] * r[2, 1] \
        + d * (r[0, 1] * r[1, 0] + r[0, 0] * r[1, 1]) + e * (r[2, 1] * r[0, 0] + r[2, 0] * r[0, 1]) \
        + f * (r[1, 1] * r[2, 0] + r[1, 0] * r[2, 1])
    e1 = 2 * a * r[0, 0] * r[0, 2] + 2 * b * r[1, 0] * r[1, 2] + 2 * c * r[2, 0] * r[2, 2] \
        + d * (r[0, 2] * r[1, 0] + r[0, 0] * r[1, 2]) + e * (r[2, 2] * r[0, 0] + r[2, 0] * r[0, 2]) \
        + f * (r[1, 2] * r[2, 0] + r[1, 0] * r[2, 2])
    f1 = 2 * a * r[0, 1] * r[0, 2] + 2 * b * r[1, 1] * r[1, 2] + 2 * c * r[2, 1] * r[2, 2] \
        + d * (r[0, 1] * r[1, 2] + r[0, 2] * r[1, 1]) + e * (r[2, 1] * r[0, 2] + r[2, 2] * r[0, 1]) \
        + f * (r[1, 1] * r[2, 2] + r[1, 2] * r[2, 1])
    g1 = g * r[0, 0] + h * r[1, 0] + i * r[2, 0]
    h1 = g * r[0, 1] + h * r[1, 1] + i * r[2, 1]
    i1 = g * r[0, 2] + h * r[1, 2] + i * r[2, 2]
    out = [a1, b1, c1, d1, e1, f1, g1, h1, i1, j]
    out = shift_z(shift_y(shift_x(out, center[0]), center[1]), center[2])
    return out, rotation_matrix(axis, theta)


def rotatematrix(R, ax, ay, az):
    """The mirror's local axes carried along by R (:980-984)."""
    return np.dot(R, ax), np.dot(R, ay), np.dot(R, az)


def shift_along(coeffs, s, axis, swapped=False):
    """A decenter by s along a local axis: shift_x / shift_y / shift_z by s * axis[k] (:2565-2612).
    swapped: the reference's decenterZ of the H ellipse applies the axis components in the order
    z, y, x (:2613-2616); kept as it is."""
    if swapped:
        return shift_x(shift_y(shift_z(coeffs, s * axis[0]), s * axis[1]), s * axis[2])
    return shift_z(shift_y(shift_x(coeffs, s * axis[0]), s * axis[1]), s * axis[2])


# ---------------------------------------------------------------- the AKB design (Setting12 / setting11)

class AKBDesign:
    """Design constants of the live configuration (:1706-1755)."""
    # vertical Wolter III, Setting12
    a_hyp_v = np.float64(72.9825)
    b_hyp_v = np.float64(0.263879113520857)
    a_ell_v = np.float64(0.1175)
    b_ell_v = np.float64(0.0283168369674688)
    hyp_length_v = np.float64(0.043)
    ell_length_v = np.float64(0.0809220387326922)
    theta1_v = np.float64(5.55983241203018E-05)
    # horizontal Wolter I, setting11
    a_ell_h = np.float64(73.1076714403445)
    b_ell_h = np.float64(0.517019631143022)
    a_hyp_h = np.float64(0.0077)
    b_hyp_h = np.float64(0.00432051448679384)
    hyp_length_h = np.float64(0.01380360633)
    ell_length_h = np.float64(0.030)
    theta1_h = np.float64(0.000145746388538841)
    # 'ray_wave' second detector and wavelength (option_HighNA, :3612-3614)
    defocus_wave = 1e-2
    wavelength_m = 13.5e-9


PARAM_NAMES = (
    "defocus", "astigH",
    "pitch_hyp_v", "roll_hyp_v", "yaw_hyp_v", "decenterX_hyp_v", "decenterY_hyp_v", "decenterZ_hyp_v",
    "pitch_hyp_h", "roll_hyp_h", "yaw_hyp_h", "decenterX_hyp_h", "decenterY_hyp_h", "decenterZ_hyp_h",
    "pitch_ell_v", "roll_ell_v", "yaw_ell_v", "decenterX_ell_v", "decenterY_ell_v", "decenterZ_ell_v",
    "pitch_ell_h", "roll_ell_h", "yaw_ell_h", "decenterX_ell_h", "decenterY_ell_h", "decenterZ_ell_h",
)  # the unpacking order of :1327-1331


def _calc_y_hyp(a, b, x):
    """calc_Y_hyp (:946-948)"""
    return np.sqrt(-b ** 2 + (b * (x - np.sqrt(a ** 2 + b ** 2)) / a) ** 2)


def _calc_y_ell(a, b, x):
    """calcEll_Yvalue (:283-284)"""
    return np.sqrt(b**2. - (b * (x - np.sqrt(a**2. - b**2.)) / a)**2.)


def _wolter3_theta5(a_hyp, b_hyp, org_hyp, a_ell, b_ell, org_ell, theta1):
    """theta5 of print_optical_design (:1996-2023), the exit angle of the Wolter III pair for a
    ray leaving the source at theta1 (the other outputs of that helper are never used)."""
    l2 = (4 * a_hyp**2 + (org_hyp * 2)**2 - 4 * a_hyp * (org_hyp * 2) * np.cos(theta1)) / (4 * org_hyp - 4 * a_hyp)
    l1 = 2 * a_hyp + l2
    theta3 = np.arcsin(l1 * np.sin(theta1) / l2)
    l4 = ((org_ell)**2 - 2 * org_ell * a_ell * np.cos(theta3) + a_ell**2) / (a_ell - org_ell * np.cos(theta3))
    return np.arcsin((2 * a_ell - l4) * np.sin(theta3) / l4)


def _col_mean(p):
    """np.mean(center[:, 1:], axis=1) of a (3, k) centre array"""
    return np.mean(p[:, 1:], axis=1)


class BuiltSystem(dict):
    """What build_akb returns: the SystemGeometry fields plus the driver's derived values."""


def build_akb(params, *, source_shift=(0.0, 0.0, 0.0), option_set=True, prims=None, design=AKBDesign,
              name=None):
    """plot_result_debug's system for params (26 floats), AKB_raytrace_20250312.py:1764-2717.

    Returns a dict with the SystemGeometry fields (mirrors in trace order V-hyperbola, V-ellipse,
    H-ellipse, H-hyperbola; det1 / det2 planes as 10 coefficients; angle_h / angle_v ranges of
    the launch grid; source) plus s2f_middle, or np.inf where the reference returns np.inf (a
    non-real centre, :1912, :1933, :2253, :2295, :2339, :2380; mirrors out of order, :2418-2426).
    option_set: the module flag choosing the misalignment centres (:2459).
    """
    if prims is None:
        from . import primitives as prims
    D = design
    p = [np.float64(x) for x in np.asarray(params, dtype=np.float64).ravel()]
    if len(p) != 26:
        raise ValueError("params must hold 26 values")
    (defocus, astigH,
     pitch_hyp_v, roll_hyp_v, yaw_hyp_v, decX_hyp_v, decY_hyp_v, decZ_hyp_v,
     pitch_hyp_h, roll_hyp_h, yaw_hyp_h, decX_hyp_h, decY_hyp_h, decZ_hyp_h,
     pitch_ell_v, roll_ell_v, yaw_ell_v, decX_ell_v, decY_ell_v, decZ_ell_v,
     pitch_ell_h, roll_ell_h, yaw_ell_h, decX_ell_h, decY_ell_h, decZ_ell_h) = p
    a_hyp_v, b_hyp_v, a_ell_v, b_ell_v = D.a_hyp_v, D.b_hyp_v, D.a_ell_v, D.b_ell_v
    a_hyp_h, b_hyp_h, a_ell_h, b_ell_h = D.a_hyp_h, D.b_hyp_h, D.a_ell_h, D.b_ell_h
    theta1_v, theta1_h = D.theta1_v, D.theta1_h
    length_hyp_v, length_ell_h = D.hyp_length_v, D.ell_length_h

    org_hyp_v = np.sqrt(a_hyp_v**2 + b_hyp_v**2)
    org_hyp_h = np.sqrt(a_hyp_h**2 + b_hyp_h**2)
    org_ell_v = np.sqrt(a_ell_v**2 - b_ell_v**2)
    org_ell_h = np.sqrt(a_ell_h**2 - b_ell_h**2)
    zero1 = np.array([[0.], [0.], [0.]])

    # mirror apertures seen from the source (:1902-1942)
    c_v = np.zeros(10)
    c_v[0] = 1 / a_hyp_v**2
    c_v[2] = -1 / b_hyp_v**2
    c_v[9] = -1.
    c_v = shift_x(c_v, np.sqrt(a_hyp_v**2 + b_hyp_v**2))
    center_v = prims.mirr_ray_intersection(c_v, np.array([[np.cos(theta1_v)], [0.], [np.sin(theta1_v)]]), zero1)
    if not np.isreal(center_v).all():
        return np.inf
    x1_v = center_v[0, 0] - length_hyp_v / 2
    x2_v = center_v[0, 0] + length_hyp_v / 2
    y1_v = _calc_y_hyp(a_hyp_v, b_hyp_v, x1_v)
    y2_v = _calc_y_hyp(a_hyp_v, b_hyp_v, x2_v)
    c_h = np.zeros(10)
    c_h[0] = 1 / a_ell_h**2
    c_h[1] = 1 / b_ell_h**2
    c_h[9] = -1.
    c_h = shift_x(c_h, np.sqrt(a_ell_h**2 - b_ell_h**2))
    center_h = prims.mirr_ray_intersection(c_h, np.array([[np.cos(theta1_h)], [np.sin(theta1_h)], [0.]]), zero1)
    if not np.isreal(center_h).all():
        return np.inf
    x1_h = center_h[0, 0] - length_ell_h / 2
    x2_h = center_h[0, 0] + length_ell_h / 2
    y1_h = _calc_y_ell(a_ell_h, b_ell_h, x1_h)
    y2_h = _calc_y_ell(a_ell_h, b_ell_h, x2_h)

    # 1st: V hyperbola, on axis then tilted by theta1_v (:1976-1989)
    axis_x, axis_y, axis_z = np.array([1., 0., 0.]), np.array([0., 1., 0.]), np.array([0., 0., 1.])
    hyp_v = np.zeros(10)
    hyp_v[0] = 1 / a_hyp_v**2
    hyp_v[2] = -1 / b_hyp_v**2
    hyp_v[9] = -1.
    hyp_v = shift_x(hyp_v, org_hyp_v)
    hyp_v, R = rotate_general_axis(hyp_v, axis_y, theta1_v, [0, 0, 0])
    axis_x, axis_y, axis_z = rotatematrix(R, axis_x, axis_y, axis_z)

    # alignment rays: the V aperture's two edge rays and its centre (:1991-2176); the Wolter III
    # exit angles of the two edges give the horizontal pair's tilt omega_v (:2047-2051)
    at1_v, at2_v = np.arctan(y1_v / x1_v), np.arctan(y2_v / x2_v)
    theta_cntr_v = (np.arctan(y2_v / x2_v) + np.arctan(y1_v / x1_v)) / 2.
    th5_v1 = _wolter3_theta5(a_hyp_v, b_hyp_v, org_hyp_v, a_ell_v, b_ell_v, org_ell_v, at1_v)
    th5_v2 = _wolter3_theta5(a_hyp_v, b_hyp_v, org_hyp_v, a_ell_v, b_ell_v, org_ell_v, at2_v)
    omega_v = (th5_v1 + th5_v2 + np.arctan(y1_v / x1_v) + np.arctan(y2_v / x2_v)) / 2
    bufray = np.zeros((3, 3))
    bufray[0, 0] = 1.
    bufray[0, 1] = 1.
    bufray[2, 1] = np.tan(np.arctan(y1_v / x1_v) - theta_cntr_v)
    bufray[0, 2] = 1.
    bufray[2, 2] = np.tan(np.arctan(y2_v / x2_v) - theta_cntr_v)
    source = np.zeros((3, 3))
    bufray = prims.normalize_vector(bufray)

    center_hyp_v = prims.mirr_ray_intersection(hyp_v, bufray, source)
    if not np.isreal(center_hyp_v).all():
        return np.inf
    refl1 = prims.reflect_ray(bufray, prims.norm_vector(hyp_v, center_hyp_v))

    # 2nd: V ellipse (:2272-2310)
    axis2_x, axis2_y, axis2_z = np.array([1., 0., 0.]), np.array([0., 1., 0.]), np.array([0., 0., 1.])
    ell_v = np.zeros(10)
    ell_v[0] = 1 / a_ell_v**2
    ell_v[2] = 1 / b_ell_v**2
    ell_v[9] = -1.
    ell_v = shift_x(ell_v, 2 * org_hyp_v + org_ell_v)
    ell_v, R = rotate_general_axis(ell_v, axis2_y, theta1_v, [0, 0, 0])
    axis2_x, axis2_y, axis2_z = rotatematrix(R, axis2_x, axis2_y, axis2_z)
    center_ell_v = prims.mirr_ray_intersection(ell_v, refl1, center_hyp_v)
    if not np.isreal(center_ell_v).all():
        return np.inf
    refl2 = prims.reflect_ray(refl1, prims.norm_vector(ell_v, center_ell_v))

    # 3rd: H ellipse, shifted by astigH, tilted by -theta1_h, then by omega_v about the V
    # ellipse's alignment centre (:2323-2352)
    axis3_x, axis3_y, axis3_z = np.array([1., 0., 0.]), np.array([0., 1., 0.]), np.array([0., 0., 1.])
    ell_h = np.zeros(10)
    ell_h[0] = 1 / a_ell_h**2
    ell_h[1] = 1 / b_ell_h**2
    ell_h[9] = -1.
    ell_h = shift_x(ell_h, org_ell_h + astigH)
    ell_h, R = rotate_general_axis(ell_h, axis3_z, -theta1_h, [0, 0, 0])
    axis3_x, axis3_y, axis3_z = rotatematrix(R, axis3_x, axis3_y, axis3_z)
    center_ell_h = prims.mirr_ray_intersection(ell_h, refl2, center_ell_v)
    if not np.isreal(center_ell_h).all():
        return np.inf
    ell_h, R = rotate_general_axis(ell_h, axis3_y, omega_v, _col_mean(center_ell_v))
    axis3_x, axis3_y, axis3_z = rotatematrix(R, axis3_x, axis3_y, axis3_z)
    center_ell_h = prims.mirr_ray_intersection(ell_h, refl2, center_ell_v)
    refl3 = prims.reflect_ray(refl2, prims.norm_vector(ell_h, center_ell_h))

    # 4th: H hyperbola, minus root (:2364-2394)
    axis4_x, axis4_y, axis4_z = np.array([1., 0., 0.]), np.array([0., 1., 0.]), np.array([0., 0., 1.])
    hyp_h = np.zeros(10)
    hyp_h[0] = 1 / a_hyp_h**2
    hyp_h[1] = -1 / b_hyp_h**2
    hyp_h[9] = -1.
    hyp_h = shift_x(hyp_h, -org_hyp_h + 2 * org_ell_h + astigH)
    hyp_h, R = rotate_general_axis(hyp_h, axis4_z, -theta1_h, [0, 0, 0])
    axis4_x, axis4_y, axis4_z = rotatematrix(R, axis4_x, axis4_y, axis4_z)
    center_hyp_h = prims.mirr_ray_intersection(hyp_h, refl3, center_ell_h, negative=True)
    if not np.isreal(center_hyp_h).all():
        return np.inf
    hyp_h, R = rotate_general_axis(hyp_h, axis4_y, omega_v, _col_mean(center_ell_v))
    axis4_x, axis4_y, axis4_z = rotatematrix(R, axis4_x, axis4_y, axis4_z)
    center_hyp_h = prims.mirr_ray_intersection(hyp_h, refl3, center_ell_h, negative=True)

    # detector (:2396-2403) and the mirrors' order along the beam (:2418-2426)
    s2f_H = -2 * org_hyp_h + 2 * org_ell_h
    s2f_V = 2 * org_hyp_v + 2 * org_ell_v
    s2f_middle = (s2f_H + s2f_V) / 2
    if center_ell_v[0, 0] < center_hyp_v[0, 0] or center_ell_h[0, 0] < center_ell_v[0, 0] \
            or center_hyp_h[0, 0] < center_ell_h[0, 0]:
        return np.inf

    # misalignment (:2458-2616): rotations about the mirrors' local axes (the axes are not
    # carried along by these), then decenters along them
    if option_set:
        c_wh = (_col_mean(center_ell_h) + _col_mean(center_hyp_h)) / 2
        if pitch_ell_h != 0:
            ell_h, _ = rotate_general_axis(ell_h, axis3_y, pitch_ell_h, c_wh)
        if yaw_ell_h != 0:
            ell_h, _ = rotate_general_axis(ell_h, axis3_z, yaw_ell_h, c_wh)
        if roll_ell_h != 0:
            ell_h, _ = rotate_general_axis(ell_h, axis3_x, roll_ell_h, c_wh)
        if pitch_hyp_h != 0:
            hyp_h, _ = rotate_general_axis(hyp_h, axis4_y, pitch_hyp_h, c_wh)
        if yaw_hyp_h != 0:
            hyp_h, _ = rotate_general_axis(hyp_h, axis4_z, yaw_hyp_h, c_wh)
        if roll_hyp_h != 0:
            hyp_h, _ = rotate_general_axis(hyp_h, axis4_x, roll_hyp_h, c_wh)
        c_wv = (_col_mean(center_ell_v) + _col_mean(center_hyp_v)) / 2
        # the V pair moves with its hyperbola; the ellipse then by its relative angles
        if yaw_hyp_v != 0:
            hyp_v, _ = rotate_general_axis(hyp_v, axis_z, yaw_hyp_v, c_wv)
            ell_v, _ = rotate_general_axis(ell_v, axis2_z, yaw_hyp_v, c_wv)
        if pitch_hyp_v != 0:
            hyp_v, _ = rotate_general_axis(hyp_v, axis_y, pitch_hyp_v, c_wv)
            ell_v, _ = rotate_general_axis(ell_v, axis2_y, pitch_hyp_v, c_wv)
        if roll_hyp_v != 0:
            hyp_v, _ = rotate_general_axis(hyp_v, axis_x, roll_hyp_v, c_wv)
            ell_v, _ = rotate_general_axis(ell_v, axis2_x, roll_hyp_v, c_wv)
        rel_yaw = yaw_ell_v - yaw_hyp_v
        rel_pitch = pitch_ell_v - pitch_hyp_v
        rel_roll = roll_ell_v - roll_hyp_v
        if rel_yaw != 0:
            ell_v, _ = rotate_general_axis(ell_v, axis2_z, rel_yaw, _col_mean(center_ell_v))
        if rel_pitch != 0:
            ell_v, _ = rotate_general_axis(ell_v, axis2_y, rel_pitch, _col_mean(center_ell_v))
        if rel_roll != 0:
            ell_v, _ = rotate_general_axis(ell_v, axis2_x, rel_roll, _col_mean(center_ell_v))
    else:
        c_ev, c_hv = _col_mean(center_ell_v), _col_mean(center_hyp_v)
        c_eh, c_hh = _col_mean(center_ell_h), _col_mean(center_hyp_h)
        if yaw_ell_v != 0:
            ell_v, _ = rotate_general_axis(ell_v, axis2_z, yaw_ell_v, c_ev)
        if pitch_ell_v != 0:
            ell_v, _ = rotate_general_axis(ell_v, axis2_y, pitch_ell_v, c_ev)
        if roll_ell_v != 0:
            ell_v, _ = rotate_general_axis(ell_v, axis2_x, roll_ell_v, c_ev)
        if yaw_hyp_v != 0:
            hyp_v, _ = rotate_general_axis(hyp_v, axis_z, yaw_hyp_v, c_hv)
        if pitch_hyp_v != 0:
            hyp_v, _ = rotate_general_axis(hyp_v, axis_y, pitch_hyp_v, c_hv)
        if roll_hyp_v != 0:
            hyp_v, _ = rotate_general_axis(hyp_v, axis_x, roll_hyp_v, c_hv)
        if pitch_ell_h != 0:
            ell_h, _ = rotate_general_axis(ell_h, axis3_y, pitch_ell_h, c_eh)
        if yaw_ell_h != 0:
            ell_h, _ = rotate_general_axis(ell_h, axis3_z, yaw_ell_h, c_eh)
        if roll_ell_h != 0:
            ell_h, _ = rotate_general_axis(ell_h, axis3_x, roll_ell_h, c_eh)
        if pitch_hyp_h != 0:
            hyp_h, _ = rotate_general_axis(hyp_h, axis4_y, pitch_hyp_h, c_hh)
        if yaw_hyp_h != 0:
            hyp_h, _ = rotate_general_axis(hyp_h, axis4_z, yaw_hyp_h, c_hh)
        if roll_hyp_h != 0:
            hyp_h, _ = rotate_general_axis(hyp_h, axis4_x, roll_hyp_h, c_hh)
    for s, ax in ((decX_hyp_v, axis_x), (decY_hyp_v, axis_y), (decZ_hyp_v, axis_z)):
        if s != 0:
            hyp_v = shift_along(hyp_v, s, ax)
    for s, ax in ((decX_hyp_h, axis4_x), (decY_hyp_h, axis4_y), (decZ_hyp_h, axis4_z)):
        if s != 0:
            hyp_h = shift_along(hyp_h, s, ax)
    for s, ax in ((decX_ell_v, axis2_x), (decY_ell_v, axis2_y), (decZ_ell_v, axis2_z)):
        if s != 0:
            ell_v = shift_along(ell_v, s, ax)
    for s, ax, sw in ((decX_ell_h, axis3_x, False), (decY_ell_h, axis3_y, False), (decZ_ell_h, axis3_z, True)):
        if s != 0:
            ell_h = shift_along(ell_h, s, ax, swapped=sw)

    # launch grid (:2694-2700): angles from the (shifted) source to the aperture edges
    ss = [np.float64(x) for x in source_shift]
    start_h = np.arctan((y1_h - ss[1]) / (x1_h - ss[0]))
    stop_h = np.arctan((y2_h - ss[1]) / (x2_h - ss[0]))
    start_v = np.arctan((y1_v - ss[2]) / (x1_v - ss[0]))
    stop_v = np.arctan((y2_v - ss[2]) / (x2_v - ss[0]))
    det1 = np.zeros(10)
    det1[6] = 1.
    det1[9] = -(s2f_middle + defocus)
    det2 = np.zeros(10)
    det2[6] = 1.
    det2[9] = -(s2f_middle + defocus + D.defocus_wave)
    src = [0.0 + ss[0], 0.0 + ss[1], 0.0 + ss[2]]  # np.zeros + source_shift (:2688-2691)
    return BuiltSystem(
        name=name or "AKB Wolter III+I Setting12/setting11 (built from params)",
        mirrors=[dict(coeffs=[float(x) for x in c], negative=neg)
                 for c, neg in ((hyp_v, False), (ell_v, False), (ell_h, False), (hyp_h, True))],
        det1=[float(x) for x in det1], det2=[float(x) for x in det2],
        angle_h=dict(start=float(start_h), stop=float(stop_h), offset=float(theta1_h)),
        angle_v=dict(start=float(start_v), stop=float(stop_v), offset=float(theta1_v)),
        source=[float(x) for x in src], wavelength_m=D.wavelength_m, defocus_wave_m=D.defocus_wave,
        s2f_middle=float(s2f_middle), defocus=float(defocus),
        meta=dict(option_set=bool(option_set), params=[float(x) for x in p]),
    )


def mirrors_of(built):
    """The trace-order Mirror list of a build_akb result."""
    return [Mirror(m["coeffs"], m["negative"]) for m in built["mirrors"]]


# ---------------------------------------------------------------- the KB pair (KB_debug)

# KBdesign_7params (AKB_raytrace_20250312.py:100): l1h, l2h, inc_h, mlen_h, wd_v, inc_v, mlen_v
KB_DESIGN_7PARAMS = (np.float64(146.), np.float64(0.21), np.float64(0.16742), np.float64(0.180), np.float64(0.030),
                     np.float64(0.15525), np.float64(0.05))


def rotate_x(coeffs, theta, center):
    """:669-693"""
    a, b, c, d, e, f, g, h, i, j = shift_z(shift_y(shift_x(coeffs, -center[0]), -center[1]), -center[2])
    Cos, Sin = np.cos(theta), np.sin(theta)
    out = [a, b * Cos**2 + c * Sin**2 - f * Sin * Cos, b * Sin**2 + c * Cos**2 + f * Sin * Cos, d * Cos - e * Sin,
           d * Sin + e * Cos, b * np.sin(2 * theta) - c * np.sin(2 * theta) + f * np.cos(2 * theta), g,
           h * Cos - i * Sin, h * Sin + i * Cos, j]
    return shift_z(shift_y(shift_x(out, center[0]), center[1]), center[2])


def rotate_y(coeffs, theta, center):
    """:695-719"""
    a, b, c, d, e, f, g, h, i, j = shift_z(shift_y(shift_x(coeffs, -center[0]), -center[1]), -center[2])
    Cos, Sin = np.cos(theta), np.sin(theta)
    out = [a * Cos**2 + c * Sin**2 + e * Sin * Cos, b, a * Sin**2 + c * Cos**2 - e * Sin * Cos, d * Cos + f * Sin,
           -a * np.sin(2 * theta) + c * np.sin(2 * theta) + e * np.cos(2 * theta), -d * Sin + f * Cos,
           g * Cos + i * Sin, h, i * Cos - g * Sin, j]
    return shift_z(shift_y(shift_x(out, center[0]), center[1]), center[2])


def rotate_z(coeffs, theta, center):
    """:721-745"""
    a, b, c, d, e, f, g, h, i, j = shift_z(shift_y(shift_x(coeffs, -center[0]), -center[1]), -center[2])
    Cos, Sin = np.cos(theta), np.sin(theta)
    out = [a * Cos**2 + b * Sin**2 - d * Sin * Cos, b * Cos**2 + a * Sin**2 + d * Sin * Cos, c,
           a * np.sin(2 * theta) - b * np.sin(2 * theta) + d * np.cos(2 * theta), e * Cos - f * Sin,
           e * Sin + f * Cos, g * Cos - h * Sin, g * Sin + h * Cos, i, j]
    return shift_z(shift_y(shift_x(out, center[0]), center[1]), center[2])


def ell_define(l1, inc, l2):
    """Ell_define (:272-281)"""
    sita1 = np.arctan(l2 * np.sin(2. * inc) / (l1 + l2 * np.cos(2. * inc)))
    a_ell = (l1 + l2) / 2.
    b_ell = np.sqrt(l1 * l2 * np.sin(inc) ** 2)
    sita3 = np.arcsin(l1 * np.sin(sita1) / l2)
    return a_ell, b_ell, sita1, sita3


def kb_define(l1h, l2h, inc_h, mlen_h, wd_v, inc_v, mlen_v):
    """KB_define (:297-336): the two ellipses of a KB pair sharing one focus; the V ellipse's source
    distance found by the reference's fixed-point iteration. Returns the reference's tuple."""
    a_h, b_h, sita1h, sita3h = ell_define(l1h, inc_h, l2h)
    s2f_h = np.sqrt(a_h**2. - b_h**2.) * 2.
    xh_s = l1h * np.cos(sita1h) - mlen_h / 2.
    xh_e = l1h * np.cos(sita1h) + mlen_h / 2.
    yh_s = _calc_y_ell(a_h, b_h, xh_s)
    yh_e = _calc_y_ell(a_h, b_h, xh_e)
    accept_h = np.abs(yh_e - yh_s)
    NA_h = np.sin(np.abs(np.arctan(yh_e / (s2f_h - xh_e)) - np.arctan(yh_s / (s2f_h - xh_s)))) / 2.
    l1v = l1h + (l2h - wd_v - mlen_v / 2.)
    l2v = wd_v + mlen_v / 2.
    while True:
        a_v, b_v, sita1v, sita3v = ell_define(l1v, inc_v, l2v)
        s2f_v = np.sqrt(a_v**2. - b_v**2.) * 2.
        diff = s2f_h - s2f_v
        if np.abs(diff) < 1e-9:
            break
        l1v += diff * 0.9
    xv_s = l1v * np.cos(sita1v) - mlen_v / 2.
    xv_e = l1v * np.cos(sita1v) + mlen_v / 2.
    yv_s = _calc_y_ell(a_v, b_v, xv_s)
    yv_e = _calc_y_ell(a_v, b_v, xv_e)
    accept_v = np.abs(yv_e - yv_s)
    NA_v = np.sin(np.abs(np.arctan(yv_e / (s2f_v - xv_e)) - np.arctan(yv_s / (s2f_v - xv_s)))) / 2.
    gap = xv_s - xh_e
    return a_h, b_h, a_v, b_v, l1v, l2v, [xh_s, xh_e, yh_s, yh_e, sita1h, sita3h, accept_h, NA_h, xv_s, xv_e, yv_s,
                                          yv_e, sita1v, sita3v, accept_v, NA_v, s2f_h, diff, gap]


def _ell_theta5(a, org, theta1):
    """theta5 of KB_debug's print_optical_design (:10463-10493), the only output it uses."""
    l4 = ((org)**2 - 2 * org * a * np.cos(theta1) + a**2) / (a - org * np.cos(theta1))
    return np.arcsin((2 * a - l4) * np.sin(theta1) / l4)


def build_kb(params, *, source_shift=(0.0, 0.0, 0.0), designparams=None, prims=None, name=None):
    """KB_debug's system for params (26 floats) with its live flags (optKBdesign False,
    option_HighNA True, option_axial / option_alignment / optin_axialrotation /
    optionLocalRotation True, optionLocalRotationonlyAll False: :9742-10935): the V and H
    ellipses of KB_define from KBdesign_7params (or designparams), aligned on five centre rays,
    then params' misalignments (pitch / roll / yaw of the V mirror about its centre ray's hit, of the
    H mirror about its local axes through its corner rays' mean hit; decenters). Returns a dict
    with the SystemGeometry fields (two mirrors, det1, launch-angle ranges, source) plus
    s2f_middle and defocus, or np.inf where the reference returns np.inf."""
    if prims is None:
        from . import primitives as prims
    p = [np.float64(x) for x in np.asarray(params, dtype=np.float64).ravel()]
    if len(p) != 26:
        raise ValueError("params must hold 26 values")
    (defocus, astigH,
     pitch_hyp_v, roll_hyp_v, yaw_hyp_v, decX_hyp_v, decY_hyp_v, decZ_hyp_v,
     pitch_hyp_h, roll_hyp_h, yaw_hyp_h, decX_hyp_h, decY_hyp_h, decZ_hyp_h) = p[:14]
    l1h, l2h, inc_h, mlen_h, wd_v, inc_v, mlen_v = (KB_DESIGN_7PARAMS if designparams is None
                                                     else [np.float64(x) for x in designparams])
    a_h, b_h, a_v, b_v, l1v, l2v, rest = kb_define(l1h, l2h, inc_h, mlen_h, wd_v, inc_v, mlen_v)
    xh_s, xh_e, yh_s, yh_e, sita1h, sita3h, _, _, xv_s, xv_e, yv_s, yv_e, sita1v = rest[:13]
    a_hyp_v, b_hyp_v, a_hyp_h, b_hyp_h = a_h, b_h, a_v, b_v
    org_hyp_v = np.sqrt(a_hyp_v**2 - b_hyp_v**2)
    org_hyp_h = np.sqrt(a_hyp_h**2 - b_hyp_h**2)
    y1_v, x1_v, y2_v, x2_v = yh_s, xh_s, yh_e, xh_e
    y1_h, x1_h, y2_h, x2_h = yv_s, xv_s, yv_e, xv_e
    theta1_v, theta1_h = sita1h, sita1v

    # V mirror (:10432-10447)
    axis_x, axis_y, axis_z = np.float64([1., 0., 0.]), np.float64([0., 1., 0.]), np.float64([0., 0., 1.])
    hyp_v = np.zeros(10)
    hyp_v[0] = 1 / a_hyp_v**2
    hyp_v[2] = 1 / b_hyp_v**2
    hyp_v[9] = -1.
    hyp_v = shift_x(hyp_v, org_hyp_v)
    hyp_v, R = rotate_general_axis(hyp_v, axis_y, theta1_v, [0., 0., 0.])
    axis_x, axis_y, axis_z = rotatematrix(R, axis_x, axis_y, axis_z)

    # the five alignment rays (:10458-10609): the centre and four corners
    at1h, at2h = np.arctan(y1_h / x1_h), np.arctan(y2_h / x2_h)
    at1v, at2v = np.arctan(y1_v / x1_v), np.arctan(y2_v / x2_v)
    theta_cntr_h = (at2h + at1h) / 2.
    theta_cntr_v = (at2v + at1v) / 2.
    theta5_v1 = _ell_theta5(a_hyp_v, org_hyp_v, at1v)
    theta5_v2 = _ell_theta5(a_hyp_v, org_hyp_v, at2v)
    omega_V = ((at1v + at2v) + theta5_v1 + theta5_v2) / 2
    ts1h, ts2h = at1h - theta_cntr_h, at2h - theta_cntr_h
    ts1v, ts2v = at1v - theta_cntr_v, at2v - theta_cntr_v
    bufray = np.zeros((3, 5))
    bufray[0, :] = 1.
    bufray[1, 0], bufray[2, 0] = np.tan(theta1_h), np.tan(theta1_v)
    bufray[1, 1], bufray[2, 1] = np.tan(ts1h), np.tan(ts1v)
    bufray[1, 2], bufray[2, 2] = np.tan(ts2h), np.tan(ts1v)
    bufray[1, 3], bufray[2, 3] = np.tan(ts2h), np.tan(ts1v)
    bufray[1, 4], bufray[2, 4] = np.tan(ts2h), np.tan(ts2v)
    source = np.zeros((3, 5))
    bufray = prims.normalize_vector(bufray)
    center_hyp_v = prims.mirr_ray_intersection(hyp_v, bufray, source)
    if not np.isreal(center_hyp_v).all():
        return np.inf
    refl1 = prims.reflect_ray(bufray, prims.norm_vector(hyp_v, center_hyp_v))

    # H mirror (:10808-10847)
    hyp_h = np.zeros(10)
    hyp_h[0] = 1 / a_hyp_h**2
    hyp_h[1] = 1 / b_hyp_h**2
    hyp_h[9] = -1.
    hyp_h = shift_x(hyp_h, org_hyp_h + astigH)
    ax2, ay2, az2 = np.float64([1., 0., 0.]), np.float64([0., 1., 0.]), np.float64([0., 0., 1.])
    ay_g, az_g = np.float64([0., 1., 0.]), np.float64([0., 0., 1.])
    hyp_h, R = rotate_general_axis(hyp_h, az_g, -theta1_h, [0, 0, 0])
    ax2, ay2, az2 = rotatematrix(R, ax2, ay2, az2)
    center_hyp_h = prims.mirr_ray_intersection(hyp_h, refl1, center_hyp_v)
    if not np.isreal(center_hyp_h).all():
        return np.inf
    hyp_h, R = rotate_general_axis(hyp_h, ay_g, omega_V, _col_mean(center_hyp_h))
    ax2, ay2, az2 = rotatematrix(R, ax2, ay2, az2)
    center_hyp_h = prims.mirr_ray_intersection(hyp_h, refl1, center_hyp_v)

    s2f_middle = (2 * org_hyp_h + 2 * org_hyp_v) / 2  # (s2f_H + s2f_V) / 2, :10862-10866

    # misalignments (:10898-10934)
    cv = center_hyp_v[:, 0]
    if pitch_hyp_v != 0:
        hyp_v = rotate_y(hyp_v, pitch_hyp_v, cv)
    if roll_hyp_v != 0:
        hyp_v = rotate_x(hyp_v, roll_hyp_v, cv)
    if yaw_hyp_v != 0:
        hyp_v = rotate_z(hyp_v, yaw_hyp_v, cv)
    ch = _col_mean(center_hyp_h)
    if pitch_hyp_h != 0:
        hyp_h, _ = rotate_general_axis(hyp_h, ay2, pitch_hyp_h, ch)
    if yaw_hyp_h != 0:
        hyp_h, _ = rotate_general_axis(hyp_h, az2, yaw_hyp_h, ch)
    if roll_hyp_h != 0:
        hyp_h, _ = rotate_general_axis(hyp_h, ax2, roll_hyp_h, ch)
    for s, f in ((decX_hyp_v, shift_x), (decY_hyp_v, shift_y), (decZ_hyp_v, shift_z)):
        if s != 0:
            hyp_v = f(hyp_v, s)
    for s, f in ((decX_hyp_h, shift_x), (decY_hyp_h, shift_y), (decZ_hyp_h, shift_z)):
        if s != 0:
            hyp_h = f(hyp_h, s)

    # launch grid (:10948-10956): angles from the shifted source, centred on the unshifted edges'
    ss = [np.float64(x) for x in source_shift]
    det1 = np.zeros(10)
    det1[6] = 1.
    det1[9] = -(s2f_middle + defocus)
    return BuiltSystem(
        name=name or "KB_debug pair (KB_define of KBdesign_7params, built from params)",
        mirrors=[dict(coeffs=[float(x) for x in hyp_v], negative=False),
                 dict(coeffs=[float(x) for x in hyp_h], negative=False)],
        det1=[float(x) for x in det1],
        angle_h=dict(start=float(np.arctan((y1_h - ss[1]) / (x1_h - ss[0]))),
                     stop=float(np.arctan((y2_h - ss[1]) / (x2_h - ss[0]))), offset=float(np.mean([at1h, at2h]))),
        angle_v=dict(start=float(np.arctan((y1_v - ss[2]) / (x1_v - ss[0]))),
                     stop=float(np.arctan((y2_v - ss[2]) / (x2_v - ss[0]))), offset=float(np.mean([at1v, at2v]))),
        source=[0.0 + ss[0], 0.0 + ss[1], 0.0 + ss[2]],
        s2f_middle=float(s2f_middle), defocus=float(defocus),
        meta=dict(params=[float(x) for x in p], design=[float(x) for x in (l1h, l2h, inc_h, mlen_h, wd_v, inc_v,
                                                                          mlen_v)]),
    )
