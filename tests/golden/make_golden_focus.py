"""Record the reference's focus sweep find_defocus (AKB_raytrace_20250312.py:9086-9170) on the
65x65 'ray_wave' pass-2 rays (build container only; the reference never travels):

    python tests/golden/make_golden_focus.py

The rays are the reference's own: its primitives re-run on the pass-2 directions recorded in
akb_raywave_65.npz (reflect4 and the last hit, as :2893-2900 form them). Writes
akb_focus_65.npz: reflect4, points, s2f_middle, the first loop's size_h_ / size_v_ (np.std of
the detector hit's y / z over the 50 planes) and find_defocus's result.
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import make_golden as MG  # noqa: E402


def main():
    MG._stub_modules()
    sys.path.insert(0, MG.REF)
    import json
    import tempfile
    os.chdir(tempfile.mkdtemp(prefix="akb_golden_focus_"))
    import AKB_raytrace_20250312 as A
    with open(os.path.join(MG.OUT, "akb_geometry.json")) as f:
        g = json.load(f)
    f = np.load(os.path.join(MG.OUT, "akb_raywave_65.npz"))
    ray = f["pass2_dir"]
    src = np.zeros_like(ray)
    for m in g["mirrors"]:
        p = A.mirr_ray_intersection(np.array(m["coeffs"]), ray, src, negative=m["negative"])
        ray = A.reflect_ray(ray, A.norm_vector(np.array(m["coeffs"]), p))
        src = p
    s2f = -g["det1"][9]  # the ray_wave detector plane x = s2f_middle + defocus (defocus 0 here)
    # the first loop's sizes, exactly as find_defocus forms them
    a = np.linspace(-0.3, 0.3, 50)
    size_h, size_v = np.zeros(50), np.zeros(50)
    for i in range(50):
        c = np.zeros(10)
        c[6] = 1
        c[9] = -(s2f + a[i])
        det = A.plane_ray_intersection(c, ray, src)
        size_v[i] = np.std(det[2, :])
        size_h[i] = np.std(det[1, :])
    best = A.find_defocus(ray, src, s2f, 0.0, 65)
    np.savez_compressed(os.path.join(MG.OUT, "akb_focus_65.npz"), reflect4=ray, points=src, s2f_middle=np.float64(s2f),
                        size_h0=size_h, size_v0=size_v, best_a=np.float64(best))
    print("best_a", best)


if __name__ == "__main__":
    main()
