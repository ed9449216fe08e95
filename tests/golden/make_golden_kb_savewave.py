"""Record KB_debug's 'wave' mode and saveWaveData's KB file set (AKB_raytrace_20250312.py:11629-11701,
:13475-13764), build container only:

    python tests/golden/make_golden_kb_savewave.py

With option_AKB False, saveWaveData(initial_params) runs KB_debug(params, 1, 1, 'wave') (:13485) on
the wave_num_H x wave_num_V grid (reset_p0's resample, the np.mean tilt, both mirror grids and the
source rotated about np.mean(detcenter), the re-intersected detector and the defocusForWave plane),
optionally thins the grids, adds calc_dS and writes points_source.npy, points_M1/M2.npy,
points_gridImage.npy, points_gridDefocus.npy and calculation_conditions.txt. Recorded at 33 x 33
(defocusForWave = 1e-3, :89) for params = kb_build.npz's case 1 (misaligned): the 'wave' tuple of
a direct KB_debug call (w_*), and saveWaveData's files without thinning and with every grid thinned
once (factors 2). Writes kb_savewave_33.npz.
"""
import contextlib
import glob
import io
import os
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import make_golden as MG  # noqa: E402

FILES = ["points_source.npy", "points_M1.npy", "points_M2.npy", "points_gridImage.npy", "points_gridDefocus.npy"]
RUNS = {"plain": (0, 0, 0, 0, 0, 0), "thin": (2, 2, 2, 2, 2, 2)}
WAVE = ("source", "vmirr_hyp", "hmirr_hyp", "detcenter", "detcenter2", "ray_num_H", "ray_num_V", "vmirr_norm",
        "hmirr_norm", "vec0to1", "vec1to2")


def main():
    MG._stub_modules()
    sys.path.insert(0, MG.REF)
    work = tempfile.mkdtemp(prefix="akb_golden_kbsavewave_")
    os.chdir(work)
    import AKB_raytrace_20250312 as A
    A.option_AKB = False
    A.wave_num_H = A.wave_num_V = 33
    params = np.load(os.path.join(MG.OUT, "kb_build.npz"))["k1_params"].copy()
    out = {"defocusForWave": np.float64(A.defocusForWave), "params": params}
    with contextlib.redirect_stdout(io.StringIO()):
        r = A.KB_debug(params.copy(), 1, 1, "wave")
    for name, v in zip(WAVE, r):
        out[f"w_{name}"] = np.array(v)
    for name, ds in RUNS.items():
        (A.downsample_h1, A.downsample_v1, A.downsample_h2, A.downsample_v2, A.downsample_h_f,
         A.downsample_v_f) = ds
        run_dir = os.path.join(work, name)
        os.makedirs(run_dir)
        os.chdir(run_dir)
        try:
            with contextlib.redirect_stdout(io.StringIO()):
                A.saveWaveData(params.copy())
        except SystemExit:
            pass
        folder = glob.glob(os.path.join(run_dir, "output_*"))
        folder = [d for d in folder if os.path.exists(os.path.join(d, "calculation_conditions.txt"))]
        assert len(folder) == 1, folder
        for fn in FILES:
            out[f"{name}_{fn[:-4]}"] = np.load(os.path.join(folder[0], fn))
        assert not os.path.exists(os.path.join(folder[0], "points_M3.npy"))
        with open(os.path.join(folder[0], "calculation_conditions.txt")) as f:
            out[f"{name}_conditions"] = np.array(f.read())
        out[f"{name}_downsample"] = np.array(ds)
        print(name, out[f"{name}_points_M1"].shape, out[f"{name}_points_gridImage"].shape)
    A.option_AKB = True
    np.savez_compressed(os.path.join(MG.OUT, "kb_savewave_33.npz"), **out)
    print("wrote kb_savewave_33.npz")


if __name__ == "__main__":
    main()
