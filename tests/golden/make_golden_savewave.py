"""Record the reference's saveWaveData file set (AKB_raytrace_20250312.py:13475-13764), build
container only:

    python tests/golden/make_golden_savewave.py

saveWaveData(initial_params) runs plot_result_debug(params, 'wave') (:3510-3561) on the
wave_num_H x wave_num_V grid, optionally thins the grids (downsample_array_3_n, :13336, module
flags downsample_h1 .. downsample_v_f), adds calc_dS area elements and writes points_source.npy,
points_M1..M4.npy, points_gridImage.npy, points_gridDefocus.npy and calculation_conditions.txt
into output_<timestamp>/, then calls sys.exit(). Two runs at the best-alignment params on a
33 x 33 grid (option_set=True, defocusForWave = 1e-3 as the module sets it, :89): without
thinning, and with every grid thinned once (downsample factors 2 -> 17 x 17). Every file is kept
(the conditions text with its time line) in savewave_33.npz.
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

FILES = ["points_source.npy", "points_M1.npy", "points_M2.npy", "points_M3.npy", "points_M4.npy",
         "points_gridImage.npy", "points_gridDefocus.npy"]
RUNS = {"plain": (0, 0, 0, 0, 0, 0), "thin": (2, 2, 2, 2, 2, 2)}


def main():
    MG._stub_modules()
    sys.path.insert(0, MG.REF)
    work = tempfile.mkdtemp(prefix="akb_golden_savewave_")
    os.chdir(work)
    import AKB_raytrace_20250312 as A
    A.option_set = True
    A.wave_num_H = A.wave_num_V = 33
    out = {"defocusForWave": np.float64(A.defocusForWave)}
    for name, ds in RUNS.items():
        (A.downsample_h1, A.downsample_v1, A.downsample_h2, A.downsample_v2, A.downsample_h_f,
         A.downsample_v_f) = ds
        run_dir = os.path.join(work, name)
        os.makedirs(run_dir)
        os.chdir(run_dir)
        try:
            with contextlib.redirect_stdout(io.StringIO()):
                A.saveWaveData(MG.best_params())
        except SystemExit:
            pass
        folder = glob.glob(os.path.join(run_dir, "output_*"))
        folder = [d for d in folder if os.path.exists(os.path.join(d, "calculation_conditions.txt"))]
        assert len(folder) == 1, folder
        for fn in FILES:
            out[f"{name}_{fn[:-4]}"] = np.load(os.path.join(folder[0], fn))
        with open(os.path.join(folder[0], "calculation_conditions.txt")) as f:
            out[f"{name}_conditions"] = np.array(f.read())
        out[f"{name}_downsample"] = np.array(ds)
        print(name, out[f"{name}_points_M1"].shape, out[f"{name}_points_gridImage"].shape)
    np.savez_compressed(os.path.join(MG.OUT, "savewave_33.npz"), **out)


if __name__ == "__main__":
    main()
