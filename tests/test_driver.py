"""plot_result_debug(params, 'ray_wave', option_legendre=True) end to end on the device
(akbraytracing_amd/driver.py), at the reference's 65 x 65 run of the best-alignment params:

* up to the corrected pupil map (psf_calc's input) against what the reference itself computed
  (tests/golden/akb_psfcalc_65.npz: plane_out, recorded by make_golden_psfcalc.py), to the
  griddata tolerance the stage tests use (1e-6 of the map's range, same NaN mask);
* past it - extract_affine_square_region (cv2 in the reference: parity unpinned here) and the
  Legendre fit - against the oracle's composition of the same steps applied to the reference's own
  plane_out (oracle/affine.py, oracle/legendre.py), to the same relative tolerance;
* the files the mode writes."""
import os

import numpy as np
import pytest

from conftest import golden


def _best_params():
    p = np.zeros(26)  # AKB_raytrace_20250312.py:14586-14592, the fixtures' params
    p[0], p[1], p[8], p[9], p[13] = -5.73452570e-03, -2.87624337e-03, 1.05000000e-02, -3.59399021e-05, 2.39536993e-06
    p[20], p[21], p[25] = 1.05000000e-02, -3.59399021e-05, 2.39536993e-06
    return p


def test_ray_wave_conditions():
    from akbraytracing_amd.driver import ray_wave_conditions
    assert ray_wave_conditions(True) == (1e-2, 13.5) and ray_wave_conditions(False) == (1e-3, 1.35)


@pytest.mark.gpu
def test_ray_wave_mode_end_to_end(gpu, tmp_path):
    import oracle.affine as OA
    import oracle.legendre as OLg
    from akbraytracing_amd.driver import plot_result_ray_wave
    g = golden("akb_psfcalc_65.npz")
    out_dir = tmp_path / "out"
    r = plot_result_ray_wave(_best_params(), 65, directory=str(out_dir), workdir=str(tmp_path), verbose=False,
                             as_dict=True)
    # the map psf_calc receives: the reference's plane_out
    c = r["maps"]["matrixWave2_Corrected"].cpu().numpy()
    ref = g["plane_out"]
    rng_ = np.nanmax(ref) - np.nanmin(ref)
    assert np.array_equal(np.isnan(c), np.isnan(ref))
    assert np.nanmax(np.abs(c - ref)) <= 1e-6 * rng_
    # the grid spans this run's detector-2 hits, within ulps of the reference's (the tilt's arctan)
    for k in ("grid_H", "grid_V"):
        assert np.max(np.abs(r[k] - g[k])) <= 1e-9 * np.ptp(g[k]), k
    # rectification + Legendre fit of the reference's plane_out by the oracle
    rect = OA.extract_affine_square_region(ref / 13.5, target_size=ref.shape[0])
    assert np.array_equal(np.isnan(r["rectified_img"]), np.isnan(rect))
    scale = np.nanmax(np.abs(rect))
    assert np.nanmax(np.abs(r["rectified_img"] - rect)) <= 1e-6 * scale
    fits, ip = OLg.fit_multi(rect[1:-2, 1:-2], 5)
    assert [tuple(o) for o in r["orders"]] == OLg.orders(5)
    assert np.max(np.abs(r["inner_products"] - ip)) <= 1e-6 * np.max(np.abs(ip))
    pv = np.array([(np.nanmax(f) - np.nanmin(f)) * np.sign(v) for f, v in zip(fits, ip)])
    assert np.max(np.abs(r["pvs"][:-1] - pv)) <= 1e-6 * np.max(np.abs(pv))
    last = np.nanstd(ref / 13.5) * 6 * np.sign(np.sum(ip))
    assert abs(r["pvs"][-1] - last) <= 1e-6 * abs(last)
    # the files
    for name in ("psf.npy", "psf_x.npy", "psf_y.npy", "matrixWave2_Corrected(lambda).txt", "rectified_img.txt",
                 "inner_products.csv", "orders.csv"):
        assert (out_dir / name).exists(), name
    assert (tmp_path / "matrixWave2(nm).txt").exists()
    assert np.allclose(np.loadtxt(out_dir / "inner_products.csv", delimiter=","), r["inner_products"], rtol=1e-15)


@pytest.mark.gpu
def test_ray_wave_plotting_run(gpu, tmp_path):
    """The live __main__ call without option_legendre (:14603-14611): the same chain, the
    conditions file, and the reference's return value np.nanstd(map / lambda) * 6 (:3913)."""
    from akbraytracing_amd.driver import plot_result_ray_wave
    g = golden("akb_psfcalc_65.npz")
    out_dir = tmp_path / "out"
    pv = plot_result_ray_wave(_best_params(), 65, directory=str(out_dir), workdir=str(tmp_path), verbose=False,
                              option_legendre=False)
    ref = np.nanstd(g["plane_out"] / 13.5) * 6
    assert abs(pv - ref) <= 1e-6 * ref
    lines = (out_dir / "optical_params.txt").read_text().splitlines()
    assert lines[:2] == ["input", "===================="] and len(lines) == 28
    assert lines[2] == f"params[0]: {np.float64(_best_params()[0])}"
    for name in ("matrixWave2_Corrected(lambda).txt", "rectified_img.txt", "inner_products.csv", "orders.csv"):
        assert (out_dir / name).exists(), name


@pytest.mark.gpu
def test_install_routes_ray_wave_legendre(gpu, tmp_path, monkeypatch):
    """install(): plot_result_debug(params, 'ray_wave', option_legendre=True) runs the device chain
    with the module's live flags, and so does the plotting run without option_legendre (its figures
    not drawn); option_save=False (no files) stays the reference's own."""
    import types
    import akbraytracing_amd
    monkeypatch.chdir(tmp_path)
    mod = types.ModuleType("fake_driver")
    mod.option_AKB, mod.option_wolter_3_1, mod.option_mpmath = True, True, False
    mod.option_set, mod.option_HighNA, mod.option_energy = True, True, "EUV"
    mod.wave_num_H = mod.wave_num_V = 65
    mod.directory_name = str(tmp_path / "d")
    seen = []
    mod.plot_result_debug = lambda params, option, **kw: seen.append((option, kw.get("option_legendre"))) or "orig"
    akbraytracing_amd.install(mod)
    try:
        ip, orders, pvs = mod.plot_result_debug(_best_params(), "ray_wave", option_legendre=True)
        assert not seen and len(ip) == 15 and len(pvs) == 16
        assert os.path.exists(os.path.join(mod.directory_name, "inner_products.csv"))
        pv = mod.plot_result_debug(_best_params(), "ray_wave")
        assert not seen and np.isfinite(pv) and pv > 0
        assert os.path.exists(os.path.join(mod.directory_name, "optical_params.txt"))
        assert mod.plot_result_debug(_best_params(), "ray_wave", option_save=False) == "orig"
        assert seen == [("ray_wave", False)]
    finally:
        akbraytracing_amd.uninstall(mod)
