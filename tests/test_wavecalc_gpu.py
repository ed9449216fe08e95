"""The Wavecalc chain at BASELINE configs[1]'s sizes and the driver's stage resume (MI355X).

configs[1] is KB_debug's pair traced on a 3163 x 3163 grid (1e7 rays) and the Wavecalc driver's
stages over it: source -> M1 (1e7 targets), M1 -> M2 (1e7 x 1e7 = 1e14 pairs,
~200 s on one MI355X: run here on 4096 sampled M2 targets, 4e10 pairs, with the real M1 field as
its sources), M2 -> image grid. The driver resumes a mirror stage from its complex_data_M<k>.npz
(Wavecalc_raytrace_fromData_CPU0402.py:261-269, :281-290), which is how the chain runs here at
full size: M2's field comes from a file, every other stage is propagated on the device and checked
against the oracle's C sum on sampled targets (<= 1e-9 of max |u|, the Huygens bar of
tests/test_gpu_parity.py). Reference stage: Wavecalc_raytrace_fromData_GPU0402_multi.py:471.
"""
import os

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu


@pytest.mark.slow
def test_wave_chain_3163_with_m2_resumed(gpu, tmp_path):
    from akbraytracing_amd import wavedata as W
    folder = W.saveWaveData(np.zeros(26), ray_num_H=3163, directory=str(tmp_path / "w"), option_AKB=False,
                            defocus_for_wave=1e-3, downsample=(0, 0, 0, 0, 12, 12), timestamp="test")
    m1 = np.load(os.path.join(folder, "points_M1.npy"))
    m2 = np.load(os.path.join(folder, "points_M2.npy"))
    img = np.load(os.path.join(folder, "points_gridImage.npy"))
    assert m1.shape == (4, 3163 * 3163) and m2.shape == (4, 3163 * 3163) and img.shape[1] == 50 * 50
    rng = np.random.default_rng(4)
    u2 = np.exp(2j * np.pi * rng.random(m2.shape[1])) * (1 + 0.1 * rng.random(m2.shape[1]))
    os.makedirs(tmp_path / "resume")
    np.savez(tmp_path / "resume" / "complex_data_M2.npz", data=u2)
    resumed = []
    fields = W.run_wave_chain(folder, out_dir=None, resume_dir=str(tmp_path / "resume"), resumed=resumed)
    assert resumed == ["M2"] and np.array_equal(fields["M2"], u2)
    assert sorted(fields) == ["Image", "Image2", "M1", "M2"]
    k = 2 * np.pi / 13.5e-9
    src = np.load(os.path.join(folder, "points_source.npy")).reshape(3, 1)
    pick = rng.choice(m1.shape[1], 20000, replace=False)
    want = O.huygens_c(m1[0, pick], m1[1, pick], m1[2, pick], src[0], src[1], src[2], np.ones(1, complex), k)
    assert np.max(np.abs(fields["M1"][pick] - want)) <= 1e-9 * np.max(np.abs(want))
    # M1 -> M2 (the driver's :471 stage) on 4096 sampled M2 targets: the real M1 field times its dS
    # as the 1e7 sources (4e10 pairs on the device), 24 of the targets against the oracle's C sum
    import torch
    from akbraytracing_amd.wavecalc import propagate
    dev = torch.device("cuda", 0)
    t12 = rng.choice(m2.shape[1], 4096, replace=False)
    tt = [torch.from_numpy(np.ascontiguousarray(m2[r, t12])).to(dev) for r in range(3)]
    ss = [torch.from_numpy(np.ascontiguousarray(m1[r])).to(dev) for r in range(3)]
    u1ds = fields["M1"] * m1[3]
    got = propagate(*tt, *ss, torch.from_numpy(u1ds).to(dev), k).cpu().numpy()
    chk = np.arange(0, 4096, 171)
    want = O.huygens_c(m2[0, t12[chk]], m2[1, t12[chk]], m2[2, t12[chk]], m1[0], m1[1], m1[2], u1ds, k)
    assert np.all(np.isfinite(got)) and np.max(np.abs(got[chk] - want)) <= 1e-9 * np.max(np.abs(want))
    del tt, ss
    # M2 -> image grid (x2 about its mean, as the driver scales it): 1e7 sources x 2500 targets
    g = img.copy()
    for r in range(3):
        g[r] = (g[r] - np.mean(img[r])) * 2.0 + np.mean(img[r])
    t = rng.choice(g.shape[1], 64, replace=False)
    want = O.huygens_c(g[0, t], g[1, t], g[2, t], m2[0], m2[1], m2[2], u2 * m2[3], k)
    assert np.max(np.abs(fields["Image"][t] - want)) <= 1e-9 * np.max(np.abs(want))


def test_wave_chain_resume_every_mirror_stage(gpu, tmp_path):
    """With every mirror stage's complex_data_M<k>.npz in the resume directory, the driver takes all
    four fields from the files and computes only the image stages - the same images as the
    propagated chain, and no mirror file is written again."""
    from akbraytracing_amd import wavedata as W
    from conftest import golden
    f = golden("akb_raywave_65.npz")
    hits = f["pass2_hits"].reshape(4, 3, 65, 65)[:, :, ::4, ::4].reshape(4, 3, -1)
    det = f["detcenter"].reshape(3, 65, 65)[:, ::4, ::4].reshape(3, -1)
    det2 = f["detcenter2"].reshape(3, 65, 65)[:, ::4, ::4].reshape(3, -1)
    W.save_wave_data(str(tmp_path), np.zeros((3, 1)), list(hits), 17, 17, det, det2, defocus_for_wave=1e-2)
    first = W.run_wave_chain(str(tmp_path), str(tmp_path / "run1"), resume_dir=None)
    resumed = []
    second = W.run_wave_chain(str(tmp_path), str(tmp_path / "run2"), resume_dir=str(tmp_path / "run1"),
                              resumed=resumed)
    assert resumed == ["M1", "M2", "M3", "M4"]
    for name in ("M1", "M2", "M3", "M4", "Image", "Image2"):
        assert np.array_equal(first[name], second[name]), name
    assert sorted(p.name for p in (tmp_path / "run2").iterdir()) == ["complex_data_Image.npz",
                                                                     "complex_data_Image2.npz"]
    # a file of the wrong length is refused, not broadcast
    np.savez(tmp_path / "complex_data_M1.npz", data=np.zeros(5, complex))
    with pytest.raises(ValueError):
        W.run_wave_chain(str(tmp_path), None, resume_dir=str(tmp_path))
