"""Where the cone solve's value error sits: the map from CONE_SWEEPS sweeps against the converged
gradients' map, split by the targets' triangles - pocket triangles, lattice cells in the boundary
band (within K + 1 cells of the lattice edge: the band sweeps' targets) and interior cells (the
patches') - beside the kernel's interior value-error estimate. Study script (GPU):
python scripts/study_cone_error.py [n ...]"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    from akbraytracing_amd.faithful import FaithfulPupil
    from akbraytracing_amd.griddata import CONE_SWEEPS, CubicGrid
    from akbraytracing_amd.wavefront import RayWave, SystemGeometry
    with open(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "akb_geometry.json")) as f:
        geom = SystemGeometry.from_dict(json.load(f))
    K = CONE_SWEEPS
    out = []
    for n in [int(a) for a in sys.argv[1:]] or [1001, 3163]:
        rw = RayWave(geom, n).run()
        y, z, w = rw["detcenter2"][1].contiguous(), rw["detcenter2"][2].contiguous(), rw["wave2"].contiguous()
        fp = FaithfulPupil(n, n, slots=2)
        t = fp.begin(y, z, w)
        r = fp.finish(t)
        got = r["map"].cpu().numpy().copy()
        est = float(r["change"].cpu().numpy().view(np.float64)[1])
        ax = r["axes"].cpu().numpy()
        owner = t.slot["owner"].cpu().numpy().reshape(128, 128)
        cg = CubicGrid(y, z, n, n)
        ref = cg.interp(w.reshape(1, -1), ax[:128], ax[128:256], tol=1e-13).cpu().numpy()[0]
        rng = float(np.nanmax(ref) - np.nanmin(ref))
        err = np.abs(got - ref) / rng
        nc2 = 2 * (n - 1) * (n - 1)
        c = owner // 2
        iv, ih = c // (n - 1), c % (n - 1)
        depth = np.minimum(np.minimum(iv, ih), np.minimum(n - 2 - iv, n - 2 - ih))
        claimed = owner != np.iinfo(np.int32).max
        pocket = claimed & (owner >= nc2)
        band = claimed & ~pocket & (depth <= K + 1)
        inner = claimed & ~pocket & ~band
        row = dict(n=n, est=est / rng, targets=int(claimed.sum()))
        for name, m in (("pocket", pocket), ("band", band), ("interior", inner)):
            e = err[m]
            row[name] = dict(count=int(m.sum()), max=float(np.nanmax(e)) if e.size else 0.0,
                             p99=float(np.nanpercentile(e, 99)) if e.size else 0.0)
        # the worst targets: their triangle kind and, for pocket triangles, their longest edge
        worst = np.argsort(np.nan_to_num(err.ravel(), nan=-1))[::-1][:5]
        row["worst"] = [dict(err=float(err.ravel()[k]), owner=int(owner.ravel()[k]),
                             kind="pocket" if pocket.ravel()[k] else "band" if band.ravel()[k] else "interior")
                        for k in worst]
        print(json.dumps(row), flush=True)
        out.append(row)
        fp.close()
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/study_cone_error.json", "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
