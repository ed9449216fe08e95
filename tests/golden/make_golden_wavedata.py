"""Record the reference's calc_dS (AKB_raytrace_20250312.py:13418-13473) on the four mirrors'
hit grids of the 65x65 'ray_wave' pass 2 (akb_raywave_65.npz), build container only:

    python tests/golden/make_golden_wavedata.py

Writes wavedata_65.npz: ds (4, 65, 65), one area-element map per mirror in trace order.
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import make_golden as MG  # noqa: E402


def main():
    MG._stub_modules()
    sys.path.insert(0, MG.REF)
    import tempfile
    os.chdir(tempfile.mkdtemp(prefix="akb_golden_wavedata_"))
    import AKB_raytrace_20250312 as A
    f = np.load(os.path.join(MG.OUT, "akb_raywave_65.npz"))
    hits = f["pass2_hits"]
    ds = np.stack([A.calc_dS(hits[k], 65, 65) for k in range(hits.shape[0])])
    np.savez_compressed(os.path.join(MG.OUT, "wavedata_65.npz"), ds=ds)
    print(ds.shape, ds[0, 1, 1])


if __name__ == "__main__":
    main()
