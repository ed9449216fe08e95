"""The boundary band's pocket chords: per ring vertex the number of chords (pocket edges to other
ring vertices) on the C3 trace's lattice, whose largest fans set the band sweep's longest wave.
Study script (GPU): python scripts/study_band.py [n ...]"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    from akbraytracing_amd.griddata import CubicGrid
    from akbraytracing_amd.wavefront import RayWave, SystemGeometry
    with open(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "akb_geometry.json")) as f:
        geom = SystemGeometry.from_dict(json.load(f))
    for n in [int(a) for a in sys.argv[1:]] or [1001, 3163]:
        rw = RayWave(geom, n).run()
        y, z = rw["detcenter2"][1].contiguous(), rw["detcenter2"][2].contiguous()
        cg = CubicGrid(y, z, n, n)
        xptr = cg.xptr.cpu().numpy()
        cnt = np.diff(xptr)
        order = np.argsort(cnt)[::-1][:8]
        print(json.dumps(dict(n=n, ring=int(cnt.size), npock=int(cg.npock), chords=int(cnt.sum()),
                              max=int(cnt.max()), over8=int((cnt > 8).sum()), over64=int((cnt > 64).sum()),
                              over512=int((cnt > 512).sum()), top=[(int(r), int(cnt[r])) for r in order])),
              flush=True)


if __name__ == "__main__":
    main()
