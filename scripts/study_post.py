"""The pupil post's phases on the device: akb_pupil_post_f64 on the reference's 1001^2 gridded map
(128^2), the post kernel's wall clock (100 MHz) at its start, after the map's load, after the
nanmean, after the plane fits, at its end, after wave 0's pairwise trees, after the count's sum and after the first plane fit, and the prefilter's after its load and each axis (the
work buffer's clock words), medians over repeated launches, beside the three launches' wall time. Study script (GPU):
python scripts/study_post.py"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    from akbraytracing_amd import pupilmap as PM
    m = np.load(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "akb_raywave_full.npz"))["n1001_map_wave"]
    md = torch.from_numpy(m + 7.0).cuda()
    o = {}
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    rows, wall = [], []
    for it in range(30):
        ev[0].record()
        o = PM.pupil_post(md, out=o)
        ev[1].record()
        torch.cuda.synchronize()
        wall.append(ev[0].elapsed_time(ev[1]) * 1e3)
        clk = o["work"][0:8].cpu().numpy().view(np.uint64).astype(np.int64)
        sp = o["work"][8:16].cpu().numpy().view(np.uint64).astype(np.int64)
        rows.append(np.concatenate([(clk - clk[0]) * 0.01, (sp - sp[0]) * 0.01]))  # us
    r = np.median(np.array(rows[5:]), axis=0)
    print(json.dumps(dict(wall_us=float(np.median(wall[5:])), phases_us=[round(float(x), 2) for x in r])))


if __name__ == "__main__":
    main()
