"""A/B timing of the chain kernel variants (AKB_CHAIN_WAVES occupancy, AKB_CHAIN_GRID workgroups)
on the bench geometry: pass-1 and pass-2 launches timed with HIP events, median of N launches. One
variant per process (variants are read once per process), all on the same GPU.
Usage: python scripts/ab_chain.py [n] [reps] [waves|grid]"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(n, reps):
    sys.path.insert(0, ROOT)
    import numpy as np
    import torch
    from akbraytracing_amd.wavefront import RayWave, SystemGeometry
    g = SystemGeometry.load(os.path.join(ROOT, "tests", "golden", "akb_geometry.json"))
    rw = RayWave(g, n)
    rw.run()
    p1, p2 = rw._p1, rw._pass2_launch(False)
    t1, t2 = [], []
    for _ in range(reps):
        for launch, acc in ((p1, t1), (p2, t2)):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            launch.launch(reset_flags=False)
            b.record()
            b.synchronize()
            acc.append(a.elapsed_time(b))
    print(json.dumps({"w": os.environ.get("AKB_CHAIN_WAVES", "4"), "grid": os.environ.get("AKB_CHAIN_GRID", "8192"),
                      "pass1_ms": float(np.median(t1)),
                      "pass2_ms": float(np.median(t2)), "pass1_min": min(t1), "pass2_min": min(t2)}))


if __name__ == "__main__":
    if len(sys.argv) > 3 and sys.argv[3] == "child":
        child(int(sys.argv[1]), int(sys.argv[2]))
        sys.exit(0)
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 3163
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    what = sys.argv[3] if len(sys.argv) > 3 else "waves"
    variants = ([{"AKB_CHAIN_WAVES": str(w)} for w in (4, 2, 8)] if what == "waves" else
                [{"AKB_CHAIN_GRID": str(g)} for g in (2048, 1024, 4096, 8192, 16384, 40000)])
    for rnd in range(2):
        for v in variants:
            env = dict(os.environ, **v)
            r = subprocess.run([sys.executable, __file__, str(n), str(reps), "child"], env=env, capture_output=True,
                               text=True, timeout=300)
            print(r.stdout.strip() or r.stderr[-500:], flush=True)
