"""Host time per bench step by phase: wraps RayWave's front/back pieces with perf_counter
accumulators and runs bench.py in-process (its arguments follow):

    python scripts/host_phases.py --steps 200 --warmup 5 --no-cpu-baseline --no-extras
"""
import collections
import functools
import os
import runpy
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from akbraytracing_amd import wavefront as W  # noqa: E402

acc = collections.defaultdict(float)
cnt = collections.Counter()


def wrap(cls, name):
    f = getattr(cls, name)

    @functools.wraps(f)
    def g(*a, **k):
        t = time.perf_counter()
        try:
            return f(*a, **k)
        finally:
            acc[name] += time.perf_counter() - t
            cnt[name] += 1
    setattr(cls, name, g)


for n in ("launch_front", "_take_picks", "_queue_picks", "_pass1", "_finish_tilt", "_pass2", "launch_back",
          "pupil", "_launch_back", "_resolve"):
    wrap(W.RayWave, n)
_fo = W.RayWave._flags_of


def _flags_of_aged(self, f):
    """_flags_of, its wait time binned by the front's age in runs (0 = the newest front)"""
    t = time.perf_counter()
    if f.flags is None and not f.flag_ev.query():
        cnt["flag event pending at first read"] += 1
        if os.environ.get("AKB_SPIN"):
            while not f.flag_ev.query():
                pass
    r = _fo(self, f)
    age = (self._runs - 1 - f.slot) % self.NSLOTS
    acc[f"_flags_of age {age}"] += time.perf_counter() - t
    cnt[f"_flags_of age {age}"] += 1
    return r


W.RayWave._flags_of = _flags_of_aged
import torch  # noqa: E402
for n in ("synchronize", "query"):
    wrap(torch.cuda.Event, n)
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[1:]
t0 = time.perf_counter()
runpy.run_path(sys.argv[0], run_name="__main__")
steps = cnt["launch_front"]
print(f"# {steps} launch_front calls; host ms per call by phase (inclusive):", file=sys.stderr)
for k, v in sorted(acc.items(), key=lambda kv: -kv[1]):
    print(f"{k:16s} {1e3 * v / max(steps, 1):8.4f} ms/step  ({cnt[k]} calls)", file=sys.stderr)
