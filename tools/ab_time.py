"""A/B timing of render-pipeline switches (environment variables read by librt_hip).

usage: python tools/ab_time.py [config=3] [reps=5] VAR=VAL[,VAR=VAL...] ...
Each argument after the first two is one variant ("-" = defaults).  Prints the median
kernel time (HIP events inside rt_render) of `reps` 1920x1080 frames per variant, and
checks every variant's frame is bit-identical to the first variant's.
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rust_tracer_amd import DeviceScene, SceneDesc  # noqa: E402


def main():
    config = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    variants = sys.argv[3:] or ["-"]
    depth = 4 if config == 2 else 8
    ref = None
    for v in variants:
        env = {} if v == "-" else dict(kv.split("=", 1) for kv in v.split(","))
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            s = DeviceScene(SceneDesc.synth_config(config))
            times = []
            for _ in range(reps + 1):
                img, cnt, ms, _ = s.render(1920, 1080, depth)
                times.append(ms)
            s.close()
        finally:
            for k, val in old.items():
                if val is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = val
        same = None
        if ref is None:
            ref = img
        else:
            same = bool(np.array_equal(ref.view(np.uint32), img.view(np.uint32)))
        print(f"{v:40s} median {np.median(times[1:]):8.3f} ms  min {min(times[1:]):8.3f}  identical={same}",
              flush=True)


if __name__ == "__main__":
    main()
