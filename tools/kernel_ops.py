"""Per-kernel test counts: tuning count=trace / shadow instruments one kernel family at a time.

usage: python tools/kernel_ops.py [config=3]
Prints, per kernel family, the lane-weighted test counts per ray of that family and the
instrumented cycle shares."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rust_tracer_amd import DeviceScene, SceneDesc  # noqa: E402


def main():
    config = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    depth = 4 if config == 2 else 8
    for which in ("trace", "shadow"):
        s = DeviceScene(SceneDesc.synth_config(config), tuning=f"count={which}")
        _, cnt, ms0, _ = s.render(1920, 1080, depth)
        s.set_scan_counting(True)
        s.scan_ops(reset=True)
        _, cnt, ms, _ = s.render(1920, 1080, depth)
        ops = s.scan_ops()
        s.close()
        rays = cnt["node_rays"] if which == "trace" else cnt["shadow_rays"]
        print(f"== {which}: rays {rays}  frame {ms0:.3f} ms (instrumented {ms:.3f})")
        for k, v in ops.items():
            if k.startswith("cycles"):
                print(f"  {k:16s} {v:.4g}  per ray {v / rays:.1f}  share {v / max(1, ops['cycles_scans']):.3f}")
            else:
                print(f"  {k:16s} {v:.4g}  per ray {v / rays:.2f}")


if __name__ == "__main__":
    main()
