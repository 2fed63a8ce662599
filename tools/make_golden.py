"""Generate the golden fixtures under tests/golden/ from the CPU oracle.

The reference (Rust) cannot be built here and holds no render-output fixture, so the
golden frames are produced by the oracle -- a C++ restatement of src/render.rs and its
callees that is itself pinned by the reference's unit tests (tests/test_oracle_kat.py).
Re-running this script must reproduce the committed files bit for bit
(tests/test_golden.py checks that).

    python tools/make_golden.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle.oracle import OracleScene, as_u8  # noqa: E402
from rust_tracer_amd import SceneDesc  # noqa: E402

GOLDEN = os.path.join(ROOT, "tests", "golden")


def my_scene_64():
    o = OracleScene()  # the oracle's own restatement of my_scene.rs
    out = {}
    for depth in (1, 2, 4, 8):
        rgb, c = o.render(64, 64, depth)
        out[f"rgb_d{depth}"] = rgb
        out[f"counters_d{depth}"] = np.array([c["node_rays"], c["shadow_rays"], c["pixels"]], np.uint64)
    out["u8_d8"] = as_u8(out["rgb_d8"])
    return out


def my_scene_256():
    o = OracleScene()
    out = {}
    for depth in (1, 8):
        rgb, c = o.render(256, 256, depth)
        out[f"rgb_d{depth}"] = rgb
        out[f"counters_d{depth}"] = np.array([c["node_rays"], c["shadow_rays"], c["pixels"]], np.uint64)
    return out


def bench_128():
    d = SceneDesc.bench_128()
    rgb, c = OracleScene(d).render(128, 128, 5)
    return {"rgb_d5": rgb, "counters_d5": np.array([c["node_rays"], c["shadow_rays"], c["pixels"]], np.uint64)}


def synth_small():
    out = {}
    for cfg, (w, h, depth) in {2: (96, 54, 4), 3: (96, 54, 8)}.items():
        d = SceneDesc.synth_config(cfg)
        rgb, c = OracleScene(d).render(w, h, depth, threads=8)
        out[f"rgb_c{cfg}"] = rgb
        out[f"counters_c{cfg}"] = np.array([c["node_rays"], c["shadow_rays"], c["pixels"]], np.uint64)
    return out


def forest_64():
    o = OracleScene()
    rgb, sizes = o.render_forest(64, 64, 8)
    return {"rgb_d8": rgb, "tree_sizes_d8": sizes}


def spp_small():
    """Config 5's supersampling (rt_render_spp: counter-hash jitter, seed 3) on small frames."""
    out = {}
    rgb, c = OracleScene().render(32, 32, 4, spp=4, seed=3)
    out["rgb_my_scene"] = rgb
    out["counters_my_scene"] = np.array([c["node_rays"], c["shadow_rays"], c["pixels"]], np.uint64)
    d = SceneDesc.synth_config(5)
    rgb, c = OracleScene(d).render(48, 27, 8, threads=8, spp=4, seed=3)
    out["rgb_c5"] = rgb
    out["counters_c5"] = np.array([c["node_rays"], c["shadow_rays"], c["pixels"]], np.uint64)
    return out


FIXTURES = {
    "my_scene_64.npz": my_scene_64,
    "my_scene_256.npz": my_scene_256,
    "bench_128.npz": bench_128,
    "synth_small.npz": synth_small,
    "forest_64.npz": forest_64,
    "spp_small.npz": spp_small,
}


def main():
    os.makedirs(GOLDEN, exist_ok=True)
    for name, fn in FIXTURES.items():
        arrays = fn()
        np.savez_compressed(os.path.join(GOLDEN, name), **arrays)
        print(name, {k: v.shape for k, v in arrays.items()})


if __name__ == "__main__":
    main()
