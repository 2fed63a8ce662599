"""The `rust_tracer` CLI (reference cli.rs / main.rs modes) on the device: normal mode
writes ./output/<t>.png equal to rt_render's Color::as_u8 frame; --method rayforest
writes render_forest's image and --stats prints RayForest::stats; bench prints the
reference's Total Time / Avg Per Op lines (basic, forest, forest filter)."""
import os
import re
import subprocess

import numpy as np
import pytest

from rust_tracer_amd import DeviceScene, SceneDesc
from .test_image_io import read_png

pytestmark = pytest.mark.gpu
CLI = os.path.join(os.path.dirname(os.path.dirname(__file__)), "rust_tracer_amd", "rust_tracer")


def run(args, cwd):
    r = subprocess.run([CLI] + args, cwd=cwd, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    return r.stdout


def test_cli_basic_png(tmp_path):
    out = run(["-w", "64", "-h", "48", "-d", "8"], tmp_path)
    files = list((tmp_path / "output").glob("*.png"))
    assert len(files) == 1, out
    _, _, _, rgb8 = DeviceScene(SceneDesc.my_scene()).render(64, 48, 8, want_u8=True)
    assert np.array_equal(read_png(files[0]), rgb8)


def test_cli_rayforest_stats(tmp_path):
    out = run(["-w", "64", "-h", "48", "--method", "rayforest", "--stats", "--out", "f.png"], tmp_path)
    f = DeviceScene(SceneDesc.my_scene()).forest(64, 48, 8)
    st = f.stats()
    assert f"Number of Trees: {st['num_trees']}" in out
    assert f"Max Tree Size: {st['largest_tree']}" in out
    assert f"p99 Size: {st['p99']}" in out
    assert f"Number of Intersections: {st['num_intersections']}" in out
    img = f.render()
    want = np.clip(np.nan_to_num(255.0 * img, nan=0.0), 0, 255).astype(np.uint8)
    assert np.array_equal(read_png(tmp_path / "f.png"), want)


@pytest.mark.parametrize("extra", [[], ["--method", "rayforest"], ["--method", "rayforest", "-f"]])
def test_cli_bench_modes(tmp_path, extra):
    args = ["-w", "64", "-h", "48"] + (["--method", "rayforest"] if "--method" in extra else []) + ["bench", "-n", "3"]
    if "-f" in extra:
        args.append("-f")
    out = run(args, tmp_path)
    assert re.search(r"Total Time: \d+ms \| \d+ns", out), out
    assert re.search(r"Avg Per Op: [\d.e+-]+ms \| [\d.e+-]+ns", out), out
    if "-f" in extra:
        assert "Trees Evaluated:" in out and "% evaluated:" in out
