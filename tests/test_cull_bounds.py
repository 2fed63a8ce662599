"""The culling hierarchy's error bounds (DESIGN.md "Exact culling") against the
reference arithmetic, replayed in numpy float32 on adversarial rays
(tools/cull_bounds_check.py).  rt_build.cpp multiplies each basis by a safety factor
(sphere 4, cube 32; triangles 4 on rho for sin(phi) < 0.1 and 4 x 10 on rho / sin(phi)
above, rt_build.cpp SAFETY_TRI / TRI_STEEP); the largest ratio measured here must stay a
factor 4 below it, or the product would cull hits the reference reports."""
import pytest

from tools.cull_bounds_check import run

SAFETY = {"sphere": 4.0, "cube": 32.0, "triangle": 4.0, "triangle_steep": 40.0}


@pytest.mark.parametrize("seed", [101, 202])
def test_bounds_hold_with_margin(seed):
    worst = run(150000, seed, chunk=150000)
    for kind, ratio in worst.items():
        assert ratio * 4.0 <= SAFETY[kind], (kind, ratio)
