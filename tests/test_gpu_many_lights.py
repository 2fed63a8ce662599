"""GPU tests of scenes with many point lights (mod.rs:189-206 per light).  Lights 0-31 keep
their shadow results in each node's node_lit word, lights 32 and up in node_lit_hi (zeroed per
pass); the trace kernel's own-shape tests and inline scans decide lights 0-31 only, the rest
always go to the shadow queue; the shadow kernel keeps up to 64 lights' positions in LDS
(rt_wavefront.hip LDS_LIGHTS) and reads the rest from the scene's records.  Frames and
counters against the oracle at 32, 33, 64, 70 and 300 lights (above 256 lights a shadow entry
is 8 B, node and light side by side: rt_device.hpp shadow_light); RT_MAX_LIGHTS + 1 (65537) are
refused."""
import numpy as np
import pytest

from oracle.oracle import OracleScene
from rust_tracer_amd import DeviceScene, SceneDesc

from .test_gpu_parity import compare

pytestmark = pytest.mark.gpu


def _scene(n_lights, seed=5):
    """n_lights point lights in all: the synthetic scene's 3 and n_lights - 3 dim ones."""
    d = SceneDesc.synth(seed, 60, 6, 20, 0.1, 0.5).editable()
    rng = np.random.default_rng(seed)
    for k in range(n_lights - 3):
        p = rng.uniform((-5.0, 1.0, -6.0), (5.0, 8.0, 2.0))
        c = rng.uniform(0.0, 0.05, 3)
        d.point_light(tuple(float(x) for x in p), tuple(float(x) for x in c))
    return d


@pytest.mark.parametrize("n_lights,tuning", [(32, None), (33, None), (64, "lb_res=16"), (70, "lb_res=16"),
                                             (70, "lb_res=16,inline_shadow=0,self_shadow=0"),
                                             (256, "lb_res=8"), (257, "lb_res=8"), (300, "lb_res=8"),
                                             (300, "lb_res=0,sort_shadow=0")])
def test_many_lights_match_the_oracle(n_lights, tuning):
    desc = _scene(n_lights)
    w, h, depth = 96, 72, 4
    ref, rcnt = OracleScene(desc).render(w, h, depth, threads=8)
    s = DeviceScene(desc, tuning=tuning)
    try:
        img, cnt, _, _ = s.render(w, h, depth)
        img2, cnt2, _, _ = s.render(w, h, depth)  # a second pass on the same pools
    finally:
        s.close()
    compare(img, ref)
    assert cnt == rcnt
    assert np.array_equal(img.view(np.uint32), img2.view(np.uint32)) and cnt2 == cnt


def test_wide_entries_larger_frame():
    """300 lights (wide entries, every light past 32 queued) at 480x270, depth 3: every 30th
    row against the oracle, counters of a second render equal (the pools are reused)."""
    desc = _scene(300)
    s = DeviceScene(desc, tuning="lb_res=0")
    try:
        a, ca, _, _ = s.render(480, 270, 3)
        b, cb, _, _ = s.render(480, 270, 3)
    finally:
        s.close()
    assert ca == cb and np.array_equal(a.view(np.uint32), b.view(np.uint32))
    ref, _ = OracleScene(desc).render(480, 270, 3, rows=(0, 270, 30), threads=8)
    compare(a[::30], ref[::30])
