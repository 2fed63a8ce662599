"""GPU tests of scenes with many point lights (mod.rs:189-206 per light).  A node's shadow
results are one 32-bit mask, so a scene holds at most 32 lights (rt_api.h rt_scene_desc; more:
RT_ERR_UNSUPPORTED at creation, nothing rendered).  At that maximum -- every light in the shadow
kernel's LDS copy, the trace kernel's own-shape tests and shadow-entry keys looping over all 32,
6-bit light fields in the shadow queue -- the frame and counters meet the oracle's."""
import numpy as np
import pytest

from oracle.oracle import OracleScene
from rust_tracer_amd import DeviceScene, RtError, SceneDesc, abi

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


@pytest.mark.parametrize("tuning", [None, "lb_res=16"])
def test_thirty_two_lights_match_the_oracle(tuning):
    desc = _scene(32)
    w, h, depth = 96, 72, 4
    ref, rcnt = OracleScene(desc).render(w, h, depth, threads=8)
    s = DeviceScene(desc, tuning=tuning)
    try:
        img, cnt, _, _ = s.render(w, h, depth)
    finally:
        s.close()
    compare(img, ref)
    assert cnt == rcnt


def test_thirty_three_lights_are_refused():
    with pytest.raises(RtError) as e:
        DeviceScene(_scene(33))
    assert e.value.status == abi.RT_ERR_UNSUPPORTED
