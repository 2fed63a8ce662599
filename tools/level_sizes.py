import sys, os
sys.path.insert(0, os.getcwd())
from rust_tracer_amd import DeviceScene, SceneDesc
s = DeviceScene(SceneDesc.synth_config(3))
prev = 0
for d in range(1, 9):
    _, c, ms, _ = s.render(1920, 1080, d)
    print(d, c["node_rays"] - prev, c["shadow_rays"], round(ms, 3))
    prev = c["node_rays"]
