import sys, os; sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from oracle.oracle import as_u8
from rust_tracer_amd import DeviceScene, SceneDesc
desc = SceneDesc.synth_config(3)
for k in range(3):
    s = DeviceScene(desc, device=0)
    img, cnt, _, img8 = s.render(320, 180, 8, want_u8=True)
    q = as_u8(img)
    bad = np.argwhere((q != img8).any(axis=2))
    print("run", k, "mismatched pixels", len(bad), bad[:10].tolist())
    for (y, x) in bad[:5]:
        print("  ", y, x, img[y, x], q[y, x], img8[y, x])
    s.close()
