"""Wall-clock of the trace kernel's phases per wave iteration (diagnostic build):
  tools/build_variant.sh pclk "-DRT_POST_CLOCK=1"
  RT_LIB=rust_tracer_amd/librt_hip_pclk.so python tools/post_clock.py
Phases (rt_wavefront.hip RT_POST_CLOCK): load (task / pixel), scan, attributes + node record,
children (append + tasks), self (own-shape and inline shadow tests), shadow entries (append +
keys).  s_memtime ticks summed over waves: a wave's time includes the other waves' issue on its
SIMD, so the shares, not the totals, are the result.  Config 3 at 1080p, depth 8: one frame at
a time, then a 20-frame batch (one pass, like the bench's).  Round 5 (profiles/r5ab/r5d2_*,
r5l1_post_clock.log): the own-shape tests and the shadow entries took two fifths of a deep
iteration, waiting on light records read as vector loads behind the iteration's stores
(DESIGN.md round 5, item 8).  With RT_DEFER_STORES (deep levels) the columns "children" and
"self" hold the own-shape tests and the appends + stores, in that order."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rust_tracer_amd import DeviceScene, SceneDesc, abi  # noqa: E402

NAMES = ["load", "scan", "attrs+record", "children", "self", "entries"]


def read(L, reset=True):
    st = (C.c_ulonglong * 16)()
    assert L.rt_debug_post_clock(st, 1 if reset else 0) == 0
    return list(st)


def show(tag, v):
    for half, name in ((0, "level 0"), (8, "levels >= 1")):
        tot = sum(v[half:half + 6])
        its = max(1, v[half + 6])
        print(f"{tag:>10s} {name:>12s} iterations {v[half + 6]:9d}  ticks/iteration {tot / its:9.0f}  " +
              "  ".join(f"{n} {v[half + k] / max(1, tot):.3f}" for k, n in enumerate(NAMES)), flush=True)


def main():
    import torch
    L = abi.lib()
    L.rt_debug_post_clock.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    s = DeviceScene(SceneDesc.synth_config(3))
    w, h = 1920, 1080
    s.render(w, h, 8)
    read(L)
    for _ in range(5):
        s.render(w, h, 8)
    show("one frame", read(L))
    n = 20
    cams = []
    for k in range(n):
        c = abi.camera(w, h)
        c.origin[0] = c.origin[0] + 0.01 * k
        cams.append(c)
    out = torch.empty((n, h, w, 3), dtype=torch.float32, device="cuda")
    cnt = torch.zeros(3, dtype=torch.int64, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    s.render_bands_batch_async(cams, 8, 8, 0, 1, out.data_ptr(), cnt.data_ptr(), st)
    torch.cuda.synchronize()
    read(L)
    for _ in range(2):
        s.render_bands_batch_async(cams, 8, 8, 0, 1, out.data_ptr(), cnt.data_ptr(), st)
    torch.cuda.synchronize()
    s.sync_status()
    show("batch 20", read(L))
    s.close()


if __name__ == "__main__":
    main()
