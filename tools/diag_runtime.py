import sys, os, time, subprocess
sys.path.insert(0, os.getcwd())
mode = sys.argv[1]
if mode == "torch_only":
    import torch; print("torch avail", torch.cuda.is_available(), torch.version.hip)
elif mode == "lib_then_torch":
    from rust_tracer_amd import SceneDesc, DeviceScene
    s = DeviceScene(SceneDesc.my_scene()); s.render(8,8,1)
    import torch; print("torch avail", torch.cuda.is_available())
elif mode == "torch_then_lib":
    import torch; print("torch avail", torch.cuda.is_available()); x = torch.zeros(4, device="cuda")
    from rust_tracer_amd import SceneDesc, DeviceScene
    s = DeviceScene(SceneDesc.my_scene()); img,c,ms,_ = s.render(64,64,8); print("lib ok", c, ms)
    import ctypes
    print([l for l in open('/proc/self/maps').read().split('\n') if 'amdhip' in l or 'hsa-runtime' in l][:4])
elif mode == "timing":
    from rust_tracer_amd import SceneDesc, DeviceScene
    for cfg, depth in ((2,4),(3,8)):
        s = DeviceScene(SceneDesc.synth_config(cfg))
        for i in range(4):
            img, c, ms, _ = s.render(1920,1080,depth)
            util = (c["node_rays"] + c["shadow_rays"]) / (64.0 * max(1, s.last_wave_iterations))
            tf = (c["node_rays"] + c["shadow_rays"]) * s.flops_per_scan / (ms / 1e3) / 1e12
            print(cfg, depth, "kernel_ms %.3f" % ms, c, "Mpix/s %.1f" % (1920*1080/ms/1e3),
                  "lane_util %.3f" % util, "alg TFLOP/s %.2f" % tf, flush=True)
