# shadow walk: how many shadow rays walk the hierarchy (no light buffer), and the scene's bound
set -o pipefail
O=gpurun_out/r4sh
mkdir -p $O
RT_LIB=rust_tracer_amd/librt_hip_stats.so timeout -k 10 200 python tools/leaf_stats.py > $O/leaf_stats.txt 2>&1 || exit 1
cat $O/leaf_stats.txt
RT_BVH_DEBUG=1 RT_LIB=rust_tracer_amd/librt_hip_diag.so timeout -k 10 100 python -c "
from rust_tracer_amd import DeviceScene, SceneDesc
s = DeviceScene(SceneDesc.synth_config(3)); print('ok')" > $O/bvh_debug.txt 2>&1 || exit 2
cat $O/bvh_debug.txt
