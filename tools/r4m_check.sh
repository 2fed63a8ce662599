set -o pipefail
mkdir -p gpurun_out/r4m gpurun_out/r4lv
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullframe.py tests/test_gpu_forest.py tests/test_gpu_seam.py -x -q -m gpu --timeout 200 --timeout-method thread -k "textured or material or forest or seam_split" > gpurun_out/r4m/tests.log 2>&1 || { tail -20 gpurun_out/r4m/tests.log; exit 1; }
tail -2 gpurun_out/r4m/tests.log
REPS=3 bash tools/ab_env.sh "RT_LIB=rust_tracer_amd/librt_hip_base.so" "RT_X=0" > gpurun_out/r4m/ab.txt 2>&1 || exit 2
cat gpurun_out/r4m/ab.txt
RT_LIB=rust_tracer_amd/librt_hip_stats.so timeout -k 10 200 python tools/leaf_stats.py > gpurun_out/r4lv/leaf_stats.txt 2>&1 || exit 3
timeout -k 10 200 python tools/level_ops.py > gpurun_out/r4lv/level_ops.txt 2>&1 || exit 4
timeout -k 10 300 python tools/subband_time.py 20 5 > gpurun_out/r4lv/subband.txt 2>&1 || exit 5
timeout -k 10 300 python tools/subband_time.py 64 3 >> gpurun_out/r4lv/subband.txt 2>&1 || exit 6
