# light-buffer tiers: parity with 3 tiers, A/B at the driver's line, where the shadow cycles go
set -o pipefail
O=gpurun_out/r4lt3
mkdir -p $O
RT_TUNE=lb_tiers=5 timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullframe.py tests/test_gpu_direct.py tests/test_gpu_cull_stress.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
REPS=4 bash tools/ab_env.sh "RT_TUNE=lb_tiers=3" "RT_TUNE=lb_tiers=4" "RT_TUNE=lb_tiers=5" > $O/ab.txt 2>&1 || exit 2
cat $O/ab.txt
RT_TUNE=lb_tiers=5 timeout -k 10 200 python tools/kernel_ops.py > $O/kernel_ops5.txt 2>&1 || exit 3
grep -A17 "== shadow" $O/kernel_ops5.txt
RT_TUNE=lb_tiers=5 RT_LIB=rust_tracer_amd/librt_hip_stats.so timeout -k 10 200 python tools/leaf_stats.py > $O/leaf_stats5.txt 2>&1 || exit 4
grep "walk serves\|shadow:" $O/leaf_stats5.txt
