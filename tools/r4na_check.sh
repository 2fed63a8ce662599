set -o pipefail
O=gpurun_out/r4na
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_cull_stress.py -x -q -m gpu --timeout 200 --timeout-method thread -k "light_buffer_tiers" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
REPS=3 bash tools/ab_env.sh "RT_X=0" "RT_TUNE=lb_near_all=1" "RT_TUNE=lb_near_all=1,lb_tiers=5" "RT_TUNE=lb_near_all=1,lb_tiers=6" > $O/ab.txt 2>&1 || exit 2
cat $O/ab.txt
RT_TUNE=lb_near_all=1,lb_tiers=5 RT_LIB=rust_tracer_amd/librt_hip_stats.so timeout -k 10 200 python tools/leaf_stats.py > $O/leaf_stats.txt 2>&1 || exit 3
grep "walk serves" $O/leaf_stats.txt | tail -1
