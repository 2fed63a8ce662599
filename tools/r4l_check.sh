# leaf descriptors in LDS (tuning lds_leaves=1): parity subset, then A/B at the driver's K = 20
set -o pipefail
O=gpurun_out/r4l
mkdir -p $O
RT_TUNE=lds_leaves=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullframe.py tests/test_gpu_direct.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
REPS=4 bash tools/ab_env.sh "RT_TUNE=lds_leaves=1" "RT_X=0" "RT_LIB=rust_tracer_amd/librt_hip_head.so" > $O/ab.txt 2>&1 || exit 2
cat $O/ab.txt
