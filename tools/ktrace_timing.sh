export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt -o run -- python tools/diag_runtime.py timing > gpurun_out/kt.log 2>&1
