#!/bin/bash
# One GPU call's steps, each under its own time limit, stopping at the first failure:
#   tools/gpu_steps.sh TAG STEP [STEP ...]
# A STEP is one quoted string, its first word the kind:
#   "tests [pytest args]"        python -m pytest -m gpu (-x, thread timeouts) + args (test files;
#                                none: pytest.ini's testpaths = tests)
#   "smoke"                      __graft_entry__.smoke()
#   "bench [bench.py args]"      python bench.py ... > TAG/NN_bench.json
#   "torchrun N [bench.py args]" bench.py under torch.distributed.run with N ranks (127.0.0.1)
#   "ab [VAR=v ...] -- SPEC ..." tools/ab_env.sh with the given environment (e.g. REPS=4 K=64)
#   "profile PTAG"               tools/profile.sh PTAG (rocprofv3 kernel trace + PMC passes)
#   "py SCRIPT [args]"           python SCRIPT args (the tools/*.py timers and statistics)
#   "sh SCRIPT [args]"           bash SCRIPT args (e.g. tools/seam_ab.sh default walk_first=0)
#   "env VAR=v ... -- STEP"      the same STEP with extra environment (e.g. RT_TUNE=..., RT_LIB=...)
# Logs: gpurun_out/TAG/NN_<kind>.log (bench: .json + .err).  Replaces round 4's one-off
# tools/r4*_check.sh launchers.
set -o pipefail
TAG=${1:?tag}
shift
O=gpurun_out/$TAG
mkdir -p "$O"
n=0
run_step() {
    local kind=$1
    shift
    local id
    id=$(printf "%02d" "$n")
    case "$kind" in
        tests)
            timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 200 --timeout-method thread "$@" \
                > "$O/${id}_tests.log" 2>&1 || { tail -30 "$O/${id}_tests.log"; return 1; }
            tail -2 "$O/${id}_tests.log" ;;
        smoke)
            timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$O/${id}_smoke.log" 2>&1 \
                || { tail -20 "$O/${id}_smoke.log"; return 1; }
            cat "$O/${id}_smoke.log" ;;
        bench)
            timeout -k 10 400 python bench.py "$@" > "$O/${id}_bench.json" 2> "$O/${id}_bench.err" \
                || { tail -20 "$O/${id}_bench.err"; return 1; }
            python -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['config'];print('bench', sys.argv[2:], d['value'], d['ms_per_step'], 'check', d.get('frame_check'), 'B', c.get('frames_per_pass'), 'S', c.get('sub_bands'))" "$O/${id}_bench.json" "$@" ;;
        torchrun)
            local np=$1
            shift
            timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$np" --master-addr 127.0.0.1 \
                --master-port $((29600 + n)) bench.py --gpus "$np" "$@" > "$O/${id}_torchrun.json" 2> "$O/${id}_torchrun.err" \
                || { tail -20 "$O/${id}_torchrun.err"; return 1; }
            python -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['config'];print('torchrun', sys.argv[2:], d['value'], d['ms_per_step'], 'check', d.get('frame_check'), c.get('parallelism'))" "$O/${id}_torchrun.json" "$np" "$@" ;;
        ab)
            local envs=()
            while [ $# -gt 0 ] && [ "$1" != "--" ]; do envs+=("$1"); shift; done
            [ "$1" = "--" ] && shift
            env "${envs[@]}" bash tools/ab_env.sh "$@" > "$O/${id}_ab.log" 2>&1 || { tail -20 "$O/${id}_ab.log"; return 1; }
            cat "$O/${id}_ab.log" ;;
        profile)
            bash tools/profile.sh "$1" > "$O/${id}_profile.log" 2>&1 || { tail -20 "$O/${id}_profile.log"; return 1; }
            tail -5 "$O/${id}_profile.log" ;;
        py)
            timeout -k 10 400 python "$@" > "$O/${id}_py.log" 2>&1 || { tail -20 "$O/${id}_py.log"; return 1; }
            tail -15 "$O/${id}_py.log" ;;
        sh)
            timeout -k 10 900 bash "$@" > "$O/${id}_sh.log" 2>&1 || { tail -20 "$O/${id}_sh.log"; return 1; }
            tail -15 "$O/${id}_sh.log" ;;
        env)
            local envs=()
            while [ $# -gt 0 ] && [ "$1" != "--" ]; do envs+=("$1"); shift; done
            shift
            (export "${envs[@]}"; run_step "$@") ;;
        *)
            echo "unknown step kind: $kind" >&2
            return 2 ;;
    esac
}
for step in "$@"; do
    # shellcheck disable=SC2086
    run_step $step || { echo "step $n failed: $step"; exit 1; }
    n=$((n + 1))
done
