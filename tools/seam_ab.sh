#!/bin/bash
# seam A/B: the bench's seam numbers (one frame at a time through rt_render_frame_async, rt_render
# with its pageable and page-locked host copies) per RT_TUNE setting, REPS rounds alternating.
#   tools/seam_ab.sh [SETTING ...]     SETTING: an RT_TUNE string; "default" = no RT_TUNE
#   (env REPS=2, TAG=seam)             e.g. tools/seam_ab.sh default dup=s dup=h dup=c
set -o pipefail
O=gpurun_out/${TAG:-seam}
mkdir -p "$O"
[ $# -eq 0 ] && set -- default
for rep in $(seq 1 "${REPS:-2}"); do
    for t in "$@"; do
        tt=$t
        [ "$t" = "default" ] && tt=""
        RT_TUNE="$tt" timeout -k 10 200 python bench.py --steps 5 --warmup 2 --cpu-baseline 0 --count-frame 0 \
            > "$O/b.json" 2> "$O/b.err" || { tail -20 "$O/b.err"; exit 3; }
        python -c "import json;d=json.load(open('$O/b.json'));s=d['seam'];print('$t', 'one_frame', s['one_frame_at_a_time_ms'], 'one_pass', s.get('one_pass_ms'), 'host_copy', s['rt_render_with_host_copy_ms'], 'pinned', s.get('rt_render_pinned_host_copy_ms'), 'render_call', s.get('render_call_ms'), flush=True)"
    done
done
