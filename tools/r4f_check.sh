set -o pipefail
bash tools/gpu_check.sh r4f || exit 1
bash tools/profile.sh r4fp || exit 2
