set -o pipefail
bash tools/gpu_check.sh r4fin || exit 1
bash tools/profile.sh r4finp || exit 2
