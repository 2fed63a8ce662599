set -o pipefail
bash tools/gpu_check.sh r4fin3 || exit 1
bash tools/profile.sh r4finp3 || exit 2
