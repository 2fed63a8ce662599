set -o pipefail
bash tools/gpu_check.sh r4fin2 || exit 1
bash tools/profile.sh r4finp2 || exit 2
