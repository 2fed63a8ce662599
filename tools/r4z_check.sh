set -o pipefail
bash tools/configs_run.sh r4cfg || exit 1
bash tools/profile.sh r4zp || exit 2
