#!/bin/bash
# GPU check of HEAD: the -m gpu suite (test failures do not stop the script; a crash, hang or
# timeout does), then one default bench line.  tools/r3_check.sh TAG [pytest selection]
set -o pipefail
TAG=${1:-r3}; shift
SEL=${@:-tests}
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest $SEL -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/$TAG.tests.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc"; exit 1; fi
timeout -k 10 400 python bench.py > gpurun_out/$TAG.bench.json 2> gpurun_out/$TAG.bench.err || exit 2
echo "done (pytest rc $rc)"
