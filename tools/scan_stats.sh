#!/bin/bash
# Build librt_hip_stats.so (scan hit-path and leaf-occupancy counters on, RT_DIAG=1) next
# to the product library: tools/leaf_stats.py / tools/scan_stats.py load it with RT_LIB.
set -e
exec bash "$(dirname "$0")/build_variant.sh" stats "-DRT_DIAG=1"
