#!/bin/bash
# the CLI's bench modes (reference main.rs:134-219) on config 3 at 1080p: basic render,
# ray-forest build + shade; the forest filter re-shade and stats on my_scene (its "blue" shape)
set -o pipefail
mkdir -p gpurun_out/r3cli
cd gpurun_out/r3cli
C=../../rust_tracer_amd/rust_tracer
timeout -k 10 200 $C -w 1920 -h 1080 -d 8 --scene synth3 bench -n 20 > basic.txt 2>&1 || exit 1
timeout -k 10 200 $C -w 1920 -h 1080 -d 8 --scene synth3 --method rayforest bench -n 20 > forest.txt 2>&1 || exit 2
timeout -k 10 200 $C -w 1920 -h 1080 -d 8 --scene my_scene --method rayforest bench -n 20 -f > filter.txt 2>&1 || exit 3
timeout -k 10 200 $C -w 1920 -h 1080 -d 8 --scene my_scene --method rayforest --stats --out f.png > stats.txt 2>&1 || exit 4
echo done
