#!/bin/bash
# Dev (GPU box): parity tests of the current build, then interleaved A/B of library variants.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest tests/test_gpu_points.py tests/test_gpu_configs.py tests/test_gpu_pipeline.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/ab/tests.log 2>&1 || { tail -30 gpurun_out/ab/tests.log; exit 1; }
tail -2 gpurun_out/ab/tests.log
V=fl-slam_amd/build_var
bash tools/ab_roof.sh 2 $V/old/libgcslam.so $V/nopair/libgcslam.so fl-slam_amd/gcslam/libgcslam.so | tee gpurun_out/ab/roof.txt
bash tools/ab_run.sh 2 256 $V/old/libgcslam.so fl-slam_amd/gcslam/libgcslam.so $V/short/libgcslam.so | tee gpurun_out/ab/h256.txt
bash tools/ab_run.sh 2 32 $V/old/libgcslam.so fl-slam_amd/gcslam/libgcslam.so $V/short/libgcslam.so | tee gpurun_out/ab/h32.txt
