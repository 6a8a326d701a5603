#!/bin/bash
# Dev (GPU box): parity tests of the current build, then interleaved A/B of library variants.
# Usage: bash tools/dev/ab_session.sh <test files...> -- <lib variants...>
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
tests=(); while [ "$1" != "--" ]; do tests+=("$1"); shift; done; shift
timeout -k 10 300 python -u -m pytest "${tests[@]}" -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/ab/tests.log 2>&1 || { tail -30 gpurun_out/ab/tests.log; exit 1; }
tail -2 gpurun_out/ab/tests.log
bash tools/dev/ab_run.sh 2 256 "$@" | tee gpurun_out/ab/h256.txt
bash tools/dev/ab_run.sh 3 32 "$@" | tee gpurun_out/ab/h32.txt
