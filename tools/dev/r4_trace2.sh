#!/bin/bash
# GPU box (round 4 dev): GPU suite, then the interleaved A/B of two build_var variants at H = 32 / 256
# and a kernel trace of each at H = 32. Usage: bash tools/dev/r4_trace2.sh <a> <b> [reps]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
a=$1; b=$2; reps=${3:-3}
XF= bash tools/dev/r4_tests.sh all || exit 1
timeout -k 10 600 bash tools/dev/r4_ab_slots.sh $reps "$a:3 $b:3" || exit 1
bash tools/dev/r4_trace_var.sh $a 32 > /dev/null && bash tools/dev/r4_trace_var.sh $b 32 > /dev/null || exit 1
for v in $a $b; do echo "## $v"; tail -7 gpurun_out/r4/trace_${v}_h32/timeline.txt; done
