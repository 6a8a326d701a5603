#!/bin/bash
# GPU box (round 5 dev): per-phase and per-wave cycles of the chain kernels at H = 32 (timing build),
# then an interleaved A/B of a library variant (tools/dev/ab_var.sh).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r5s14; rm -rf $o; mkdir -p $o
timeout -k 10 120 python3 tools/phase_timing.py 32 > $o/phases.txt 2>&1 || { tail -5 $o/phases.txt; exit 1; }
cat $o/phases.txt
[ -n "$1" ] && bash tools/dev/ab_var.sh $1 ${2:-3}
