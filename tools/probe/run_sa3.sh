#!/bin/bash
# Dev: timing + FETCH_SIZE / WRITE_SIZE passes of tools/probe/probe_sa3 (GPU box).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/sa3; mkdir -p $o
timeout -k 10 60 ./tools/probe/probe_sa3 > $o/time.txt 2>&1
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d $o/f -o f --output-format csv -- ./tools/probe/probe_sa3 > $o/f.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d $o/w -o w --output-format csv -- ./tools/probe/probe_sa3 > $o/w.log 2>&1
cat $o/time.txt
