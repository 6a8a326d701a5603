#!/bin/bash
# PMC passes over a short bench run (dev helper). Usage: bash tools/pmc.sh <tag> [bench args]
# Each counter group is its own rocprofv3 pass (--pmc only with --kernel-trace-free runs).
set -e
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/pmc_$tag
mkdir -p $out
timeout -k 10 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES -d $out/sq -o sq --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu "$@" > $out/sq.log 2>&1
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d $out/fetch -o fetch --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu "$@" > $out/fetch.log 2>&1
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d $out/write -o write --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu "$@" > $out/write.log 2>&1
python3 tools/pmc_summ.py $out
