#!/bin/bash
# HBM traffic of the contract pair (roofline.traffic in bench.py): separate rocprofv3 --pmc passes
# over `bench.py --roofline-only`, summarised by tools/pmc_traffic.py into
# gpurun_out/pmc_traffic_<round>.json (committed as profiles/<round>/pmc_traffic.json). Usage (GPU box): bash tools/pmc_traffic.sh r01
set -e
round=${1:-r01}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/pmc_traffic
rm -rf $out; mkdir -p $out
args="bench.py --roofline-only --roofline-reps 2"
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $out/fetch -o fetch --output-format csv -- python3 $args > $out/fetch.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $out/write -o write --output-format csv -- python3 $args > $out/write.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ TCC_EA0_RDREQ_128B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_32B -d $out/rdreq -o rdreq --output-format csv -- python3 $args > $out/rdreq.log 2>&1
python3 tools/pmc_traffic.py $out gpurun_out/pmc_traffic_$round.json  # then copied into profiles/$round/
