#!/bin/bash
# HBM traffic of the C5 PrimitiveMap kernels: the standalone 1M-slot fuse (bench.py --map-only:
# k_fuse_runs, k_fuse_apply, k_fuse_colors) and the in-scan map update (bench.py --c5-only:
# k_smap_block, k_smap_apply), one rocprofv3 --pmc pass per
# counter set; summarised by tools/pmc_fuse.py. Usage (GPU box): bash tools/pmc_fuse.sh r03
set -e
round=${1:-r03}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/pmc_fuse
rm -rf $out; mkdir -p $out
for leg in map-only c5-only; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $out/$leg/fetch -o fetch --output-format csv -- python3 bench.py --$leg > $out/$leg.fetch.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $out/$leg/write -o write --output-format csv -- python3 bench.py --$leg > $out/$leg.write.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ TCC_EA0_RDREQ_128B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_32B -d $out/$leg/rdreq -o rdreq --output-format csv -- python3 bench.py --$leg > $out/$leg.rdreq.log 2>&1
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $out/$leg/kt -o kt --output-format csv -- python3 bench.py --$leg > $out/$leg.kt.log 2>&1
done
python3 tools/pmc_fuse.py $out gpurun_out/pmc_fuse_$round.json
