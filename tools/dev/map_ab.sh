#!/bin/bash
# Dev (GPU box): the map / ingest GPU tests, the C5 fuse leg in both device layouts (interleaved),
# the C5 map kernels' PMC traffic and the H = 32 shard timeline.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/map; rm -f gpurun_out/map/ab.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_map.py tests/test_map_ops.py tests/test_association.py tests/test_gpu_scanmap.py tests/test_gpu_ingest.py -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/map/tests.log 2>&1 || { tail -30 gpurun_out/map/tests.log; exit 1; }
tail -2 gpurun_out/map/tests.log
for l in packed fields packed fields; do timeout -k 10 120 python3 bench.py --map-only --map-layout $l >> gpurun_out/map/ab.txt 2>>gpurun_out/map/ab.err; done
cat gpurun_out/map/ab.txt
bash tools/pmc_fuse.sh r03 > /dev/null 2>&1 && python3 -c "
import json; d=json.load(open('gpurun_out/pmc_fuse_r03.json'))
for leg in d:
  for k,v in d[leg]['kernels'].items(): print(leg,k,v)"
bash tools/trace_scan.sh 32 h32 > /dev/null && cat gpurun_out/trace_h32/timeline.txt
