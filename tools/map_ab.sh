set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/map
timeout -k 10 300 python -u -m pytest tests/test_gpu_map.py tests/test_map_ops.py tests/test_association.py tests/test_gpu_scanmap.py -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/map/tests.log 2>&1 || { tail -30 gpurun_out/map/tests.log; exit 1; }
tail -2 gpurun_out/map/tests.log
for l in packed fields packed fields; do timeout -k 10 120 python3 bench.py --map-only --map-layout $l >> gpurun_out/map/ab.txt 2>>gpurun_out/map/ab.err; done
cat gpurun_out/map/ab.txt
bash tools/pmc_fuse.sh r03 > /dev/null 2>&1 && python3 -c "
import json; d=json.load(open('gpurun_out/pmc_fuse_r03.json'))
for leg in d: 
  for k,v in d[leg]['kernels'].items(): print(leg,k,v)"
