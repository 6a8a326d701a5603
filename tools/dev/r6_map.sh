#!/bin/bash
# GPU box (round 6 dev): the map / scan-map / C5 tests, the C5 map PMC passes (tools/pmc_fuse.sh), the
# standalone fuse leg, the C5 legs and the C5 rank-shard leg (owner / non-owner).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=${1:-map}; o=gpurun_out/r6/$tag; rm -rf $o; mkdir -p $o
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "map or scanmap or c5 or association" > $o/tests.txt 2>&1 || { tail -30 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
bash tools/pmc_fuse.sh r06 > $o/pmc.log 2>&1 || { tail -20 $o/pmc.log; exit 1; }
cp gpurun_out/pmc_fuse_r06.json $o/ && python3 -c "
import json; d=json.load(open('$o/pmc_fuse_r06.json'))
for leg,v in d.items(): print(leg, json.dumps(v)[:1500])"
timeout -k 10 200 python3 bench.py --map-only > $o/map.json 2>&1 && cat $o/map.json
timeout -k 10 300 python3 bench.py --c5-only > $o/c5.json 2>&1 && cat $o/c5.json
timeout -k 10 300 python3 bench.py --c5-shard-only > $o/c5_shard.json 2>&1 && cat $o/c5_shard.json
