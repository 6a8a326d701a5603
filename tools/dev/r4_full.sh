#!/bin/bash
# GPU box (round 4): the whole -m gpu suite (no -x), then the default bench line and the H = 32 line.
# Output: gpurun_out/r4/full/.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r4/full; rm -rf $o; mkdir -p $o
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $o/gpu_tests.txt 2>&1; rc=$?
echo "tests rc=$rc $(tail -1 $o/gpu_tests.txt)"
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 420 python3 bench.py > $o/bench.json 2> $o/bench.err || exit 1
timeout -k 10 180 python3 bench.py --hyps 32 --no-cpu --no-map --no-c5 --no-roofline --steps 400 --warmup 50 > $o/bench_h32.json 2>> $o/bench.err || exit 1
python3 - <<'PY'
import json
for f in ("bench", "bench_h32"):
    d = json.loads(open("gpurun_out/r4/full/%s.json" % f).read().strip().splitlines()[-1])
    print(f, "ms/step %.4f" % d["ms_per_step"], "value %.1f" % d["value"], "stages", {k: round(v, 4) for k, v in d.get("stages_ms", {}).items() if k.endswith("_ms")})
    for k in ("roofline", "fused_roofline", "c5", "c5_dense", "c5_map_fuse", "inscan_certs", "host"):
        if k in d: print(" ", k, json.dumps(d[k])[:300])
PY
