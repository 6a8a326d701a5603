#!/bin/bash
# GPU box (round 6): the round evidence (tools/round_profile.sh <tag>: -m gpu suite, default bench line,
# kernel stats of the same command, PMC traffic of the contract pair and the C5 map kernels, H = 32 / 256
# timelines), then the H = 32 shard line, the C2 (H = 1) line and the C5 rank-shard leg.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=${1:-r06}
bash tools/round_profile.sh $tag || exit $?
o=gpurun_out/$tag
timeout -k 10 200 python3 bench.py --hyps 32 --steps 400 --warmup 50 --no-cpu --no-roofline --no-map --no-c5 --no-dropin > $o/bench_h32.json 2> $o/bench_h32.err || { tail -5 $o/bench_h32.err; exit 1; }
python3 tools/summ.py $o/bench_h32.json
timeout -k 10 300 python3 bench.py --hyps 1 --steps 400 --warmup 50 --no-roofline --no-map --no-c5 --no-dropin > $o/bench_h1.json 2> $o/bench_h1.err || { tail -5 $o/bench_h1.err; exit 1; }
python3 tools/summ.py $o/bench_h1.json
