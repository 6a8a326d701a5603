#!/bin/bash
# GPU box, round 5 final evidence: tools/round_profile.sh r05 (the -m gpu suite, the default bench line,
# rocprofv3 kernel stats of the same command, PMC traffic of the contract pair and of the C5 map kernels,
# the H = 32 / 256 timelines), then the H = 32 shard line and the C2 (H = 1) line.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/round_profile.sh r05 || exit $?
o=gpurun_out/r05
timeout -k 10 200 python3 bench.py --hyps 32 --steps 400 --warmup 50 --no-cpu --no-roofline --no-map --no-c5 --no-dropin > $o/bench_h32.json 2> $o/bench_h32.err || { tail -5 $o/bench_h32.err; exit 1; }
python3 tools/summ.py $o/bench_h32.json
timeout -k 10 200 python3 bench.py --hyps 1 --steps 400 --warmup 50 --no-cpu --no-roofline --no-map --no-c5 --no-dropin > $o/bench_h1.json 2> $o/bench_h1.err || { tail -5 $o/bench_h1.err; exit 1; }
python3 tools/summ.py $o/bench_h1.json
