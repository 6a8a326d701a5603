#!/bin/bash
# Dev (GPU box): H = 32 step time with per-step ingest (default copy path, and with the SDMA engine
# requested), and without ingest; interleaved. Prints the copy-related environment.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/ingest_ab; rm -rf $o; mkdir -p $o
env | grep -E "^(HSA|GPU|ROC|HIP|AMD)_" | sort > $o/env.txt
stop() { case $1 in 124|134|137|139) echo "stopped rc=$1" >> $o/ab.txt; exit $1;; esac; }
run() {  # tag env... -- args
  tag=$1; shift
  extra=""; if [ "$2" = "--no-ingest" ]; then extra="--no-ingest"; set -- "$1"; fi
  timeout -k 10 120 env "$@" python3 bench.py --hyps 32 --no-cpu --no-roofline --no-map --no-c5 --steps 400 --warmup 50 $extra > $o/$tag.json 2>>$o/err.txt; stop $?
  echo "$tag $(tail -1 $o/$tag.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],4), d.get('ingest_host_ms_per_scan'), d.get('run_scan_host_ms'))")" >> $o/ab.txt
}
for r in 1 2; do
  run ingest X=1
  run ingest_wg1 DEBUG_CLR_LIMIT_BLIT_WG=1
  run ingest_wg4 DEBUG_CLR_LIMIT_BLIT_WG=4
  run noingest X=1 --no-ingest
done
cat $o/ab.txt
