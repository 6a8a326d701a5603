#!/bin/bash
# GPU box (round 5 dev): the -m gpu suite with Σ_post's first phase by 2 x 2 blocks (chol_inverse_phase1_blk) in k_evidence (in-tree), then interleaved
# A/B against build_var/subst (the substitution over all rows) at H = 32 and 256, and smoke().
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r5s39; rm -rf $o; mkdir -p $o
rc=0; timeout -k 10 500 python -u -m pytest tests -q -x -m gpu --timeout 120 --timeout-method thread > $o/gpu_tests.log 2>&1 || rc=$?
tail -2 $o/gpu_tests.log
case $rc in 0) ;; *) grep -E "Error|assert|FAIL|^E " $o/gpu_tests.log | head -30; echo "gpu tests rc=$rc"; exit $rc;; esac
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
ab() {  # tag lib args...
  local tag=$1 lib=$2; shift 2
  timeout -k 10 180 python3 tools/dev/ab_bench.py $lib --no-cpu --no-map --no-c5 --no-roofline --no-dropin --no-extras "$@" > $o/$tag.json 2>> $o/err.txt || { tail -5 $o/err.txt; exit 1; }
  echo "$tag $(tail -1 $o/$tag.json | python3 -c "import json,sys; print(round(json.loads(sys.stdin.read())['ms_per_step'],4))")"
}
for i in 1 2 3; do
  ab new_h32_$i fl-slam_amd/gcslam/libgcslam.so --hyps 32 --steps 400 --warmup 50
  ab subst_h32_$i fl-slam_amd/build_var/subst/libgcslam.so --hyps 32 --steps 400 --warmup 50
  ab new_h256_$i fl-slam_amd/gcslam/libgcslam.so --steps 100 --warmup 30
  ab subst_h256_$i fl-slam_amd/build_var/subst/libgcslam.so --steps 100 --warmup 30
done | tee $o/ab.txt
