#!/bin/bash
# GPU box (round 4 dev): pipeline tests on the in-tree library, then the interleaved A/B of the
# period of the combine_final completion events the slot staging orders on (build_var/bind<k>).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r4/bound; rm -rf $o; mkdir -p $o
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "pipeline or ingest or slot or stage" > $o/tests.txt 2>&1; rc=$?
echo "tests rc=$rc $(tail -1 $o/tests.txt)"
[ $rc -eq 0 ] || exit $rc
bash tools/dev/r4_ab_slots.sh 3 "bind0:3 bind1:3 bind2:3 bind3:3 bind2:4" || exit 1
cp gpurun_out/r4/ab_slots/ab.txt $o/ab.txt
