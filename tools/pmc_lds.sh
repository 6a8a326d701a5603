#!/bin/bash
# Dev (GPU box): SQ issue / wait / LDS counters of the roofline kernels (bench.py --roofline-only:
# k_soft_assign, k_moment_partials, k_bins_fused), one rocprofv3 --pmc pass per counter set.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/pmc_lds; rm -rf $out; mkdir -p $out
args="bench.py ${PMC_ARGS:---roofline-only --roofline-reps 2}"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES -d $out/a -o a --output-format csv -- python3 $args > $out/a.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_MISC SQ_INSTS_SALU -d $out/b -o b --output-format csv -- python3 $args > $out/b.log 2>&1
python3 - <<'PY'
import csv, glob, collections, re
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/pmc_lds/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(k_\w+)", r["Kernel_Name"]); k = m.group(1) if m else r["Kernel_Name"][:40]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    if not k.startswith("k_"): continue
    print(k, {c: "%.4g" % (sum(v) / len(v)) for c, v in sorted(cs.items())})
PY
