#!/bin/bash
# GPU box (round 5 final evidence): SQ issue / wait / LDS counters of the pipeline kernels at C3 (bench.py --steps 10, no
# extra legs) with the round's final code (tools/pmc_lds.sh with PMC_ARGS), plus GRBM_GUI_ACTIVE and the f64 MFMA
# counters of the same command.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PMC_ARGS="--steps 10 --warmup 5 --no-cpu --no-roofline --no-map --no-c5 --no-dropin --no-extras"
timeout -k 10 300 bash tools/pmc_lds.sh > gpurun_out/pmc_sq_pipeline_r05.txt 2>&1 || { tail -5 gpurun_out/pmc_sq_pipeline_r05.txt; exit 1; }
out=gpurun_out/pmc_mfma; rm -rf $out; mkdir -p $out
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA -d $out/m -o m --output-format csv -- python3 bench.py $PMC_ARGS > $out/m.log 2>&1 || { tail -5 $out/m.log; exit 1; }
python3 - <<'PY' >> gpurun_out/pmc_sq_pipeline_r05.txt
import csv, glob, collections, re
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/pmc_mfma/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(k_\w+)", r["Kernel_Name"]); k = m.group(1) if m else r["Kernel_Name"][:40]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    if not k.startswith("k_"): continue
    print(k, {c: "%.4g" % (sum(v) / len(v)) for c, v in sorted(cs.items())})
PY
cat gpurun_out/pmc_sq_pipeline_r05.txt
