#!/bin/bash
# PMC passes over a probe binary (dev helper). Usage: bash tools/pmc_probe.sh <tag> <binary> [args]
set -e
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/pmcp_$tag
mkdir -p $out
timeout -s KILL 60 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES -d $out/p1 -o p1 --output-format csv -- "$@" > $out/p1.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_THREAD_CYCLES_VALU -d $out/p2 -o p2 --output-format csv -- "$@" > $out/p2.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d $out/p3 -o p3 --output-format csv -- "$@" > $out/p3.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d $out/p4 -o p4 --output-format csv -- "$@" > $out/p4.log 2>&1
python3 tools/pmc_summ.py $out
