#!/bin/bash
# Dev: timing + SQ/GRBM counter passes of the fused bins kernel (tools/probe/probe_fused) on the GPU box.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/fpmc; rm -rf $o; mkdir -p $o
timeout -k 10 60 ./tools/probe/probe_fused > $o/time.txt 2>&1
timeout -s KILL 60 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU -d $o/p1 -o p1 --output-format csv -- ./tools/probe/probe_fused > $o/p1.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_FMA_F64 SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_ADD_F64 GRBM_GUI_ACTIVE -d $o/p2 -o p2 --output-format csv -- ./tools/probe/probe_fused > $o/p2.log 2>&1
cat $o/time.txt
