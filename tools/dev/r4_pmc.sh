#!/bin/bash
# GPU box, round 4 PMC evidence: contract-pair HBM traffic and the C5 map kernels' traffic, each pass
# its own rocprofv3 run under its own time limit. Output: gpurun_out/pmc_traffic_r04.json, pmc_fuse_r04.json.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/pmc_traffic.sh r04 && bash tools/pmc_fuse.sh r04
