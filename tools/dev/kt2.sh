mkdir -p gpurun_out && timeout -k 10 400 python -m pytest tests/ -x -q -m gpu > gpurun_out/t.log 2>&1; tail -3 gpurun_out/t.log; bash tools/ktrace.sh "$@"
