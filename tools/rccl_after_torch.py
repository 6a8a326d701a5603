"""Dev check (GPU box): the RCCL exchange tests in a process that initialised torch.distributed
(gloo) first, as bench.py does at N > 1: torch bundles its own librccl.so, libgcslam links
/opt/rocm/lib/librccl.so.1; this shows the product's communicator still binds and runs."""
import os
import sys

import torch.distributed as td

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29511")
td.init_process_group("gloo", rank=0, world_size=1)
import pytest  # noqa: E402

# the two-process gloo test spawns its own process groups: only the in-process RCCL cases here
sys.exit(pytest.main(["tests/test_gpu_exchange.py", "-m", "gpu", "-v", "-x", "-k", "not two_process", "-p", "no:cacheprovider"]))
