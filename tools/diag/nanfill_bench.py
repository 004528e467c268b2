"""Run bench.py with every uninitialised torch allocation (torch.empty / at::empty, including our
bindings' outputs and workspaces) filled with NaN: a kernel that reads memory it never wrote then
poisons the loss deterministically instead of depending on stale pool contents.
Usage: python tools/diag/nanfill_bench.py <bench.py args...>"""
import os
import runpy
import sys

import torch

torch.use_deterministic_algorithms(True, warn_only=True)
torch.utils.deterministic.fill_uninitialized_memory = True
root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.argv = [os.path.join(root, "bench.py")] + sys.argv[1:]
sys.path.insert(0, root)
runpy.run_path(sys.argv[0], run_name="__main__")
