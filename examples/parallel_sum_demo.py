"""Sum an array over ranks to the root (reference tests/smf_example/parallel_sum_mpi4py_demo.py).

    python -m multigrad_amd.launch -n 4 examples/parallel_sum_demo.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

import multigrad_amd as mg  # noqa: E402

if __name__ == "__main__":
    comm = mg.init_distributed() if int(os.environ.get("WORLD_SIZE", "1")) > 1 else mg.get_world_comm()
    arr = np.zeros(5) + comm.rank
    arr_tot = np.zeros_like(arr)
    comm.Reduce(arr, arr_tot, op=mg.parallel.SUM, root=0)
    print(f"rank = {comm.rank}, arr_tot={arr_tot}")
