"""Hierarchical (MPMD) fitting: different loss terms on disjoint sub-communicators,
combined with OnePointGroup (reference multigrad/multigrad.py:547-607).

    python -m multigrad_amd.launch -n 4 examples/hierarchical_groups.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import multigrad_amd as mg  # noqa: E402
from multigrad_amd.models.toy import SumOfSquaresModel, make_toy_data  # noqa: E402

if __name__ == "__main__":
    world = mg.init_distributed() if int(os.environ.get("WORLD_SIZE", "1")) > 1 else mg.get_world_comm()
    ngroups = min(2, world.size)
    subcomm, ngroups, group = mg.split_subcomms(num_groups=ngroups, comm=world)
    # each group fits its own data set; the group loss is the sum over groups
    data = make_toy_data(ndim=4, npoints=200, seed=100 + group, comm=subcomm)
    model = SumOfSquaresModel(aux_data=data, comm=subcomm)
    group_model = mg.OnePointGroup(model, main_comm=world)
    res = group_model.run_bfgs(torch.zeros(4))
    if world.rank == 0:
        print(f"{ngroups} groups on {world.size} ranks; optimum = {res.x}, loss = {res.fun:.6f}")
