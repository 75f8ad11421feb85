"""Quick-start (reference docs/source/notebooks/smf_gradient_descent.py + intro.ipynb):
build the SMF target at the true parameters with reduce_sum, then fit it with L-BFGS-B.

    python examples/quickstart_bfgs.py
    python -m multigrad_amd.launch -n 3 examples/quickstart_bfgs.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import multigrad_amd as mg  # noqa: E402
from multigrad_amd.models.smf import DocsSMFModel, make_docs_data  # noqa: E402

if __name__ == "__main__":
    comm = mg.init_distributed() if int(os.environ.get("WORLD_SIZE", "1")) > 1 else mg.get_world_comm()
    true_params = torch.tensor([-2.0, -0.5])
    data = make_docs_data(true_params=tuple(true_params.tolist()), comm=comm)
    model = DocsSMFModel(aux_data=data, comm=comm)
    print_root = comm.rank == 0
    loss, grad = model.calc_loss_and_grad_from_params(true_params + 0.1)
    init_params = true_params + torch.tensor([-1.5, 0.7])
    results = model.run_bfgs(init_params)
    if print_root:
        print("loss, grad at truth+0.1:", float(loss), grad.tolist())
        print("BFGS has converged:", results.success)
        print("Initial guess =", init_params.tolist())
        print("True params =", true_params.tolist())
        print("Converged params =", results.x)
        print(results)
