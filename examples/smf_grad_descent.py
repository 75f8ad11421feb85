"""Fit the 2-parameter stellar mass function by gradient descent (reference
tests/smf_example/smf_grad_descent.py), on the HIP SMF kernel when a GPU is present.

    python examples/smf_grad_descent.py --num-halos 1000000
    python -m multigrad_amd.launch -n 8 examples/smf_grad_descent.py --num-halos 100000000
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import multigrad_amd as mg  # noqa: E402
from multigrad_amd.models.smf import MySMFModel, ParamTuple, make_test_data  # noqa: E402

parser = argparse.ArgumentParser(__file__, description="Example pipeline fitting the SMF")
parser.add_argument("--num-halos", type=int, default=10_000)
parser.add_argument("--num-steps", type=int, default=2000)
parser.add_argument("--learning-rate", type=float, default=1e-3)
parser.add_argument("--plots", action="store_true")

if __name__ == "__main__":
    args = parser.parse_args()
    comm = mg.init_distributed() if int(os.environ.get("WORLD_SIZE", "1")) > 1 else mg.get_world_comm()
    data = make_test_data(args.num_halos, comm=comm)
    model = MySMFModel(aux_data=data, comm=comm)
    guess = ParamTuple(log_shmrat=-1, sigma_logsm=0.5)
    t0 = time.time()
    gd = model.run_simple_grad_descent(guess=guess, nsteps=args.num_steps,
                                       learning_rate=args.learning_rate)
    t = time.time() - t0
    truth = ParamTuple(log_shmrat=-2.0, sigma_logsm=0.2)
    final = ParamTuple(*gd.params[-1].tolist())
    true_smf = model.calc_sumstats_from_params(truth)
    if comm.rank == 0:
        print(f"Initial guess: {guess} ... {t:.3f} seconds later ...")
        print(f"Final solution: {final}")
        print(f"Truth: {truth}")
        print(f"True SMF: {true_smf.tolist()}")
        if args.plots:
            try:
                import matplotlib.pyplot as plt
            except ImportError:
                print("matplotlib is not installed; skipping plots")
            else:
                plt.plot(gd.loss.cpu().numpy())
                plt.semilogy()
                plt.xlabel("step")
                plt.ylabel("loss")
                plt.savefig("gd_loss.png", bbox_inches="tight")
