"""Device-resident ("in-graph") gradient descent -- the mpi4jax variant of the reference.

Reference: ``multigrad/mpi4jax/multigrad.py:17-61`` (``distribute_data``, in-graph
``reduce_sum`` via ``mpi4jax.allreduce``, and ``simple_grad_descent`` as a ``lax.scan``
with in-graph collectives, returning a pandas DataFrame).

Here the "graph" is a HIP graph: the whole step -- user loss/grad function, stream-ordered
all-reduce, parameter update, and the writes of this step's loss and parameters into
preallocated device histories -- is captured once with ``torch.cuda.CUDAGraph`` and
replayed ``nsteps`` times with no host work per step.  On several GPU ranks the
all-reduce is the two-shot peer-memory exchange (:meth:`~multigrad_amd.parallel.xgmi.
TwoShot.all_reduce_`, device-side sequence numbers, so it replays inside the graph);
where that is unavailable (fp64 values, ``MULTIGRAD_TWOSHOT=0``, CPU/gloo) the step runs
eagerly with RCCL/gloo all-reduces enqueued on the compute stream.  Unlike the reference (update on rank 0 then
bcast, which it notes is needed "probably due to a bug"), every rank applies the same
all-reduced update.
"""
from __future__ import annotations

import os
from typing import Callable

import torch

from .parallel.comm import get_world_comm
from .parallel.subcomm import distribute_data as _distribute_data
from .utils.hooks import StepHooks, driver_guard
from .utils.tensors import as_param_tensor

__all__ = ["distribute_data", "reduce_sum", "simple_grad_descent"]


def distribute_data(data, comm=None):
    """This rank's ceil-sized contiguous chunk of ``data``."""
    return _distribute_data(data, comm=get_world_comm() if comm is None else comm)


def _device_allreduce(t: torch.Tensor, comm):
    """The two-shot context that can sum ``t`` over ``comm`` inside a graph, or None."""
    if comm.size < 2 or t.device.type != "cuda" or t.dtype != torch.float32:
        return None
    from .parallel.xgmi import get_twoshot_allreduce
    return get_twoshot_allreduce(comm, t.numel())


def reduce_sum(partial_value: torch.Tensor, comm=None) -> torch.Tensor:
    """Stream-ordered sum over ranks, returning a new tensor.  fp32 CUDA values on several
    ranks go through the two-shot peer-memory exchange, which is capturable into a HIP
    graph and bitwise identical on every rank; others use ``comm.all_reduce``."""
    comm = get_world_comm() if comm is None else comm
    out = partial_value.clone() if not partial_value.is_contiguous() else partial_value
    if comm.size > 1:
        out = out.clone()
        ts = _device_allreduce(out, comm)
        if ts is not None:
            ts.all_reduce_(out)
        else:
            comm.all_reduce(out)
    return out


def simple_grad_descent(data_dict, loss_and_grad_func: Callable, guess, learning_rate=0.01,
                        nsteps=100, comm=None, graph=None, block=None):
    """Fixed-step gradient descent with the whole loop device resident.

    ``loss_and_grad_func(data_dict, params) -> (loss, grad)`` returns this rank's partial
    loss and gradient (summed over ranks here, as in the reference).  Returns a pandas
    DataFrame with columns ``loss`` and ``params`` (one row per step, parameters at
    which the loss was evaluated).  ``block``: steps per captured graph (default
    ``MULTIGRAD_GRAPH_STEPS``, 16); the run replays ``nsteps // block`` block graphs and one
    graph of the remaining steps.
    """
    import pandas as pd

    comm = get_world_comm() if comm is None else comm
    params = as_param_tensor(guess).clone()
    dev = params.device
    n = int(nsteps)
    losses = torch.zeros(n, dtype=params.dtype, device=dev)
    hist = torch.zeros((n,) + tuple(params.shape), dtype=params.dtype, device=dev)
    step = torch.zeros((), dtype=torch.long, device=dev)
    # several ranks: capturable only when the loss/grad vector can take the two-shot path
    ts = _device_allreduce(torch.empty(1 + params.numel(), dtype=params.dtype, device=dev), comm)
    if graph is None:
        graph = dev.type == "cuda" and (comm.size == 1 or ts is not None)
    use_graph = bool(graph)

    def body():
        loss, grad = loss_and_grad_func(data_dict, params)
        lg = torch.cat([torch.as_tensor(loss, dtype=params.dtype, device=dev).reshape(1),
                        torch.as_tensor(grad, dtype=params.dtype, device=dev).reshape(-1)])
        lg = reduce_sum(lg, comm)
        # record (loss, params-at-evaluation) at the device step index, then update
        losses.index_copy_(0, step.reshape(1), lg[:1])
        hist.index_copy_(0, step.reshape(1), params.reshape((1,) + tuple(params.shape)))
        params.sub_(learning_rate * lg[1:].reshape(params.shape))
        step.add_(1)

    done = False
    pins0 = ts.pins if ts is not None else 0
    if use_graph and n > 0:
        saved = params.clone()
        # whole-loop capture in blocks: one graph of K unrolled steps replayed n // K times,
        # plus one graph of the n % K remaining steps (the scan of the reference, without
        # one graph node per optimizer step for long runs)
        K = max(1, min(n, int(block) if block else int(os.environ.get("MULTIGRAD_GRAPH_STEPS", "16"))))
        graphs = []
        try:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):  # warm-up (allocator, lazy init) outside the capture
                body()
            torch.cuda.current_stream().wait_stream(s)
            params.copy_(saved)
            step.zero_()
            for k, reps in ((K, n // K), (n % K, 1)):
                if k == 0 or reps == 0:
                    continue
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    for _ in range(k):
                        body()
                graphs.append((g, reps))
            done = True
        except RuntimeError:
            # the user function is not capturable (host sync, dynamic shapes): run eagerly
            torch.cuda.synchronize()
            params.copy_(saved)
            step.zero_()
        if comm.size > 1 and not all(comm.allgather(done)):
            done = False  # every rank replays or none does (same collective sequence)
            params.copy_(saved)
            step.zero_()
        if done:
            for g, reps in graphs:
                for _ in range(reps):
                    g.replay()
    if not done:
        hooks = StepHooks(comm)  # MULTIGRAD_CHECK_EVERY / MULTIGRAD_METRICS (eager steps)
        with driver_guard(comm):
            for i in range(n):
                body()
                if hooks.active:
                    hooks(i, losses[i], None, lambda: params)
    if use_graph and n > 0:
        del graphs  # the exchanges they recorded no longer pin the cached context
    if ts is not None:
        from .parallel.xgmi import unpin_twoshot_allreduce
        unpin_twoshot_allreduce(ts, ts.pins - pins0)
        ts.check("ingraph.simple_grad_descent", comm)  # a timed-out exchange raises here
    loss_np = losses.detach().cpu().numpy()
    par_np = hist.detach().cpu().numpy()
    return pd.DataFrame(dict(loss=list(loss_np), params=list(par_np)))
