"""Parallel layer: communicators, sub-communicator groups, device collectives."""
from .comm import (Comm, SerialComm, TorchComm, SUM, MAX, MIN, PROD, IN_PLACE, get_world_comm,
                   set_world_comm, init_distributed, launcher_env, is_distributed)
from .subcomm import (reduce_sum, split_subcomms, split_subcomms_by_node, scatter_nd,
                      distribute_data)

__all__ = ["Comm", "SerialComm", "TorchComm", "SUM", "MAX", "MIN", "PROD", "IN_PLACE",
           "get_world_comm", "set_world_comm", "init_distributed", "launcher_env",
           "is_distributed", "reduce_sum", "split_subcomms", "split_subcomms_by_node",
           "scatter_nd", "distribute_data"]
