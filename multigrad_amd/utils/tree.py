"""Merger-tree index utilities (reference ``multigrad/diffdesi_experimental/util.py:4-35``).

``find_ultimate_top_indices`` follows host pointers to the root of each forest by
pointer jumping (``idx <- idx[idx]``, at most 50 doublings, so trees up to 2^50 deep);
it runs on the GPU for device tensors.  ``sort_all_by_ultimate_top_dump`` groups arrays by
their ultimate host and ``sort_and_reindex`` remaps index arrays after a permutation.
"""
from __future__ import annotations

import numpy as np
import torch

__all__ = ["find_ultimate_top_indices", "sort_all_by_ultimate_top_dump", "sort_and_reindex"]


def find_ultimate_top_indices(indices, max_recursion: int = 50):
    """Root index of every node of a forest given each node's parent index."""
    is_np = not isinstance(indices, torch.Tensor)
    idx = torch.as_tensor(np.asarray(indices) if is_np else indices).long()
    for _ in range(max_recursion + 1):
        nxt = idx[idx]
        if torch.equal(nxt, idx):
            return idx.numpy() if is_np else idx
        idx = nxt
    raise RecursionError(f"Host search hasn't finished after {max_recursion} steps")


def sort_and_reindex(indices, argsort=None, argsort2=None):
    """Reorder an index array by ``argsort`` and remap its values to the new positions."""
    is_np = not isinstance(indices, torch.Tensor)
    ind = torch.as_tensor(np.asarray(indices) if is_np else indices).long()
    if argsort is None:
        argsort = torch.argsort(ind, stable=True)
    argsort = torch.as_tensor(argsort).long()
    if argsort2 is None:
        argsort2 = torch.argsort(argsort)
    argsort2 = torch.as_tensor(argsort2).long()
    out = argsort2[ind][argsort]
    return out.numpy() if is_np else out


def sort_all_by_ultimate_top_dump(ultimate_dump, arrays_to_sort=(), arrays_to_sort_and_reindex=()):
    """Sort arrays (and re-index index arrays) so that each forest is contiguous."""
    tops = find_ultimate_top_indices(ultimate_dump)
    t = torch.as_tensor(np.asarray(tops) if not isinstance(tops, torch.Tensor) else tops)
    argsort = torch.argsort(t, stable=True)
    argsort2 = torch.argsort(argsort)
    a_np = argsort.numpy()
    sorted_arrays = [np.asarray(x)[a_np] if not isinstance(x, torch.Tensor) else x[argsort]
                     for x in arrays_to_sort]
    reindexed = [sort_and_reindex(x, argsort, argsort2) for x in arrays_to_sort_and_reindex]
    return sorted_arrays, reindexed
