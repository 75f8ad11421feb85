"""Pure-Python tile-schedule builder (mirror of ``csrc/runtime.cpp:build_tiles``; used
only when the native extension is unavailable, and as its test oracle)."""
from __future__ import annotations

import numpy as np
import torch


def build_tiles_py(counts, breaks, tile_halos: int, tile_pops: int):
    cnt = np.asarray(torch.as_tensor(counts).cpu().numpy(), dtype=np.int64)
    J = cnt.size
    brk = sorted({int(b) for b in breaks if 0 < int(b) < J}) + [J]
    tiles, giant = [], []
    chunk_tiles, chunk_giant = [0], [0]
    nslots = 0
    h = 0
    bi = 0
    state = {"tp0": 0, "th0": 0}

    def close(p_end, h_end):
        if p_end > state["tp0"]:
            tiles.append((state["th0"], h_end, state["tp0"], p_end, -1))
        state["tp0"], state["th0"] = p_end, h_end

    for p in range(J):
        n = int(cnt[p])
        if n > tile_halos:
            close(p, h)
            s0 = nslots
            for off in range(0, n, tile_halos):
                tiles.append((h + off, h + min(n, off + tile_halos), p, p + 1, nslots))
                nslots += 1
            giant.append((p, s0, nslots))
            h += n
            state["tp0"], state["th0"] = p + 1, h
        else:
            if h + n - state["th0"] > tile_halos or p + 1 - state["tp0"] > tile_pops:
                close(p, h)
            h += n
        if p + 1 == brk[bi]:
            close(p + 1, h)
            chunk_tiles.append(len(tiles))
            chunk_giant.append(len(giant))
            bi += 1
    if J == 0:
        chunk_tiles.append(0)
        chunk_giant.append(0)
    t = torch.zeros((len(tiles), 4), dtype=torch.int64)
    for i, (h0, h1, p0, p1, slot) in enumerate(tiles):
        t[i, 0], t[i, 1] = h0, h1
        t[i, 2] = (p0 & 0xFFFFFFFF) | (p1 << 32)
        t[i, 3] = slot & 0xFFFFFFFF
    g = torch.tensor(giant, dtype=torch.int32).reshape(-1, 3)
    return t, g, torch.tensor(chunk_tiles), torch.tensor(chunk_giant), nslots


def build_lanes_py(counts, breaks, window: int, lmax: int, order_counts=None):
    """Mirror of ``csrc/runtime.cpp:build_lanes`` (lanes layout schedule); same outputs."""
    lanes = 64
    cnt = np.asarray(torch.as_tensor(counts).cpu().numpy(), dtype=np.int64)
    key = cnt if order_counts is None else \
        np.asarray(torch.as_tensor(order_counts).cpu().numpy(), dtype=np.int64)
    J = cnt.size
    brk = sorted({int(b) for b in breaks if 0 < int(b) < J}) + [J]
    off = np.zeros(J + 1, dtype=np.int64)
    off[1:] = np.cumsum(cnt)
    slot_pop, slot_src, slot_len, slot_part = [], [], [], []
    group_base, group_len = [0], []
    chunk_groups, chunk_giant = [0], [0]
    giant = []
    fwd_order = []
    part_begin = {}
    nparts = 0
    p = 0
    for pend in brk:
        cgroups = []  # (glen, [64 slot tuples]) of this chunk
        for w0 in range(p, pend, window):
            w1 = min(pend, w0 + window)
            items = []
            for q in range(w0, w1):
                n = int(cnt[q])
                if n > lmax:
                    k = -(-n // lmax)
                    items += [(int(key[q]), min(lmax, n - i * lmax), q, i, int(off[q]) + i * lmax)
                              for i in range(k)]
                    giant.append((q, nparts, nparts + k))
                    part_begin[q] = nparts
                    nparts += k
                else:
                    items.append((int(key[q]), n, q, -1, int(off[q])))
            items.sort(key=lambda it: -it[0])  # stable: ties keep population/part order
            padded = -(-len(items) // lanes) * lanes
            for i in range(0, padded, lanes):
                slots = []
                for l in range(lanes):
                    if i + l < len(items):
                        _, n, q, part, src = items[i + l]
                        slots.append((q, n, src, part_begin[q] + part if part >= 0 else -1))
                    else:
                        slots.append((-1, 0, 0, -1))
                cgroups.append((max(sl[1] for sl in slots), slots))
        gbase = len(group_len)
        fwd_order += [gbase + k for k in sorted(range(len(cgroups)), key=lambda k: -cgroups[k][0])]
        for glen, slots in cgroups:  # stored in window order; the forward goes longest first
            for q, n, src, part in slots:
                slot_pop.append(q)
                slot_len.append(n)
                slot_src.append(src)
                slot_part.append(part)
            group_len.append(glen)
            group_base.append(group_base[-1] + glen * lanes)
        p = pend
        chunk_groups.append(len(group_len))
        chunk_giant.append(len(giant))
    pidx_of = {}
    perm, slot_pidx = [], []
    for q in slot_pop:
        if q >= 0 and q not in pidx_of:
            pidx_of[q] = len(perm)
            perm.append(q)
        slot_pidx.append(pidx_of[q] if q >= 0 else -1)
    assert len(perm) == J, "every population needs a slot"
    i32 = lambda v: torch.tensor(v, dtype=torch.int32)  # noqa: E731
    i64 = lambda v: torch.tensor(v, dtype=torch.int64)  # noqa: E731
    g = torch.tensor(giant, dtype=torch.int32).reshape(-1, 3)
    return [i32(slot_pop), i64(slot_src), i32(slot_len), i32(slot_part), i64(group_base),
            i32(group_len), i64(chunk_groups), g, i64(chunk_giant), i32(fwd_order),
            i32(slot_pidx), i32(perm)]


def build_lanes_torch(counts, breaks, window: int, lmax: int, order_counts=None, device=None):
    """The lanes schedule of ``csrc/runtime.cpp:build_lanes`` as a few sorts and scatters on
    ``device`` (the GPU: ~ms at 5e6 populations, where the host builder takes ~1 s), for
    shards without split populations (every count <= ``lmax``); returns None otherwise (the
    caller then uses the host builder).  Same outputs, same order, as device tensors.

    Used to re-lay the lanes out during a fit (engine re-classification), where a host
    rebuild would cost thousands of optimizer steps."""
    dev = torch.device(device) if device is not None else torch.as_tensor(counts).device
    cnt = torch.as_tensor(counts).to(device=dev, dtype=torch.int64).reshape(-1)
    J = int(cnt.numel())
    if J == 0 or bool((cnt > lmax).any()):
        return None
    key = cnt if order_counts is None else \
        torch.as_tensor(order_counts).to(device=dev, dtype=torch.int64).reshape(-1)
    if bool((key < 0).any()) or bool((key >= (1 << 43)).any()):
        return None
    lanes = 64
    brk = sorted({int(b) for b in breaks if 0 < int(b) < J}) + [J]
    starts = [0] + brk[:-1]
    C = len(brk)
    brk_t = torch.tensor(brk, dtype=torch.int64, device=dev)
    q = torch.arange(J, dtype=torch.int64, device=dev)
    c_of = torch.searchsorted(brk_t, q, right=True)              # chunk of each population
    start_t = torch.tensor(starts, dtype=torch.int64, device=dev)
    nwin = [-(-(b - a) // window) for a, b in zip(starts, brk)]
    win_base = torch.tensor([0] + list(np.cumsum(nwin)[:-1]), dtype=torch.int64, device=dev)
    gw = win_base[c_of] + (q - start_t[c_of]) // window          # global window index
    # window ascending, key descending, population ascending (stable sort on a composite)
    comp = gw * (1 << 43) + ((1 << 43) - 1 - key)
    _, order = torch.sort(comp, stable=True)                     # populations in slot order
    W = int(sum(nwin))
    n_w = torch.bincount(gw, minlength=W)
    g_w = (n_w + lanes - 1) // lanes                             # groups per window
    gbase_w = torch.cumsum(g_w, 0) - g_w
    pos_w = torch.cumsum(n_w, 0) - n_w                           # first sorted position
    gw_s = gw[order]
    r = torch.arange(J, dtype=torch.int64, device=dev) - pos_w[gw_s]
    slot = (gbase_w[gw_s] + r // lanes) * lanes + r % lanes
    G = int(g_w.sum())
    S = G * lanes
    off = torch.cumsum(cnt, 0) - cnt
    slot_pop = torch.full((S,), -1, dtype=torch.int32, device=dev)
    slot_pop[slot] = order.to(torch.int32)
    slot_len = torch.zeros(S, dtype=torch.int32, device=dev)
    slot_len[slot] = cnt[order].to(torch.int32)
    slot_src = torch.zeros(S, dtype=torch.int64, device=dev)
    slot_src[slot] = off[order]
    slot_part = torch.full((S,), -1, dtype=torch.int32, device=dev)
    group_len = slot_len.view(G, lanes).amax(1)
    group_base = torch.zeros(G + 1, dtype=torch.int64, device=dev)
    group_base[1:] = torch.cumsum(group_len.to(torch.int64) * lanes, 0)
    # groups per chunk: windows of chunk c are [win_base[c], win_base[c] + nwin[c])
    gcum = torch.cumsum(g_w, 0)
    ends = [int(wb) + n for wb, n in zip(np.cumsum([0] + nwin[:-1]), nwin)]
    chunk_groups = torch.tensor([0] + [int(gcum[e - 1]) if e > 0 else 0 for e in ends],
                                dtype=torch.int64)
    # forward order: each chunk's groups longest first (stable)
    gidx = torch.arange(G, dtype=torch.int64, device=dev)
    cg_t = chunk_groups.to(dev)
    chunk_of_g = torch.searchsorted(cg_t[1:], gidx, right=True)
    gcomp = chunk_of_g * (1 << 32) + ((1 << 31) - group_len.to(torch.int64))
    _, fwd = torch.sort(gcomp, stable=True)
    slot_pidx = torch.full((S,), -1, dtype=torch.int32, device=dev)
    slot_pidx[slot] = torch.arange(J, dtype=torch.int32, device=dev)
    return [slot_pop, slot_src, slot_len, slot_part, group_base, group_len.to(torch.int32),
            chunk_groups, torch.zeros((0, 3), dtype=torch.int32),
            torch.zeros(C + 1, dtype=torch.int64), fwd.to(torch.int32), slot_pidx,
            order.to(torch.int32)]
