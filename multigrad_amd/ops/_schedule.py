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
