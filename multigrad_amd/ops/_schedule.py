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
