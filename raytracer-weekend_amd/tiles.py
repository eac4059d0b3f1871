"""Frame partitioning for N ranks (one process per GPU) — SURVEY.md §8(e).

The frame is cut into 8x8 pixel tiles (tile id = ty * ceil(w/8) + tx, row 0 at the top,
matching lib.rs:58's emission order).  Tiles are dealt round-robin: rank r renders tiles
r, r+N, r+2N, ...  Neighbouring tiles have similar cost (sky vs ground rows), so the
interleave balances ranks to within one tile.  Each rank's packed buffer is padded to
ceil(nt/N) tiles so a single RCCL all-gather (equal sizes) collects the frame; the padding
ids equal nt, which the unpack kernel skips.  Pixels depend only on (seed, j, i, sample),
so the image is bit-identical for any N.
"""
from __future__ import annotations

import numpy as np

TILE = 8


def n_tiles(w: int, h: int) -> int:
    return ((w + TILE - 1) // TILE) * ((h + TILE - 1) // TILE)


def rank_tiles(nt: int, world: int, rank: int) -> np.ndarray:
    return np.arange(rank, nt, world, dtype=np.int32)


def per_rank(nt: int, world: int) -> int:
    return (nt + world - 1) // world


def gather_layout(nt: int, world: int) -> np.ndarray:
    """Tile id of every slot of the all-gathered buffer (rank-major, padded with nt)."""
    pr = per_rank(nt, world)
    out = np.full((world, pr), nt, dtype=np.int32)
    for r in range(world):
        ids = rank_tiles(nt, world, r)
        out[r, :len(ids)] = ids
    return out.reshape(-1)


def tile_pixels(tile: int, w: int, h: int):
    """(row, col) of the 64 lanes of a tile; lane = 8 * (row % 8) + col % 8."""
    tx_n = (w + TILE - 1) // TILE
    tx, ty = tile % tx_n, tile // tx_n
    lane = np.arange(64)
    return ty * TILE + (lane >> 3), tx * TILE + (lane & 7)
