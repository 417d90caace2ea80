"""Screen-tile sharding bookkeeping for multi-GPU frames.

Tiles of tile_w x tile_h cover the frame in row-major tile order; rank r of N owns tiles
t = r, r + N, r + 2N, ...  A rank's slab is its tiles back to back, each row-major inside the
tile, padded to the largest slab so that every rank contributes the same byte count to the
gather.  These functions restate rt_tiles_for_rank / the kernel's tile addressing / the
assemble kernel (csrc/assemble.hip) for host-side use and CPU tests.
"""
from __future__ import annotations

import numpy as np


def tiles_xy(width, height, tw, th):
    return (width + tw - 1) // tw, (height + th - 1) // th


def rank_tiles(width, height, tw, th, rank, count):
    nx, ny = tiles_xy(width, height, tw, th)
    return list(range(rank, nx * ny, count))


def tiles_for_rank(width, height, tw, th, rank, count):
    return len(rank_tiles(width, height, tw, th, rank, count))


def slab_tiles(width, height, tw, th, count):
    return max(tiles_for_rank(width, height, tw, th, r, count) for r in range(count))


def tile_origin(t, width, tw, th):
    nx = (width + tw - 1) // tw
    return (t % nx) * tw, (t // nx) * th


def assemble(gathered, width, height, tw, th, count):
    """gathered: uint8 array (count, slab_tiles * tw * th, 4) -> frame (height, width, 4)."""
    frame = np.zeros((height, width, 4), np.uint8)
    for r in range(count):
        for k, t in enumerate(rank_tiles(width, height, tw, th, r, count)):
            x0, y0 = tile_origin(t, width, tw, th)
            tile = gathered[r, k * tw * th:(k + 1) * tw * th].reshape(th, tw, 4)
            h = min(th, height - y0)
            w = min(tw, width - x0)
            frame[y0:y0 + h, x0:x0 + w] = tile[:h, :w]
    return frame
