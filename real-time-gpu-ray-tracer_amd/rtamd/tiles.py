"""Screen-tile sharding bookkeeping for multi-GPU frames, through the library.

Tiles of tile_w x tile_h cover the frame in row-major tile order; rank r of N owns tiles
t = r, r + N, r + 2N, ...  A rank's slab is its tiles back to back, each row-major inside the
tile, padded to the largest slab so that every rank contributes the same byte count to the
gather.  The mapping from slab pixels to frame pixels is the library's own (rt_tile_pixels /
rt_slab_tiles, csrc/layout.hpp tile_pixel: the function the assemble kernel uses), so host-side
tools and the CPU protocol tests exercise the product's bookkeeping.  Host-only: no GPU needed.
"""
from __future__ import annotations

import numpy as np

from . import abi


def tiles_xy(width, height, tw, th):
    return (width + tw - 1) // tw, (height + th - 1) // th


def rank_tiles(width, height, tw, th, rank, count):
    nx, ny = tiles_xy(width, height, tw, th)
    return list(range(rank, nx * ny, count))


def tiles_for_rank(width, height, tw, th, rank, count):
    return len(rank_tiles(width, height, tw, th, rank, count))


def slab_tiles(width, height, tw, th, count):
    """Tiles per padded slab (rt_slab_tiles)."""
    return int(abi.load_library().rt_slab_tiles(width, height, tw, th, count))


def slab_pixels(width, height, tw, th, rank, count):
    """(slab_px, 2) int32: frame (x, y) of each pixel of rank's slab, (-1, -1) outside the frame
    (rt_tile_pixels)."""
    lib = abi.load_library()
    n = slab_tiles(width, height, tw, th, count) * tw * th
    xy = np.zeros((n, 2), np.int32)
    abi.check(lib, lib.rt_tile_pixels(width, height, tw, th, rank, count, 0, n, xy.ctypes.data))
    return xy


def tile_origin(t, width, tw, th):
    nx = (width + tw - 1) // tw
    return (t % nx) * tw, (t // nx) * th


def pack(frame_region_fn, width, height, tw, th, rank, count):
    """A rank's slab from frame pixels: frame_region_fn() -> (height, width, 4) frame (only the rank's
    pixels need be valid); pixels outside the frame stay 0."""
    xy = slab_pixels(width, height, tw, th, rank, count)
    frame = frame_region_fn()
    slab = np.zeros((xy.shape[0], 4), np.uint8)
    ok = xy[:, 0] >= 0
    slab[ok] = frame[xy[ok, 1], xy[ok, 0]]
    return slab


def assemble(gathered, width, height, tw, th, count):
    """gathered: uint8 array (count, slab_px, 4) -> frame (height, width, 4), scattered with the
    library's slab -> frame mapping (what the assemble kernel does on the GPU)."""
    frame = np.zeros((height, width, 4), np.uint8)
    for r in range(count):
        xy = slab_pixels(width, height, tw, th, r, count)
        ok = xy[:, 0] >= 0
        frame[xy[ok, 1], xy[ok, 0]] = gathered[r][ok]
    return frame
