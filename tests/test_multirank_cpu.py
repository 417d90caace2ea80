"""World-size-2 gloo test of the multi-GPU frame protocol on CPU.

Each rank fills only its interleaved screen tiles, packed into a padded tile-compact slab through the
library's own slab -> frame mapping (rt_slab_tiles / rt_tile_pixels, csrc/layout.hpp tile_pixel — the
function the trace kernel's tile map and the assemble kernel use); the slabs are gathered to rank 0 as the
library's RCCL chain does, and rank 0 assembles the frame with the same mapping.  A pixel's content is a
function of its frame position and the frame number only (as a traced pixel is: the RNG is keyed by the
global padded pixel index), so the assembled frame must equal that function over the whole frame for any
world size.  No renderer runs here: the GPU chain itself is tested in tests/test_gpu_multigpu.py.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from rtamd import tiles

W, H, TW, TH = 200, 120, 64, 32


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def pixel_values(frame):
    """(H, W, 4) uint8: a pixel's content as a function of (x, y, frame) only, distinct for every pixel."""
    y, x = np.mgrid[0:H, 0:W]
    return np.stack([x & 255, y & 255, ((x >> 8) | ((y >> 8) << 4)) ^ (frame & 15),
                     np.full_like(x, 255 - (frame & 127))], axis=-1).astype(np.uint8)


def _render_slab(frame, rank, count):
    """The rank's slab: only its own tiles' pixels are taken (through rt_tile_pixels); the rest of the
    canvas is poisoned, so a pixel landing in another rank's tile shows up in the assembled frame."""
    mine = np.zeros((H, W), bool)
    for t in tiles.rank_tiles(W, H, TW, TH, rank, count):
        x0, y0 = tiles.tile_origin(t, W, TW, TH)
        mine[y0:y0 + TH, x0:x0 + TW] = True
    canvas = np.where(mine[..., None], pixel_values(frame), np.uint8(0xAB))
    return tiles.pack(lambda: canvas, W, H, TW, TH, rank, count)


def _worker(rank, world, port, result_path):
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [repo, os.path.join(repo, "real-time-gpu-ray-tracer_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    slab = torch.from_numpy(_render_slab(5, rank, world))
    gather = [torch.zeros_like(slab) for _ in range(world)] if rank == 0 else None
    dist.gather(slab, gather, dst=0)
    if rank == 0:
        g = torch.stack(gather).numpy()
        frame = tiles.assemble(g, W, H, TW, TH, world)
        np.save(result_path, np.stack([frame, pixel_values(5)]))
    dist.barrier()
    dist.destroy_process_group()


def _pipelined_worker(rank, world, port, result_path):
    """bench.py's N > 1 loop: double-buffered slabs, frame k's gather issued async and completed
    (then assembled on rank 0) only after frame k + 1 has been rendered into the other slab."""
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [repo, os.path.join(repo, "real-time-gpu-ray-tracer_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    st = tiles.slab_tiles(W, H, TW, TH, world)
    slabs = [torch.zeros(st * TW * TH, 4, dtype=torch.uint8) for _ in range(2)]
    gathered = [[torch.zeros_like(slabs[0]) for _ in range(world)] if rank == 0 else None for _ in range(2)]
    frames, pending = [], []

    def finish():
        if pending:
            work, g, f = pending.pop()
            work.wait()
            if rank == 0:
                frames.append((f, tiles.assemble(torch.stack(g).numpy(), W, H, TW, TH, world)))

    for f in range(3):
        b = f % 2
        slabs[b].copy_(torch.from_numpy(_render_slab(f, rank, world)))
        work = dist.gather(slabs[b], gathered[b], dst=0, async_op=True)
        finish()
        pending.append((work, gathered[b], f))
    finish()
    if rank == 0:
        out = []
        for f, frame in frames:
            out.append(np.stack([frame, pixel_values(f)]))
        np.save(result_path, np.stack(out))
    dist.barrier()
    dist.destroy_process_group()


def _lanes_worker(rank, world, port, result_path, nl=3):
    """bench.py's N > 1 loop with option "overlap" = nl lanes: frame f runs on lane f % nl, whose
    chain is trace into slabs[lane] -> gather into gathered[lane] (waited in lane order) -> assemble
    into frame_bufs[lane] on rank 0; a lane's buffers are reused only by its next frame."""
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [repo, os.path.join(repo, "real-time-gpu-ray-tracer_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    st = tiles.slab_tiles(W, H, TW, TH, world)
    slabs = [torch.zeros(st * TW * TH, 4, dtype=torch.uint8) for _ in range(nl)]
    gathered = [[torch.zeros_like(slabs[0]) for _ in range(world)] if rank == 0 else None for _ in range(nl)]
    frame_bufs = [np.zeros((H, W, 4), np.uint8) for _ in range(nl)]
    out = []
    for f in range(2 * nl):
        b = f % nl
        slabs[b].copy_(torch.from_numpy(_render_slab(f, rank, world)))
        dist.gather(slabs[b], gathered[b], dst=0, async_op=True).wait()
        if rank == 0:
            frame_bufs[b][:] = tiles.assemble(torch.stack(gathered[b]).numpy(), W, H, TW, TH, world)
            if f >= nl:       # lane b's previous frame has been replaced by frame f
                out.append(np.stack([frame_bufs[b].copy(), pixel_values(f)]))
    if rank == 0:
        np.save(result_path, np.stack(out))
    dist.barrier()
    dist.destroy_process_group()


def test_overlap_lanes_gather_gloo(tmp_path):
    out = str(tmp_path / "res.npy")
    mp.spawn(_lanes_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    res = np.load(out)
    assert res.shape[0] == 3
    for frame, full in res:
        assert np.array_equal(frame, full)


def test_pipelined_gather_gloo(tmp_path):
    out = str(tmp_path / "res.npy")
    mp.spawn(_pipelined_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    res = np.load(out)
    assert res.shape[0] == 3
    for frame, full in res:
        assert np.array_equal(frame, full)


@pytest.mark.parametrize("world", [2, 3])
def test_tile_gather_assemble_gloo(tmp_path, world):
    out = str(tmp_path / "res.npy")
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    frame, full = np.load(out)
    assert np.array_equal(frame, full)


def test_tile_bookkeeping_covers_frame_once():
    """The library's slab -> frame mapping (rt_tile_pixels) puts every frame pixel in exactly one slab
    pixel of exactly one rank, agrees with the row-major tile restatement, and rt_slab_tiles is the
    largest rank's tile count."""
    for w, h in ((W, H), (1920, 1080), (64, 64), (65, 7)):
        for count in (1, 2, 3, 8):
            seen = np.zeros((h, w), int)
            st = tiles.slab_tiles(w, h, TW, TH, count)
            assert st == max(tiles.tiles_for_rank(w, h, TW, TH, r, count) for r in range(count))
            for r in range(count):
                xy = tiles.slab_pixels(w, h, TW, TH, r, count)
                assert xy.shape == (st * TW * TH, 2)
                ok = xy[:, 0] >= 0
                np.add.at(seen, (xy[ok, 1], xy[ok, 0]), 1)
                for k, t in enumerate(tiles.rank_tiles(w, h, TW, TH, r, count)[:3]):
                    x0, y0 = tiles.tile_origin(t, w, TW, TH)
                    p = xy[k * TW * TH]
                    assert tuple(p) == (x0, y0)
            assert (seen == 1).all(), (w, h, count)
