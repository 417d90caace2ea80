import sys, os
sys.path[:0] = ['.', 'real-time-gpu-ray-tracer_amd']
import numpy as np, torch
from rtamd import Renderer, scenes
torch.cuda.set_device(0)
s = scenes.demo_with_particles(10)
W, H = 400, 232
for joiners in (1, 0, 1):
  for trial in range(2):
    r = Renderer(s).build_acceleration_structure(0).configure_camera(W, H, ray_trace_depth=2)
    r.set_option("joiners", joiners)
    full, _, _ = r.render(0)
    for count, tw, th in ((2, 64, 64), (3, 64, 32), (8, 32, 32)):
        slab_tiles = max(r.tiles_for_rank(tw, th, k, count) for k in range(count))
        slab_px = slab_tiles * tw * th
        gathered = torch.zeros(count * slab_px * 4, dtype=torch.uint8, device="cuda")
        pix = []
        for k in range(count):
            _, _, st = r.render(0, tiles=(tw, th, k, count), rgba8_device=gathered.data_ptr() + k * slab_px * 4,
                     skip_update=True, want_rgba=False)
            pix.append(st["pixels"])
        frame = torch.zeros(W * H * 4, dtype=torch.uint8, device="cuda")
        r.assemble_tiles(gathered.data_ptr(), slab_tiles, tw, th, count, frame.data_ptr())
        r.synchronize(); torch.cuda.synchronize()
        f = frame.cpu().numpy().reshape(H, W, 4)
        bad = np.argwhere((f != full).any(axis=2))
        g = gathered.cpu().numpy().reshape(count, slab_px, 4)
        zero_slab = [(k, int((g[k, :, 3] == 0).sum())) for k in range(count)]
        print(joiners, trial, count, tw, th, 'bad px', len(bad), 'pixels', pix, 'zero alpha per slab', zero_slab,
              'bad tiles', sorted(set((int(y)//th)*((W+tw-1)//tw)+int(x)//tw for y, x in bad))[:20], flush=True)
    r.cleanup()
