"""Back-to-back launches of one shard (no host sync in between) vs synchronised launches,
for shards of N = 1 and 8, and the full frame at a few spp."""
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from raytracingproject_amd import _native as N  # noqa: E402
from raytracingproject_amd import api, rtweekend, scenes  # noqa: E402

import torch  # noqa: E402

rtweekend.reset_stream()
S, M = api.flatten(scenes.random_spheres())
r = N.Renderer(0, 0x5EED, N.RT_PREC_F32)
r.upload_scene(S, M)
for spp, n, reps in ((256, 1, 4), (256, 8, 24), (32, 1, 24), (2048, 8, 3)):
    cam_api = scenes.main_camera()
    cam_api.image_width, cam_api.samples_per_pixel = 1920, spp
    cam = cam_api.native
    full = N.shard_layout(cam.image_width, cam.image_height, 0, 1)
    out = torch.empty(full.max_shard_tiles * 64 * 3, dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    for _ in range(2):
        r.render(cam, spp, 50, 0, n, out.data_ptr())
    sync = []
    for _ in range(3):
        r.render(cam, spp, 50, 0, n, out.data_ptr())
        sync.append(r.last_kernel_ms())
    t0 = time.perf_counter()
    for _ in range(reps):
        r.render(cam, spp, 50, 0, n, out.data_ptr())
    r.last_kernel_ms()
    dt = (time.perf_counter() - t0) / reps * 1e3
    rays = cam.image_width * cam.image_height * spp / n
    print(json.dumps({"spp": spp, "n": n, "sync_kernel_ms": round(min(sync), 3), "back_to_back_ms": round(dt, 3),
                      "mrays_per_gpu_b2b": round(rays / dt / 1e3, 1)}), flush=True)
r.close()
