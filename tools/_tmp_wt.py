import json, os, sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np
out = Path(sys.argv[1])
from raytracingproject_amd import _native as N
from raytracingproject_amd import api, rtweekend, scenes
import torch
rtweekend.reset_stream()
S, M = api.flatten(scenes.random_spheres())
r = N.Renderer(0, 0x5EED, N.RT_PREC_F32)
r.upload_scene(S, M)
for spp, n in ((256, 8), (256, 1), (2048, 8)):
    cam_api = scenes.main_camera(); cam_api.image_width, cam_api.samples_per_pixel = 1920, spp
    cam = cam_api.native
    full = N.shard_layout(cam.image_width, cam.image_height, 0, 1)
    buf = torch.empty(full.max_shard_tiles * 64 * 3, dtype=torch.float32, device="cuda")
    r.render(cam, spp, 50, 0, n, buf.data_ptr()); r.last_kernel_ms()
    f = out / f"wt_{spp}_{n}.bin"
    os.environ["RT_WAVE_TIMES"] = str(f)
    r.render(cam, spp, 50, 0, n, buf.data_ptr()); ms = r.last_kernel_ms()
    os.environ["RT_WAVE_TIMES"] = ""
    t = np.fromfile(f, dtype=np.uint64).reshape(-1, 4).astype(np.int64)
    t = t[t[:, 2] > 0]
    t0 = t[:, 0].min()
    b, e, z = (t[:, 0] - t0) / 1e5, (t[:, 2] - t0) / 1e5, (t[:, 1][t[:, 1] > 0] - t0) / 1e5   # ms (100 MHz)
    q = lambda x, p: round(float(np.percentile(x, p)), 3)
    print(json.dumps({"spp": spp, "n": n, "kernel_ms": round(ms, 3), "waves": len(t),
                      "start_ms p50/p100": [q(b, 50), q(b, 100)],
                      "queue_empty_ms min/p50": [q(z, 0), q(z, 50)] if len(z) else None,
                      "end_ms min/p10/p50/p90/max": [q(e, 0), q(e, 10), q(e, 50), q(e, 90), q(e, 100)]}), flush=True)
r.close()
