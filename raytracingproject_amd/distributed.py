"""Multi-GPU framebuffer split: one process per GPU, 8x8 tiles dealt
round-robin (tile t -> rank t % N, so every rank gets the same mix of expensive and cheap
regions), finished shard buffers gathered to rank 0 with torch.distributed (backend
"nccl" = RCCL over xGMI on the MI355X node; "gloo" in the CPU tests), then un-interleaved
on rank 0 (rt_unshard on the device; unshard_host here for host buffers).

The per-(pixel, sample) RNG is keyed by the global pixel index, so the frame is
bit-identical for any N (tests/test_gpu_parity.py::test_tiling_is_invisible).
"""
from __future__ import annotations

import numpy as np

TILE = 8


def layout(width: int, height: int, rank: int, world: int) -> dict:
    """Pure-Python mirror of rt_shard_layout (include/rt_hip.h)."""
    if width <= 0 or height <= 0 or world <= 0 or not 0 <= rank < world:
        raise ValueError("bad layout arguments")
    tx, ty = -(-width // TILE), -(-height // TILE)
    n = tx * ty
    return {"tiles_x": tx, "tiles_y": ty, "num_tiles": n, "shard_tiles": -(-(n - rank) // world),
            "max_shard_tiles": -(-n // world)}


def shard_pixels(width: int, height: int, rank: int, world: int) -> np.ndarray:
    """(x, y) of every slot of this rank's shard buffer, in buffer order; (-1, -1) for the
    slots of a tile that fall outside the image."""
    L = layout(width, height, rank, world)
    lt = np.arange(L["shard_tiles"])
    t = lt * world + rank
    lane = np.arange(TILE * TILE)
    x = (t % L["tiles_x"])[:, None] * TILE + (lane % TILE)[None, :]
    y = (t // L["tiles_x"])[:, None] * TILE + (lane // TILE)[None, :]
    inside = (x < width) & (y < height)
    xy = np.stack([np.where(inside, x, -1), np.where(inside, y, -1)], axis=-1)
    return xy.reshape(-1, 2)


def unshard_host(gathered: np.ndarray, width: int, height: int, world: int, channels: int = 3) -> np.ndarray:
    """Host restatement of rt_unshard: N stacked shard buffers -> [H, W, C] frame."""
    L = layout(width, height, 0, world)
    per = L["max_shard_tiles"] * TILE * TILE
    g = gathered.reshape(world, per, channels)
    frame = np.zeros((height, width, channels), dtype=gathered.dtype)
    for r in range(world):
        xy = shard_pixels(width, height, r, world)
        ok = xy[:, 0] >= 0
        frame[xy[ok, 1], xy[ok, 0]] = g[r, : len(xy)][ok]
    return frame


class FrameGather:
    """Shard buffer of this rank and, on rank 0, the stacked receive buffer, as torch
    tensors on `device`; gather() is the one exchange step of the path."""

    def __init__(self, torch, dist, width: int, height: int, rank: int, world: int, device, dtype,
                 channels: int = 3):
        self.torch, self.dist = torch, dist
        self.rank, self.world = rank, world
        L = layout(width, height, rank, world)
        self.elems = L["max_shard_tiles"] * TILE * TILE * channels
        self.shard = torch.zeros(self.elems, dtype=dtype, device=device)
        self.gathered = torch.zeros(world * self.elems, dtype=dtype, device=device) if rank == 0 else None
        self._views = list(self.gathered.split(self.elems)) if rank == 0 else None

    def gather(self, group=None):
        """Rank 0 receives every shard (its own included) into `gathered` (over `group`,
        default: the default process group)."""
        if self.world == 1:
            self.gathered.copy_(self.shard) if self.gathered is not None else None
            return self.gathered
        self.dist.gather(self.shard, self._views if self.rank == 0 else None, dst=0, group=group)
        return self.gathered
