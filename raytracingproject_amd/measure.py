"""Keys that tie a PMC traffic profile (tools/pmc_traffic.py, profiles/pmc/*.json) to the
exact launch a bench line times: the workload (scene, frame size, spp) and the kernel
(precision, the traversal flags the scene actually runs -- rt_scene_info.render_traversal
-- its block, the work-queue knobs and, for meshes, the tree).  bench.py takes
roofline.traffic only from a profile whose keys both match; tools/profile_target.py
prints the same keys so that the PMC passes can be filed under them."""
from __future__ import annotations

# Algorithmic work per primary ray of the benchmark configs (SURVEY.md §8(d)'s probe method
# re-derived for the level-7 mesh: tests/work_model.py over tests/cpp/work_model.cpp, the
# oracle's paths with world.hit answered by the product's default host-built trees; 262,144
# primary rays per config; profiles/r04/work_model_r04.json).  hbm_bytes: 128 B per Node4
# visit + 48 B per triangle test (the HBM-resident mesh); lds_bytes: 64 B per sphere-tree
# node visit + 32 B per sphere test (LDS-resident); flop: the survey's cost model + 46 per
# triangle test.  The C3 headline keeps the survey's fixed constants (3,500 FLOP, 4,170 B,
# median-split tree); c3 here is the same count over the product's SAH tree, for reference.
WORK_MODEL = {
    "c3": {"hbm_bytes_per_primary": 0.0, "lds_bytes_per_primary": 2045.533952,
           "flop_per_primary_ray": 2000.041668},
    "c4": {"hbm_bytes_per_primary": 1177.2432640000002, "lds_bytes_per_primary": 64.006592,
           "flop_per_primary_ray": 1074.7209269999998},
    "c5": {"hbm_bytes_per_primary": 1017.803712, "lds_bytes_per_primary": 2118.5797119999997,
           "flop_per_primary_ray": 2838.209495},
}


def pmc_workload_key(scene: str, mesh_level: int, W: int, H: int, spp: int, shards: int = 1) -> str:
    """The workload of ONE launch: a rank of an N-way split renders shard r of N (1/N of
    the tiles, and fp32 meshes double mesh_item_balance on shards with fewer pixels than
    resident lanes), so its counters are not a full frame's: N > 1 gets its own key, and a
    full-frame profile never prices a shard launch."""
    key = f"{W}x{H}x{spp}" if scene == "random" else f"{scene}{mesh_level}:{W}x{H}x{spp}"
    return key if shards <= 1 else f"{key}/shard_of_{shards}"


def pmc_tuning_key(tun, info, mesh_builder: str = "host", precision: str = "f32") -> str:
    mesh = info.num_triangles > 0
    key = f"{precision},queue,ib={(tun.mesh_item_balance if mesh else tun.item_balance):g},is={tun.item_samples}"
    key += f",kernel={info.render_traversal},block={info.render_block},refill={tun.coh_refill}"
    if mesh:
        key += (f",bvh4,leaf={tun.mesh_max_leaf},cost={tun.mesh_cost_traverse:g},builder={mesh_builder},"
                # the resolved LDS stack entries and register budget (auto by default, ABI 7)
                f"mstack={info.render_mesh_lds_stack},wpe={info.render_waves_per_eu},"
                # the LDS tree top exists only in TRAV_MTOP kernels (4096; before r03u: always)
                f"mlds={tun.mesh_lds_nodes if info.render_traversal & 4096 else 'off'}")
    if info.render_traversal & 65536:   # the uniform sphere grid (ABI 8): as built (ABI 10)
        key += f",grid={info.grid_density:g},slabs={info.grid_time_slabs}"
    elif not mesh:
        key += f",leaf={tun.max_leaf},cost={tun.cost_intersect:g}"
    return key
