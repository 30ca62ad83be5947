"""Keys that tie a PMC traffic profile (tools/pmc_traffic.py, profiles/pmc/*.json) to the
exact launch a bench line times: the workload (scene, frame size, spp) and the kernel
(precision, the traversal flags the scene actually runs -- rt_scene_info.render_traversal
-- its block, the work-queue knobs and, for meshes, the tree).  bench.py takes
roofline.traffic only from a profile whose keys both match; tools/profile_target.py
prints the same keys so that the PMC passes can be filed under them."""
from __future__ import annotations


def pmc_workload_key(scene: str, mesh_level: int, W: int, H: int, spp: int) -> str:
    return f"{W}x{H}x{spp}" if scene == "random" else f"{scene}{mesh_level}:{W}x{H}x{spp}"


def pmc_tuning_key(tun, info, mesh_builder: str = "host", precision: str = "f32") -> str:
    mesh = info.num_triangles > 0
    key = f"{precision},queue,ib={(tun.mesh_item_balance if mesh else tun.item_balance):g},is={tun.item_samples}"
    key += f",kernel={info.render_traversal},block={info.render_block},refill={tun.coh_refill}"
    if mesh:
        key += (f",bvh4,leaf={tun.mesh_max_leaf},cost={tun.mesh_cost_traverse:g},builder={mesh_builder},"
                f"mstack={tun.mesh_lds_stack},"
                # the LDS tree top exists only in TRAV_MTOP kernels (4096; before r03u: always)
                f"mlds={tun.mesh_lds_nodes if info.render_traversal & 4096 else 'off'}")
    else:
        key += f",leaf={tun.max_leaf},cost={tun.cost_intersect:g}"
    return key
