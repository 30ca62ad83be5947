#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes for the render kernel.

python tools/pmc_traffic.py OUT_JSON DIR1 [DIR2 ...] [--key WxHxSPP] [--tuning KEY] [--meta META_JSON]
(--meta: the keys tools/profile_target.py --meta wrote for the profiled launch)
Reads every *counter_collection.csv below the given directories, keeps the dispatches of
render_kernel, and writes per-launch averages.  HBM traffic follows
/opt/skills/guides/MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in KiB and come
from separate passes; on gfx950 FETCH_SIZE reports half the bytes of a wide (16 B/lane)
coalesced read, so it is doubled (the kernel's only bulk reads are 16-B-per-lane scene
copies into LDS).  traffic = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 bytes per launch.
"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path


def main():
    argv = list(sys.argv[1:])
    key = "1920x1080x256"
    tuning = None
    if "--key" in argv:
        i = argv.index("--key")
        key = argv[i + 1]
        del argv[i:i + 2]
    if "--tuning" in argv:
        i = argv.index("--tuning")
        tuning = argv[i + 1]
        del argv[i:i + 2]
    if "--meta" in argv:
        i = argv.index("--meta")
        meta = json.loads(Path(argv[i + 1]).read_text())
        key, tuning = meta["workload"], meta["tuning"]
        del argv[i:i + 2]
    out = Path(argv[0])
    vals = defaultdict(list)
    grid = None
    for d in argv[1:]:
        for f in Path(d).rglob("*counter_collection.csv"):
            for row in csv.DictReader(open(f)):
                if "render_kernel" not in row.get("Kernel_Name", ""):
                    continue
                vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
                grid = row.get("Grid_Size", grid)
    avg = {k: sum(v) / len(v) for k, v in vals.items()}
    res = {"source": [str(p) for p in argv[1:]], "per_launch_avg": avg, "grid_size": grid, "tuning": tuning}
    if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
        b = (2 * avg["FETCH_SIZE"] + avg["WRITE_SIZE"]) * 1024
        res["per_launch_bytes"] = {key: b}
        res["note"] = "bytes = (2*FETCH_SIZE + WRITE_SIZE) KiB * 1024, gfx950 FETCH_SIZE x2 correction"
    out.write_text(json.dumps(res, indent=1) + "\n")
    print(json.dumps(res))


if __name__ == "__main__":
    main()
