"""Build the native library in-tree: raytracingproject_amd/lib/librt_hip.so.

hipcc cross-compiles for gfx950 (MI355X) without a GPU present.  The two kernel
translation units differ only in FP contraction: the fp32 fast path may fuse into FMAs,
the fp64 reference-exact path may not (-ffp-contract=off) so that its roundings are
those of the g++-built reference.
"""
from __future__ import annotations

import os
import subprocess
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
OBJ = PKG / "build"
LIB = PKG / "lib" / "librt_hip.so"
ARCH = os.environ.get("RT_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

COMMON = ["-x", "hip", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall",
          "-Wno-unused-function", f"-I{ROOT / 'include'}"] + os.environ.get("RT_HIPCC_EXTRA", "").split()
UNITS = {
    "rt_render_f32.hip": ["-fno-hip-fp32-correctly-rounded-divide-sqrt", "-fgpu-flush-denormals-to-zero",
                          os.environ.get("RT_F32_CONTRACT", "-ffp-contract=on")],
    "rt_render_f64.hip": ["-ffp-contract=off"],
    "rt_abi.cpp": ["-ffp-contract=off"],
    "rt_bvh.cpp": ["-ffp-contract=off"],
    "rt_obj.cpp": ["-ffp-contract=off"],
    "rt_lbvh.hip": ["-ffp-contract=off"],
    "rt_comm.cpp": [],
}
HEADERS = ["rt_device.h", "rt_render_impl.h", "rt_scene.h", "rt_launch.h", "rt_bvh.h", "rt_lbvh.h", "rt_ctx.h",
           "rt_treelet.h"]


def _stale(target: Path, deps: list[Path]) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def _compile(src: str, extra: list[str], verbose: bool) -> Path:
    obj = OBJ / (src.rsplit(".", 1)[0] + ".o")
    # build.py itself: a changed flag rebuilds every object
    deps = [CSRC / src] + [CSRC / h for h in HEADERS] + [ROOT / "include" / "rt_hip.h", Path(__file__)]
    if _stale(obj, deps):
        cmd = [HIPCC, *COMMON, *extra, "-c", str(CSRC / src), "-o", str(obj)]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    return obj


def build_native(verbose: bool = False) -> Path:
    OBJ.mkdir(parents=True, exist_ok=True)
    LIB.parent.mkdir(parents=True, exist_ok=True)
    with ThreadPoolExecutor(max_workers=4) as ex:
        objs = list(ex.map(lambda kv: _compile(kv[0], kv[1], verbose), UNITS.items()))
    if _stale(LIB, objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(LIB), *map(str, objs),
               "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    return LIB


def build_dropin(verbose: bool = False) -> list[Path]:
    """C++ programs over the drop-in headers (include/rt) linked to librt_hip.so:
    examples/pixelmatch.cpp always; and, where /root/reference exists, the reference's
    own src/main.cpp compiled UNCHANGED against include/rt (fed on stdin from the
    include/rt directory so that its quoted includes resolve to the drop-in headers;
    nothing is copied)."""
    out_dir = ROOT / "examples" / "_build"
    out_dir.mkdir(parents=True, exist_ok=True)
    inc = ROOT / "include" / "rt"
    link = [f"-L{LIB.parent}", "-lrt_hip", f"-Wl,-rpath,{LIB.parent}", "-Wl,-rpath,$ORIGIN/../../raytracingproject_amd/lib"]
    built = []
    exe = out_dir / "pixelmatch"
    src = ROOT / "examples" / "pixelmatch.cpp"
    if _stale(exe, [src, LIB, *inc.glob("*.h")]):
        subprocess.run(["g++", "-O2", "-std=c++17", f"-I{inc}", str(src), "-o", str(exe), *link], check=True)
    built.append(exe)
    exe = out_dir / "host_queries"
    src = ROOT / "examples" / "host_queries.cpp"
    if _stale(exe, [src, LIB, *inc.glob("*.h")]):
        subprocess.run(["g++", "-O2", "-std=c++17", f"-I{inc}", str(src), "-o", str(exe), *link], check=True)
    built.append(exe)
    exe = out_dir / "mesh_scene"
    src = ROOT / "examples" / "mesh_scene.cpp"
    if _stale(exe, [src, LIB, *inc.glob("*.h")]):
        subprocess.run(["g++", "-O2", "-std=c++17", f"-I{inc}", str(src), "-o", str(exe), *link], check=True)
    built.append(exe)
    ref_main = Path("/root/reference/src/main.cpp")
    if ref_main.exists():
        exe = out_dir / "reference_main_on_mi355x"
        if _stale(exe, [ref_main, LIB, *inc.glob("*.h")]):
            with open(ref_main, "rb") as f:
                subprocess.run(["g++", "-O2", "-std=c++17", "-x", "c++", "-", f"-I{inc}", "-o", str(exe), *link],
                               check=True, stdin=f, cwd=inc)
        built.append(exe)
    return built


SAN_FLAGS = ["-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
             "-fno-sanitize-recover=all"]
SAN_EXE = OBJ / "san" / "san_driver"


def build_sanitize(verbose: bool = False) -> Path:
    """Host-only sanitizer build (the reference's ASan flags are commented
    out, CMakeLists.txt:18-23): the product's host sources that take untrusted input or
    build the trees (csrc/rt_obj.cpp, csrc/rt_bvh.cpp) and the oracle (oracle/rt_oracle.c)
    compiled with g++/gcc -fsanitize=address,undefined into one driver,
    tests/cpp/sanitize_driver.cpp (run by tests/test_sanitize.py).  No GPU code."""
    out = SAN_EXE.parent
    out.mkdir(parents=True, exist_ok=True)
    srcs = [ROOT / "tests" / "cpp" / "sanitize_driver.cpp", CSRC / "rt_obj.cpp", CSRC / "rt_bvh.cpp"]
    orc = ROOT / "oracle" / "rt_oracle.c"
    deps = srcs + [orc, CSRC / "rt_bvh.h", CSRC / "rt_scene.h", ROOT / "include" / "rt_hip.h",
                   ROOT / "oracle" / "rt_oracle.h", Path(__file__)]
    if _stale(SAN_EXE, deps):
        oo = out / "rt_oracle.o"
        cmd = ["gcc", "-std=c11", *SAN_FLAGS, "-c", str(orc), "-o", str(oo)]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        cmd = ["g++", "-std=c++17", *SAN_FLAGS, f"-I{ROOT / 'include'}", *map(str, srcs), str(oo), "-o",
               str(SAN_EXE), "-lm"]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    return SAN_EXE


def build_oracle(verbose: bool = False) -> None:
    """Compile the C restatement (test infrastructure) and, where /root/reference is
    present, the reference driver into oracle/_ref (test infrastructure: oracle/_ref/
    ref_golden ships to the GPU box as bench.py's CPU-baseline binary, and the product
    never loads either)."""
    oracle = ROOT / "oracle"
    out = None if verbose else subprocess.DEVNULL
    subprocess.run(["make", "-C", str(oracle), "liboracle.so", "rt_oracle_cli"], check=True, stdout=out)
    if Path("/root/reference/src/main.cpp").exists():
        subprocess.run(["make", "-C", str(oracle), "ref"], check=True, stdout=out)


if __name__ == "__main__":
    import sys
    if "--sanitize" in sys.argv[1:]:
        print(build_sanitize(verbose=True))
        sys.exit(0)
    print(build_native(verbose=True))
    print(build_dropin(verbose=True))
    build_oracle(verbose=True)
