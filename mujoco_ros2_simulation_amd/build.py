"""Build the product shared library libmrs.so in-tree (hipcc, gfx950) and the test oracle.

`python -m mujoco_ros2_simulation_amd.build` compiles every C++/HIP source under csrc/ into
mujoco_ros2_simulation_amd/libmrs.so; objects are cached under build/ keyed on source mtimes.
"""
from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
OBJ = ROOT / "build" / "obj"
LIB = PKG / "libmrs.so"
ARCH = os.environ.get("MRS_OFFLOAD_ARCH", "gfx950")

HIP_SOURCES = ["hip/step.hip", "hip/batch.hip"]
# step.hip is compiled once per part (-DMRS_STEP_PART=n), in parallel: part 0 is the dispatcher, the
# others each instantiate one group width's kernels (17: the G = 16 primal-solver kernel; 18 / 65: the
# G = 16 / 64 kernels with the extended code, MRS_EXT -- MPR contact polish, > 32 ray geoms -- which
# parts 16, 17, 19 and 64 leave out; 19: the G = 16 step kernels with ray helper waves)
STEP_PARTS = [0, 8, 16, 17, 18, 19, 32, 64, 65]
STEP_NO_EXT = {16, 17, 19, 64}
# fp32 division/sqrt via v_rcp/v_sqrt (<= 2.5 ulp) instead of the correctly-rounded sequences:
# the parity tolerance is 1e-5 relative, and the ray/contact math is division-heavy
HIP_FLAGS = ["-fno-hip-fp32-correctly-rounded-divide-sqrt",
             # fp32 denormals flushed: a division then lowers to v_rcp + v_mul instead of the
             # denormal-safe frexp / rcp / ldexp sequence (~1,600 fewer instructions in the G = 16 step
             # kernel; C3 +1.3 %, same-box A/B); values below 1.2e-38 do not occur in the step's state
             "-fgpu-flush-denormals-to-zero"]
CXX_SOURCES = ["capi.cc", "mjcf/compiler.cc", "mjcf/mesh.cc", "mjcf/xml.cc"]
HEADERS = ["hip/devmodel.h", "hip/batch.h", "hip/raymesh.h", "mjcf/model.h", "mjcf/mesh.h", "mjcf/xml.h"]


def _newer(src: Path, dst: Path, deps: list[Path]) -> bool:
    if not dst.exists():
        return True
    t = dst.stat().st_mtime
    # (this file holds the compile flags: a flag change rebuilds every object)
    return src.stat().st_mtime > t or any(d.stat().st_mtime > t for d in deps + [Path(__file__)])


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError("build failed: " + " ".join(cmd))


def _up_to_date(lib: Path, inputs: list[Path]) -> bool:
    """the library exists and is newer than every input: nothing to compile (the GPU box receives the
    in-tree .so but not build/, so without this check it would recompile every object)"""
    return lib.exists() and all(p.stat().st_mtime <= lib.stat().st_mtime for p in inputs)


def build_lib(verbose: bool = False) -> Path:
    deps = [CSRC / h for h in HEADERS] + [ROOT / "include" / "mrs.h", ROOT / "include" / "mrs_model.h"]
    if _up_to_date(LIB, deps + [CSRC / rel for rel in HIP_SOURCES + CXX_SOURCES] + [Path(__file__)]):
        return LIB
    OBJ.mkdir(parents=True, exist_ok=True)
    objs = []
    jobs = []
    units = [(rel, None) for rel in HIP_SOURCES + CXX_SOURCES if rel != "hip/step.hip"]
    units += [("hip/step.hip", part) for part in STEP_PARTS]
    for rel, part in units:
        src = CSRC / rel
        obj = OBJ / (rel.replace("/", "_") + (f".part{part}" if part is not None else "") + ".o")
        objs.append(obj)
        if not _newer(src, obj, deps):
            continue
        if rel.endswith(".hip"):
            extra = [f"-DMRS_STEP_PART={part}", f"-DMRS_EXT={0 if part in STEP_NO_EXT else 1}"] if part is not None else []
            cmd = ["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", *HIP_FLAGS, *extra, "-c", str(src),
                   "-o", str(obj)]
        else:
            cmd = ["hipcc", "-O2", "-std=c++17", "-fPIC", "-Wall", "-c", str(src), "-o", str(obj)]
        jobs.append(cmd)
    procs = [(cmd, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)) for cmd in jobs]
    failed = False
    for cmd, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            failed = True
            sys.stderr.write(out)
        elif verbose and out:
            sys.stderr.write(out)
    if failed:
        raise RuntimeError("build of libmrs.so failed")
    if jobs or not LIB.exists():
        _run(["hipcc", f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(LIB)] + [str(o) for o in objs])
    return LIB


def build_variant(name: str, flags: list[str]) -> Path:
    """an A/B variant libmrs_<name>.so: every step.hip part compiled with extra flags (e.g.
    -DMRS_PHASE_TIMING), linked with the product's other objects (scripts/build_variant.sh)"""
    build_lib()
    vdir = OBJ / f"variant_{name}"
    vdir.mkdir(parents=True, exist_ok=True)
    src = CSRC / "hip" / "step.hip"
    objs, procs = [], []
    # the profiling build keeps one translation unit: its device-side phase counters
    # (g_phase_cycles) must be the one copy every kernel instantiation adds into
    parts = [None] if "-DMRS_PHASE_TIMING" in flags else STEP_PARTS
    for part in parts:
        obj = vdir / f"step.part{part}.o"
        objs.append(obj)
        pflags = [] if part is None else [f"-DMRS_STEP_PART={part}", f"-DMRS_EXT={0 if part in STEP_NO_EXT else 1}"]
        cmd = ["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", *HIP_FLAGS, *pflags,
               *flags, "-c", str(src), "-o", str(obj)]
        procs.append((cmd, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)))
    for cmd, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            sys.stderr.write(out)
            raise RuntimeError("variant build failed: " + " ".join(cmd))
    others = [OBJ / (rel.replace("/", "_") + ".o") for rel in HIP_SOURCES + CXX_SOURCES if rel != "hip/step.hip"]
    lib = PKG / f"libmrs_{name}.so"
    _run(["hipcc", f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(lib)] + [str(o) for o in objs + others])
    return lib


PLUGIN_LIB = PKG / "libmrs_plugin.so"
PLUGIN_SOURCES = ["plugin/src/mujoco_system_interface.cpp", "plugin/src/mujoco_lidar.cpp",
                  "plugin/src/mujoco_cameras.cpp", "plugin/src/mj_types.cpp", "plugin/src/plugin_capi.cc", "mjcf/xml.cc"]


def build_plugin(verbose: bool = False) -> Path:
    """The MujocoSystemInterface plugin host against the ROS API shim (csrc/plugin/ros_shim) and
    libmrs.so; host C++ only (no device code), linked with rpath $ORIGIN."""
    lib = build_lib(verbose)
    srcs = [CSRC / rel for rel in PLUGIN_SOURCES] + [p for p in (CSRC / "plugin").rglob("*.hpp")]
    if _up_to_date(PLUGIN_LIB, srcs + [lib, ROOT / "include" / "mrs_plugin.h"]):
        return PLUGIN_LIB
    inc = [f"-I{CSRC / 'plugin' / 'include'}", f"-I{CSRC / 'plugin' / 'ros_shim'}", f"-I{ROOT / 'include'}"]
    deps = [p for p in (CSRC / "plugin").rglob("*.hpp")] + [ROOT / "include" / "mrs.h", ROOT / "include" / "mrs_model.h",
                                                          ROOT / "include" / "mrs_plugin.h", CSRC / "mjcf" / "xml.h"]
    objs, procs = [], []
    for rel in PLUGIN_SOURCES:
        src = CSRC / rel
        obj = OBJ / ("plugin_" + rel.replace("/", "_") + ".o")
        objs.append(obj)
        if _newer(src, obj, deps):
            cmd = ["g++", "-O2", "-std=c++17", "-fPIC", "-Wall", "-pthread", *inc, "-c", str(src), "-o", str(obj)]
            procs.append((cmd, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)))
    failed = False
    for cmd, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            failed = True
            sys.stderr.write(out)
        elif verbose and out:
            sys.stderr.write(out)
    if failed:
        raise RuntimeError("build of libmrs_plugin.so failed")
    if procs or not PLUGIN_LIB.exists() or PLUGIN_LIB.stat().st_mtime < lib.stat().st_mtime:
        _run(["g++", "-shared", "-fPIC", "-pthread", "-o", str(PLUGIN_LIB), *[str(o) for o in objs],
              f"-L{PKG}", "-lmrs", "-Wl,-rpath,$ORIGIN"])
    return PLUGIN_LIB


def build_oracle() -> Path:
    """TEST INFRASTRUCTURE: the fp64 CPU oracle (oracle/Makefile)."""
    _run(["make", "-s", "-C", str(ROOT / "oracle")])
    return ROOT / "oracle" / "_build" / "liboracle.so"


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "variant":
        print(build_variant(sys.argv[2], sys.argv[3:]))
        sys.exit(0)
    print(build_lib(verbose=True))
    print(build_plugin(verbose=True))
    print(build_oracle())
