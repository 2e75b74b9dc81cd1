"""Build the in-tree HIP extension (gfx950) and the C-ABI shared library."""
from __future__ import annotations

import os
import subprocess

from ._lib import PKG_DIR, REPO_DIR, LIB_PATH

SOURCES = ["csrc/gm_capi.hip", "csrc/gm_calib.hip", "csrc/gm_host_model.cpp", "csrc/gm_mjcf.cpp"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
         "-fhip-fp32-correctly-rounded-divide-sqrt", "-munsafe-fp-atomics",
         "-ffp-contract=off",
         # MachineLICM off: in the outlined substep loop (gm_kernels.hip substep_loop) it
         # hoists constant materialisations out of the loop and the body then spills
         "-mllvm", "-disable-machine-licm"]


def build(verbose: bool = False, force: bool = False, out: str | None = None, extra_flags=()) -> str:
    """Compile each translation unit in parallel (the env-step kernel and the calibration
    variant are separate device modules), then link libgm.so (or `out`: developer A/B
    builds, with `extra_flags` added to every compile)."""
    lib_path = out or LIB_PATH
    srcs = [os.path.join(PKG_DIR, s) for s in SOURCES]
    deps = srcs + [os.path.join(PKG_DIR, "csrc", f) for f in ("gm_kernels.hip", "gm_newton.hip", "gm_math.h", "gm_fphelpers.inc", "gm_policy.hip", "gm_state.h")] + \
        [os.path.join(REPO_DIR, "include", f) for f in ("gripper_mi355x.h", "gm_settings.def")]
    if not force and out is None and os.path.exists(LIB_PATH):
        t = os.path.getmtime(LIB_PATH)
        if all(os.path.getmtime(d) <= t for d in deps):
            return LIB_PATH
    objdir = os.path.join(os.path.dirname(LIB_PATH), "obj" if out is None else "obj_" + os.path.basename(out))
    os.makedirs(objdir, exist_ok=True)
    inc = ["-I" + os.path.join(REPO_DIR, "include"), "-I" + os.path.join(PKG_DIR, "csrc")]
    procs, objs = [], []
    headers = [os.path.join(PKG_DIR, "csrc", "gm_state.h")] + \
        [os.path.join(REPO_DIR, "include", f) for f in ("gripper_mi355x.h", "gm_settings.def")]
    for src in srcs:
        obj = os.path.join(objdir, os.path.basename(src) + ".o")
        objs.append(obj)
        # host-only translation units (.cpp) depend on their source and the shared headers;
        # the device ones on every kernel source
        tu_deps = [src] + headers if src.endswith(".cpp") else deps
        if not force and os.path.exists(obj) and all(os.path.getmtime(d) <= os.path.getmtime(obj) for d in tu_deps):
            continue
        cmd = [HIPCC, *FLAGS, *extra_flags, *inc, "-c", src, "-o", obj]
        if verbose:
            print(" ".join(cmd))
        procs.append((subprocess.Popen(cmd), cmd))
    for p, cmd in procs:
        if p.wait() != 0:
            raise subprocess.CalledProcessError(p.returncode, cmd)
    link = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", *objs, "-o", lib_path + ".tmp"]
    if verbose:
        print(" ".join(link))
    subprocess.run(link, check=True)
    os.replace(lib_path + ".tmp", lib_path)
    return lib_path
