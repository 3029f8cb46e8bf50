"""Build the native libraries in-tree (reference analogue: src/main/cpp/CMakeLists.txt
for libsystemml_*.so and the nvcc build of kernels/SystemML.cu).

  ops/hip/*.hip      -> ops/lib/libsysml_hip.so     (hipcc --offload-arch=gfx950)
  ops/csrc/*.cpp     -> ops/lib/libsysml_native.so  (g++ -O3 -fopenmp, host-side IO)

Usage: python -m systemml_amd.ops.build [--force]
"""
from __future__ import annotations

import glob
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "lib")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0]


def _hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def _stale(out, srcs):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(s) > t for s in srcs)


def build_hip(force=False, verbose=True):
    os.makedirs(LIB, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(HERE, "hip", "*.hip")))
    out = os.path.join(LIB, "libsysml_hip.so")
    if not force and not _stale(out, srcs + glob.glob(os.path.join(HERE, "hip", "*.h"))):
        return out
    objs, cmds = [], []
    hdrs = glob.glob(os.path.join(HERE, "hip", "*.h"))
    for s in srcs:
        o = os.path.join(LIB, os.path.basename(s) + ".o")
        if force or _stale(o, [s] + hdrs):   # objects are kept: only edited units recompile
            cmds.append([_hipcc(), f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-c", s, "-o", o])
        objs.append(o)
    # one hipcc per translation unit, in parallel (rowstream.hip alone is ~2 min)
    procs = []
    for cmd in cmds:
        if verbose:
            print(" ".join(cmd), flush=True)
        procs.append(subprocess.Popen(cmd))
    bad = [c for c, p in zip(cmds, procs) if p.wait() != 0]
    if bad:
        raise subprocess.CalledProcessError(1, bad[0])
    # librtc: the run-time compiler of the generated fused kernels (ops/hip/rtc.hip)
    cmd = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out] + objs + ["-lhiprtc"]
    subprocess.check_call(cmd)
    return out


def build_native(force=False, verbose=True):
    os.makedirs(LIB, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(HERE, "csrc", "*.cpp")))
    if not srcs:
        return None
    out = os.path.join(LIB, "libsysml_native.so")
    if not force and not _stale(out, srcs):
        return out
    cmd = ["g++", "-O3", "-march=x86-64-v2", "-fPIC", "-shared", "-std=c++17", "-fopenmp", "-o", out] + srcs
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    return out


def build_all(force=False, verbose=True):
    return build_hip(force, verbose), build_native(force, verbose)


if __name__ == "__main__":
    print(build_all(force="--force" in sys.argv))
