"""Build the native libraries in-tree (no JIT cache, so the .so files travel with the repo).

* ``_lib/libmxr_kernels.so`` -- every HIP kernel in ``csrc/kernels/*.hip`` compiled with
  ``hipcc --offload-arch=gfx950 -O3`` (cross-compiles without a GPU);
* ``_lib/libmxr_comm.so``    -- the native communication core (``csrc/comm/*.hip``: RCCL
  communicator, in-order gradient-bucket engine on a dedicated HIP stream, timeline writer);
* ``_lib/libmxr_cpu.so``     -- host C++ runtime pieces (IoU / anchor targets oracle, NMS,
  image resize / affine warp, COCO-eval IoU, CRC32C) compiled with g++ -O3.

Objects are cached by a hash of (source, headers, flags); ``python -m
batchai_retinanet_horovod_coco_amd.build`` rebuilds what changed.
"""
from __future__ import annotations

import glob
import hashlib
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(ROOT, "csrc")
LIBDIR = os.path.join(PKG, "_lib")
OBJDIR = os.path.join(ROOT, "build", "obj")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0]

HIPCC = os.path.join(ROCM, "bin", "hipcc")
HIP_FLAGS = ["-O3", "-fPIC", "-std=c++17", "--offload-arch=" + ARCH, "-Wno-unused-result", "-Wno-unused-value"]
CXX = os.environ.get("CXX", "g++")
CXX_FLAGS = ["-O3", "-fPIC", "-std=c++17", "-march=x86-64-v2", "-fopenmp"]


def _hash(paths, flags) -> str:
    h = hashlib.sha1()
    for p in sorted(paths):
        with open(p, "rb") as f:
            h.update(f.read())
    h.update(" ".join(flags).encode())
    return h.hexdigest()[:16]


def _compile(cmd, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("compile failed:\n{}\n{}".format(" ".join(cmd), r.stdout))
    return r.stdout


def _build_lib(name, sources, headers, compiler, flags, link_flags, verbose, jobs):
    os.makedirs(OBJDIR, exist_ok=True)
    os.makedirs(LIBDIR, exist_ok=True)
    objs, todo = [], []
    for src in sources:
        key = _hash([src] + headers, flags + [compiler])
        obj = os.path.join(OBJDIR, "{}.{}.o".format(os.path.basename(src), key))
        objs.append(obj)
        if not os.path.exists(obj):
            todo.append([compiler] + flags + ["-c", src, "-o", obj])
    if todo:
        with ThreadPoolExecutor(max_workers=max(1, min(jobs, len(todo)))) as ex:
            list(ex.map(lambda c: _compile(c, verbose), todo))
    out = os.path.join(LIBDIR, name)
    os.makedirs(os.path.dirname(out), exist_ok=True)
    key = _hash(objs, link_flags)
    stamp = out + ".stamp"
    if os.path.exists(out) and os.path.exists(stamp) and open(stamp).read() == key:
        return out
    tmp = out + ".tmp"
    _compile([compiler] + flags + ["-shared", "-o", tmp] + objs + link_flags, verbose)
    os.replace(tmp, out)
    with open(stamp, "w") as f:
        f.write(key)
    return out


def build_kernels(verbose=False, jobs=8) -> str:
    srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    hdrs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.h")))
    return _build_lib("libmxr_kernels.so", srcs, hdrs, HIPCC, HIP_FLAGS, [], verbose, jobs)


def build_kernels_diag(verbose=False, jobs=8) -> str:
    """Timing-only (DIAG) kernel instantiations -- wrong results by design -- go into a SEPARATE library,
    _lib/diag/libmxr_kernels.so (load it with MXR_KERNEL_LIB=<path>); the production library never holds them."""
    srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    hdrs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.h")))
    return _build_lib(os.path.join("diag", "libmxr_kernels.so"), srcs, hdrs, HIPCC, HIP_FLAGS + ["-DMXR_DIAG_KERNELS=1"],
                      [], verbose, jobs)


def build_comm(verbose=False, jobs=8) -> str:
    srcs = sorted(glob.glob(os.path.join(CSRC, "comm", "*.hip")))
    if not srcs:
        return ""
    return _build_lib("libmxr_comm.so", srcs, [], HIPCC, HIP_FLAGS, ["-ldl"], verbose, jobs)


# AddressSanitizer + UndefinedBehaviorSanitizer build of the host runtime: built next to the
# production library as _lib/asan/libmxr_cpu.so; load it with MXR_CPU_LIB=<path> and the sanitizer runtimes
# preloaded (scripts/run_sanitized_cpu_tests.sh).  The HIP libraries are never sanitized (no GPU ASan here).
SAN_FLAGS = ["-O1", "-g", "-fPIC", "-std=c++17", "-fopenmp", "-fno-omit-frame-pointer",
             "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"]


def build_cpu(verbose=False, jobs=8, sanitize=False) -> str:
    srcs = sorted(glob.glob(os.path.join(CSRC, "cpu", "*.cpp")))
    if not srcs:
        return ""
    hdrs = sorted(glob.glob(os.path.join(CSRC, "cpu", "*.h")))
    if sanitize:
        return _build_lib(os.path.join("asan", "libmxr_cpu.so"), srcs, hdrs, CXX, SAN_FLAGS,
                          ["-fopenmp", "-fsanitize=address,undefined"], verbose, jobs)
    return _build_lib("libmxr_cpu.so", srcs, hdrs, CXX, CXX_FLAGS, ["-fopenmp"], verbose, jobs)


def build_all(verbose=False, jobs=None):
    jobs = jobs or min(8, os.cpu_count() or 4)
    out = []
    out.append(build_cpu(verbose, jobs))
    if os.environ.get("MXR_SANITIZE", "0") == "1":
        out.append(build_cpu(verbose, jobs, sanitize=True))
    if os.path.exists(HIPCC):
        out.append(build_kernels(verbose, jobs))
        out.append(build_comm(verbose, jobs))
        if os.environ.get("MXR_BUILD_DIAG", "0") == "1":
            out.append(build_kernels_diag(verbose, jobs))
    elif verbose:
        print("hipcc not found; HIP kernels not built", file=sys.stderr)
    return [o for o in out if o]


if __name__ == "__main__":
    if "--sanitize" in sys.argv:
        os.environ["MXR_SANITIZE"] = "1"
    if "--diag" in sys.argv:
        os.environ["MXR_BUILD_DIAG"] = "1"
    for p in build_all(verbose="-v" in sys.argv):
        print(p)
