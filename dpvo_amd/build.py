"""In-tree build of the MI355X (gfx950) native code.

    python -m dpvo_amd.build            # build everything (incremental)
    python -m dpvo_amd.build --force    # rebuild

Products (dpvo_amd/_native/, git-ignored, shipped to the GPU box by gpurun):
  libdpvo_hot.so                      HIP kernels + the C ABI of include/dpvo_hot.h
  cuda_corr.<ext>, cuda_ba.<ext>,     pybind11 extension modules with the
  lietorch_backends.<ext>             reference's module / function names,
                                      thin wrappers over libdpvo_hot.so

hipcc compiles the kernels directly for gfx950; the extension modules are
host-only C++ compiled with g++ against the PyTorch-ROCm headers (no hipify,
no JIT cache outside the tree).
"""
from __future__ import annotations

import argparse
import os
import shlex
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "_native")
INCLUDE = os.path.join(REPO, "include")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("DPVO_OFFLOAD_ARCH", "gfx950")

HIP_SOURCES = ["corr.hip", "corr_nhwc.hip", "corr_nchw.hip", "ba.hip", "ba_window.hip", "ba_large.hip", "lie.hip", "pgo.hip", "pg.hip",
               "keyframe.hip", "spd_solve.hip"]
EXTENSIONS = {
    "cuda_corr": "ext_cuda_corr.cpp",
    "cuda_ba": "ext_cuda_ba.cpp",
    "lietorch_backends": "ext_lietorch.cpp",
}
HEADERS = ["common.hpp", "ext_common.hpp", "ba_device.hpp", "ba_solve.hpp", "pyr_insert.hpp", "ba_bgj.hpp"]
# per-source device flags.  The BA window kernel is a chain of short dependent
# steps run by few waves: clang's SLP vectoriser packs its scalar fp32 math into
# v_pk_fma_f32 and pays for it with register-pair v_mov shuffles (3x the
# instructions of the 6x6 pivot factorisation), so it is off there.
SOURCE_FLAGS = {"ba_window.hip": ["-fno-slp-vectorize"]}


def _git_rev():
    try:
        return subprocess.check_output(["git", "-C", REPO, "rev-parse", "--short", "HEAD"],
                                       stderr=subprocess.DEVNULL).decode().strip()
    except Exception:
        return "nogit"


def _run(cmd, verbose):
    if verbose:
        print("+", " ".join(shlex.quote(c) for c in cmd), flush=True)
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    if r.returncode != 0:
        sys.stderr.write(r.stdout.decode(errors="replace"))
        raise RuntimeError(f"build step failed: {cmd[0]} -> {cmd[-1]}")


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def lib_path():
    return os.path.join(OUT, "libdpvo_hot.so")


def ext_suffix():
    return sysconfig.get_config_var("EXT_SUFFIX")


def build(force=False, verbose=False):
    os.makedirs(OUT, exist_ok=True)
    hipcc = os.path.join(ROCM, "bin", "hipcc")
    hdr = [os.path.join(INCLUDE, "dpvo_hot.h")] + [os.path.join(CSRC, h) for h in HEADERS]
    lib = lib_path()
    srcs = [os.path.join(CSRC, s) for s in HIP_SOURCES]
    # one object per HIP source (incremental), then one shared library
    objdir = os.path.join(OUT, "obj")
    os.makedirs(objdir, exist_ok=True)
    objs, cmds = [], []
    for src in srcs:
        obj = os.path.join(objdir, os.path.basename(src).replace(".hip", ".o"))
        objs.append(obj)
        if force or _stale(obj, [src] + hdr + [__file__]):
            cmds.append([hipcc, "-O3", "-std=c++17", f"--offload-arch={ARCH}", "-fPIC", "-c",
                         "-fvisibility=hidden", "-mcode-object-version=5", "-Wno-unused-result",
                         f"-I{INCLUDE}", f'-DDPVO_GIT_REV="{_git_rev()}"',
                         *SOURCE_FLAGS.get(os.path.basename(src), []), src, "-o", obj])
    # the objects are independent: compile them concurrently (bounded by the
    # host's share of CPUs; MAX_JOBS is honoured as on the GPU box)
    jobs = max(1, min(len(cmds), int(os.environ.get("MAX_JOBS", os.cpu_count() or 1)), 16))
    if cmds:
        from concurrent.futures import ThreadPoolExecutor

        with ThreadPoolExecutor(jobs) as ex:
            list(ex.map(lambda c: _run(c, verbose), cmds))
    if force or _stale(lib, objs):
        cmd = [hipcc, f"--offload-arch={ARCH}", "-fPIC", "-shared", *objs, "-o", lib]
        _run(cmd, verbose)

    import torch
    from torch.utils import cpp_extension as ce

    tinc = ce.include_paths()
    tlib = ce.library_paths()[0]
    abi = []
    for getter in ("_get_pybind11_abi_build_flags", "_get_glibcxx_abi_build_flags"):
        fn = getattr(ce, getter, None)
        if fn is not None:
            abi += list(fn())
    pyinc = sysconfig.get_paths()["include"]
    for name, src in EXTENSIONS.items():
        target = os.path.join(OUT, name + ext_suffix())
        srcp = os.path.join(CSRC, src)
        if not (force or _stale(target, [srcp, lib] + hdr + [__file__])):
            continue
        cmd = ["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-fvisibility=hidden",
               "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", "-DTORCH_API_INCLUDE_EXTENSION_H",
               f"-DTORCH_EXTENSION_NAME={name}", *abi, f"-I{INCLUDE}", f"-I{CSRC}",
               *[f"-I{p}" for p in tinc], f"-I{ROCM}/include", f"-I{pyinc}", srcp, "-o", target,
               f"-L{OUT}", "-ldpvo_hot", f"-L{tlib}", "-lc10", "-lc10_hip", "-ltorch",
               "-ltorch_cpu", "-ltorch_hip", "-ltorch_python",
               "-Wl,-rpath,$ORIGIN", f"-Wl,-rpath,{tlib}"]
        _run(cmd, verbose)
    del torch
    return OUT


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args()
    out = build(force=a.force, verbose=a.verbose)
    print("built", out)


if __name__ == "__main__":
    main()
