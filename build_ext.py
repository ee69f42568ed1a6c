#!/usr/bin/env python
"""Build the gfx950 extension in-tree: ``mingpt_distributed_amd/_C.so``.

Explicit ``hipcc --offload-arch=gfx950`` compiles (no hipify pass, no JIT cache):

* each ``csrc/kernels/*.hip`` -> object with device code for gfx950 only,
* ``csrc/comm/*.cpp``         -> the native RCCL communicator (no link-time RCCL: it binds the
  RCCL torch already loaded, see csrc/comm/rccl_comm.cpp),
* ``csrc/bindings.cpp``       -> host object against the torch headers,
* link against the HIP runtime *bundled with torch* (``torch/lib/libamdhip64.so``), so the
  process holds exactly one HIP runtime and our kernels share torch's streams and allocator.

Incremental: an object is rebuilt only when its source or any header is newer.
Usage: ``python build_ext.py [--force] [-j N] [--tools]``
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "mingpt_distributed_amd")
BUILD = os.path.join(ROOT, "build", "obj")
ARCH = os.environ.get("MINGPT_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

COMMON_FLAGS = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-Wno-unused-result",
                "-I" + os.path.join(ROOT, "csrc", "include"), "-ffp-contract=fast"]
# per-source extras.  attention_train.hip: no SLP vectoriser -- it packs the softmax-gradient
# multiplies into v_pk_mul/fma_f32 pairs with s_nop between them, an anti-lever beside MFMAs
# (MI355X_MICROARCH 'price of one filler'), and the hd = 64 backward's register budget is tight
FILE_FLAGS = {"attention_train.hip": ["-fno-slp-vectorize"]}



def _torch_paths():
    import torch
    from torch.utils.cpp_extension import include_paths

    tdir = os.path.dirname(torch.__file__)
    return include_paths(), os.path.join(tdir, "lib"), int(torch._C._GLIBCXX_USE_CXX11_ABI)


def _newer(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(" ".join(cmd) + "\n" + r.stdout + r.stderr)
        raise RuntimeError(f"compile failed: {cmd[-1]}")
    return r


DEBUG_SO = os.path.join(ROOT, "build", "debug", "_C.so")


def build(force: bool = False, jobs: int = 8, verbose: bool = True, debug: bool = False) -> str:
    """Release: ``mingpt_distributed_amd/_C.so``.  ``debug=True``: the same sources with
    ``-DMG_DEBUG`` (device-side range checks on token ids / targets, common.h MG_CHECK_INDEX) into
    ``build/debug/_C.so``; load it with ``MINGPT_EXT_SO=build/debug/_C.so MINGPT_DEBUG_CHECKS=1``."""
    flags = COMMON_FLAGS + (["-DMG_DEBUG"] if debug else [])
    flags += os.environ.get("MG_EXTRA_FLAGS", "").split()  # kernel variant switches (A/B builds)
    bdir = BUILD + "_debug" if debug else BUILD
    os.makedirs(bdir, exist_ok=True)
    # the objects' compile flags (MG_EXTRA_FLAGS variant switches included): a change rebuilds
    # every object, so a variant build never leaves objects a later plain build would link
    stamp = os.path.join(bdir, "flags.stamp")
    key = " ".join(flags) + " " + repr(sorted(FILE_FLAGS.items()))
    old = open(stamp).read() if os.path.exists(stamp) else None
    if old != key:
        force = True
    headers = glob.glob(os.path.join(ROOT, "csrc", "include", "*.h"))
    kernels = sorted(glob.glob(os.path.join(ROOT, "csrc", "kernels", "*.hip")))
    kernels += sorted(glob.glob(os.path.join(ROOT, "csrc", "comm", "*.cpp")))  # host code (HIP runtime + RCCL)
    incs, tlib, abi = _torch_paths()
    py_inc = sysconfig.get_paths()["include"]

    jobs_list = []
    objs = []
    for src in kernels:
        obj = os.path.join(bdir, os.path.basename(src) + ".o")
        objs.append(obj)
        if force or _newer(obj, [src] + headers):
            jobs_list.append([HIPCC, *flags, *FILE_FLAGS.get(os.path.basename(src), []), "-x", "hip", "-c",
                              "-o", obj, src])
    bsrc = os.path.join(ROOT, "csrc", "bindings.cpp")
    bobj = os.path.join(bdir, "bindings.o")
    objs.append(bobj)
    if force or _newer(bobj, [bsrc] + headers):
        jobs_list.append([HIPCC, *flags, "-x", "hip", "-c", "-o", bobj,
                          *["-I" + p for p in incs], "-I" + py_inc,
                          f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DTORCH_EXTENSION_NAME=_C",
                          "-DTORCH_API_INCLUDE_EXTENSION_H", "-D__HIP_PLATFORM_AMD__=1",
                          "-DUSE_ROCM=1", bsrc])
    if jobs_list:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            futs = {ex.submit(_run, c): c[-1] for c in jobs_list}
            for f in cf.as_completed(futs):
                f.result()
                if verbose:
                    print(f"[build_ext] compiled {os.path.relpath(futs[f], ROOT)}", flush=True)
    if old != key:
        with open(stamp, "w") as f:
            f.write(key)
    out = DEBUG_SO if debug else os.path.join(PKG, "_C.so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    if force or _newer(out, objs):
        _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", out, *objs,
              "-L" + tlib, "-Wl,-rpath," + tlib, "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu",
              "-ltorch_hip", "-ltorch_python", "-lamdhip64"])
        bad = anon_undefined(out)
        if bad:
            os.remove(out)
            raise RuntimeError(f"link produced unresolvable internal symbols (e.g. a kernel whose host "
                               f"launch stub was not emitted): {bad[:5]}")
        if verbose:
            print(f"[build_ext] linked {os.path.relpath(out, ROOT)}", flush=True)
    return out


def anon_undefined(so: str):
    """Undefined symbols of ``so`` in an anonymous namespace (``_GLOBAL__N_``): nothing outside the
    library can define them, so each one is a build bug that would only surface as an ImportError
    on the GPU box (seen: a target builtin in a ``__global__`` template body made hipcc drop the
    host launch stub of that instantiation).  Empty when ``nm`` is not available."""
    try:
        r = subprocess.run(["nm", "-D", "--undefined-only", so], capture_output=True, text=True)
    except OSError:
        return []
    return [ln.split()[-1] for ln in r.stdout.splitlines() if "_GLOBAL__N_" in ln]


def _torch_runtime_dir() -> str:
    """build/torchlibs: links, under their sonames, to the HIP runtime and RCCL that torch ships
    (torch/lib holds them as libamdhip64.so / librccl.so, so a NEEDED libamdhip64.so.7 /
    librccl.so.1 would otherwise resolve to /opt/rocm's).  Native tools link and run against
    these: the RCCL they time is the one training loads (2.26.6 here, not /opt/rocm's 2.27.7),
    and one HIP runtime per process."""
    _, tlib, _ = _torch_paths()
    d = os.path.join(ROOT, "build", "torchlibs")
    os.makedirs(d, exist_ok=True)
    # torch's RCCL asks for the unversioned names of its own dependencies; point those at torch's
    # files too, so the process maps each runtime library once
    names = [("libamdhip64.so", "libamdhip64.so.7"), ("libamdhip64.so", "libamdhip64.so"),
             ("librccl.so", "librccl.so.1")]
    names += [(n, n) for n in ("libhsa-runtime64.so", "libroctx64.so", "librocm_smi64.so",
                               "librocprofiler-register.so") if os.path.exists(os.path.join(tlib, n))]
    for name, soname in names:
        link = os.path.join(d, soname)
        target = os.path.join(tlib, name)
        if os.path.lexists(link) and os.readlink(link) != target:
            os.remove(link)
        if not os.path.lexists(link):
            os.symlink(target, link)
    return d


def build_tools(verbose: bool = True):
    """Native tools (standalone executables: HIP + the RCCL bundled with torch, see
    _torch_runtime_dir)."""
    outdir = os.path.join(ROOT, "build", "bin")
    os.makedirs(outdir, exist_ok=True)
    tdir = _torch_runtime_dir()
    built = []
    for src in sorted(glob.glob(os.path.join(ROOT, "tools", "*.cpp"))):
        exe = os.path.join(outdir, os.path.splitext(os.path.basename(src))[0])
        if _newer(exe, [src, os.path.abspath(__file__)]):
            _run([HIPCC, "-O2", "-std=c++17", f"--offload-arch={ARCH}", "-x", "hip", "-o", exe, src,
                  "-I/opt/rocm/include", "-L" + tdir, "-l:librccl.so.1", "-l:libamdhip64.so.7",
                  "-Wl,--disable-new-dtags", "-Wl,-rpath," + tdir])
            if verbose:
                print(f"[build_ext] built {os.path.relpath(exe, ROOT)}", flush=True)
        built.append(exe)
    return built


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=min(8, os.cpu_count() or 8))
    ap.add_argument("--tools", action="store_true", help="also build tools/*.cpp executables")
    ap.add_argument("--debug", action="store_true", help="also build the MG_DEBUG variant")
    a = ap.parse_args()
    build(force=a.force, jobs=a.jobs)
    if a.debug:
        build(force=a.force, jobs=a.jobs, debug=True)
    if a.tools:
        build_tools()
