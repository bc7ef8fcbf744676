"""Native build for the framework: explicit ``hipcc --offload-arch=gfx950`` / ``g++`` commands.

No hipify, no ``torch.utils.cpp_extension`` JIT cache: every object is built in-tree under
``build/`` and linked into ``pytorch_distributed_example_amd/_lib/*.so`` so that the shared
objects travel with the repo snapshot to the GPU box (see ``_ext.py`` for loading).

Two extension modules are produced:

* ``_runtime``  - C++ distributed runtime (TCP rendezvous store, host TCP collectives, RCCL
                  communicator, xGMI peer all-reduce kernel ``runtime/peer_allreduce.hip``).
                  pybind11 only, no torch headers, links torch's bundled
                  ``librccl.so.1`` / ``libamdhip64.so.7`` (same sonames as /opt/rocm).
* ``_kernels``  - CDNA4 HIP kernels (``csrc/kernels/*.hip``, device code, no torch headers)
                  plus a thin torch C++ binding layer (``csrc/ops_bindings.cpp``).

Usage: ``python -m pytorch_distributed_example_amd.utils.build [-j N] [--force]``.
"""
from __future__ import annotations

import argparse
import glob
import hashlib
import json
import os
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = os.path.join(REPO, "pytorch_distributed_example_amd")
LIBDIR = os.path.join(PKG, "_lib")
BUILDDIR = os.path.join(REPO, "build")
CSRC = os.path.join(REPO, "csrc")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = "gfx950"
EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _torch_paths():
    import torch  # noqa: F401  (only for include / lib paths)
    tdir = os.path.dirname(torch.__file__)
    inc = [os.path.join(tdir, "include"), os.path.join(tdir, "include", "torch", "csrc", "api", "include")]
    return tdir, inc, os.path.join(tdir, "lib"), int(torch._C._GLIBCXX_USE_CXX11_ABI)


def _pybind_inc():
    import pybind11
    return pybind11.get_include()


def _py_inc():
    return sysconfig.get_paths()["include"]


def _hash_file(path, extra=""):
    h = hashlib.sha1(extra.encode())
    with open(path, "rb") as f:
        h.update(f.read())
    # crude header dependency: every header under csrc/include and the source's own dir
    for hdr in sorted(glob.glob(os.path.join(CSRC, "include", "*.h")) +
                      glob.glob(os.path.join(os.path.dirname(path), "*.h"))):
        with open(hdr, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


# Per-source extra flags.  attention.hip: no SLP vectorization -- the softmax / dS math sits between
# MFMAs, where packed f32 ops (v_pk_mul/add/fma_f32, 206 of them from SLP packing adjacent scalar ops)
# cost more issue time than the two scalar ops they replace (MI355X_MICROARCH.md: an anti-lever beside
# MFMAs; profiles/r5_gpt2/attention_no_slp/); lenet_v2.hip: the same, -45 VALU in the conv backward
# loop (profiles/r5_lenet/lenet_no_slp/)
_FILE_FLAGS = {"attention.hip": ["-fno-slp-vectorize"], "lenet_v2.hip": ["-fno-slp-vectorize"]}


def _targets():
    tdir, tinc, tlib, abi = _torch_paths()
    common_inc = ["-I" + os.path.join(CSRC, "include"), "-I" + _pybind_inc(), "-I" + _py_inc()]
    hip_dev = ["hipcc", "-c", "-x", "hip", f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17",
               "-munsafe-fp-atomics", "-Wno-unused-result"] + common_inc
    host_cpp = ["g++", "-c", "-O2", "-fPIC", "-std=c++17", "-Wall", "-Wno-unused-function",
                f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-D__HIP_PLATFORM_AMD__=1",
                "-I" + os.path.join(ROCM, "include")] + common_inc
    torch_cpp = host_cpp + ["-DUSE_ROCM=1", "-DTORCH_EXTENSION_NAME=_kernels",
                            "-DTORCH_API_INCLUDE_EXTENSION_H"] + ["-I" + p for p in tinc]
    rpath = ["-Wl,-rpath," + tlib, "-Wl,-rpath," + os.path.join(ROCM, "lib")]
    return {
        "_runtime": dict(
            sources=[(s, host_cpp) for s in sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))]
            + [(s, hip_dev) for s in sorted(glob.glob(os.path.join(CSRC, "runtime", "*.hip")))],
            link=["hipcc", "-shared", "-fPIC", f"--offload-arch={ARCH}", "-L" + tlib, "-l:librccl.so",
                  "-l:libamdhip64.so", "-lpthread"] + rpath,
        ),
        "_kernels": dict(
            sources=[(s, hip_dev + _FILE_FLAGS.get(os.path.basename(s), []))
                     for s in sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))]
            + [(os.path.join(CSRC, "ops_bindings.cpp"), torch_cpp)]
            + [(s, torch_cpp) for s in sorted(glob.glob(os.path.join(CSRC, "bind_*.cpp")))],
            link=["hipcc", "-shared", "-fPIC", f"--offload-arch={ARCH}", "-L" + tlib,
                  "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python",
                  "-l:libamdhip64.so"] + rpath,
        ),
    }


def _compile(src, cmd, force, verbose):
    rel = os.path.relpath(src, CSRC).replace(os.sep, "__")
    key = _hash_file(src, " ".join(cmd))
    obj = os.path.join(BUILDDIR, f"{rel}.{key}.o")
    if os.path.exists(obj) and not force:
        return obj, False
    full = cmd + [src, "-o", obj + ".tmp"]
    if verbose:
        print(" ".join(full), flush=True)
    r = subprocess.run(full, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{' '.join(full)}\n{r.stdout}\n{r.stderr}")
    os.replace(obj + ".tmp", obj)
    return obj, True


def build(targets=None, jobs=None, force=False, verbose=False):
    """Compile and link the requested extension modules. Returns {name: so_path}."""
    os.makedirs(BUILDDIR, exist_ok=True)
    os.makedirs(LIBDIR, exist_ok=True)
    allt = _targets()
    names = list(targets or allt.keys())
    jobs = jobs or min(8, os.cpu_count() or 4)
    out = {}
    for name in names:
        t = allt[name]
        with ThreadPoolExecutor(jobs) as ex:
            res = list(ex.map(lambda sc: _compile(sc[0], sc[1], force, verbose), t["sources"]))
        objs = [o for o, _ in res]
        so = os.path.join(LIBDIR, name + EXT_SUFFIX)
        stamp = so + ".objs.json"
        prev = None
        if os.path.exists(stamp):
            with open(stamp) as f:
                prev = json.load(f)
        if force or prev != objs or not os.path.exists(so):
            cmd = t["link"][:1] + objs + ["-o", so + ".tmp"] + t["link"][1:]
            if verbose:
                print(" ".join(cmd), flush=True)
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"link failed: {name}\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
            os.replace(so + ".tmp", so)
            with open(stamp, "w") as f:
                json.dump(objs, f)
        out[name] = so
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("targets", nargs="*")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args(argv)
    res = build(a.targets or None, a.jobs, a.force, a.verbose)
    for k, v in res.items():
        print(f"{k}: {v}")


if __name__ == "__main__":
    sys.exit(main())
