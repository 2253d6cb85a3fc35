"""In-tree build of the native extension ``pytorch_distributed_mnist_amd/_C*.so``.

    python -m pytorch_distributed_mnist_amd.build [--force] [-j N] [--verbose]

Every ``csrc/**/*.hip`` / ``csrc/**/*.cpp`` file is compiled by ``hipcc`` for
``--offload-arch=gfx950`` only (CDNA4; no other targets, no hipify, no CUDA),
objects are cached under ``build/obj`` keyed by a hash of source + headers +
flags, and the objects are linked into one shared library against torch's own
HIP runtime and RCCL (``torch/lib``), so the extension shares the process's
single copy of libamdhip64/librccl (SURVEY.md §7.5 risk 2).  hipcc
cross-compiles without a GPU, so this runs on the CPU-only dev box.
"""
from __future__ import annotations

import argparse
import glob
import hashlib
import re
import os
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor
from . import knobs

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "pytorch_distributed_mnist_amd")
CSRC = os.path.join(REPO, "csrc")
OBJ_DIR = os.path.join(REPO, "build", "obj")
ARCH = "gfx950"


def _torch_paths():
    import torch
    from torch.utils import cpp_extension as ce
    inc = [os.path.join(os.path.dirname(torch.__file__), "include"),
           os.path.join(os.path.dirname(torch.__file__), "include", "torch", "csrc", "api", "include")]
    lib = os.path.join(os.path.dirname(torch.__file__), "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi, ce


def hipcc() -> str:
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    p = os.path.join(rocm, "bin", "hipcc")
    return p if os.path.exists(p) else "hipcc"


def sources():
    out = sorted(glob.glob(os.path.join(CSRC, "**", "*.hip"), recursive=True))
    out += sorted(glob.glob(os.path.join(CSRC, "**", "*.cpp"), recursive=True))
    return out


def headers():
    return sorted(glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True))


def compile_flags(abi: int, inc):
    flags = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}",
             "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
             "-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H",
             f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
             "-Wno-unused-result", "-Wno-deprecated-declarations",
             "-Werror=misleading-indentation",
             f"-I{CSRC}", f"-I{sysconfig.get_paths()['include']}"]
    flags += [f"-I{p}" for p in inc]
    if knobs.get("PDM_DEBUG_BOUNDS"):
        flags.append("-DPDM_DEBUG_BOUNDS=1")
    if knobs.get("PDM_STAMPS"):
        flags.append("-DPDM_STAMPS=1")
    if knobs.get("PDM_HIPCC_FLAGS"):                  # compiler experiments (diagnostic builds)
        flags += os.environ["PDM_HIPCC_FLAGS"].split()
    return flags


# Per-file compiler flags.  fc1_fwd / fc1_bwd are translation units of their own (wrappers
# that include cnn_fwd.hip / cnn_bwd.hip with a section switch) so that they can use the
# max-ilp machine scheduler, which measured faster for them and slower for cnn_fwd /
# cnn_bwd (docs/kernels.md, tools/gpu_ab.sh).
FILE_FLAGS = {
    "kernels/fc1_fwd.hip": ["-mllvm", "-amdgpu-sched-strategy=max-ilp"],
    "kernels/fc1_bwd.hip": ["-mllvm", "-amdgpu-sched-strategy=max-ilp"],
    "kernels/cnn_head.hip": ["-mllvm", "-amdgpu-sched-strategy=iterative-ilp"],
}


def file_flags():
    """FILE_FLAGS, overridden per file by $PDM_FILE_FLAGS ("rel/path.hip=flags;..."; diagnostic
    builds)."""
    ff = dict(FILE_FLAGS)
    for item in filter(None, knobs.get("PDM_FILE_FLAGS", "").split(";")):
        path, _, fl = item.partition("=")
        ff[path.strip()] = fl.split()
    return ff


def _included_sources(path):
    """.hip files a wrapper source #includes (their text is part of its object's hash)."""
    out = []
    with open(path) as f:
        for line in f:
            m = re.match(r'\s*#include\s+"([^"]+\.hip)"', line)
            if m:
                out.append(os.path.join(os.path.dirname(path), m.group(1)))
    return out


def _hash(path, flags, hdr_digest):
    h = hashlib.sha256()
    for p in [path] + _included_sources(path):
        with open(p, "rb") as f:
            h.update(f.read())
    h.update(" ".join(flags).encode())
    h.update(hdr_digest)
    return h.hexdigest()[:20]


def build(force: bool = False, jobs: int | None = None, verbose: bool = False,
          out: str | None = None) -> str:
    inc, lib, abi, _ = _torch_paths()
    custom_out = out is not None
    flags = compile_flags(abi, inc)
    os.makedirs(OBJ_DIR, exist_ok=True)
    hd = hashlib.sha256()
    for hpath in headers():
        with open(hpath, "rb") as f:
            hd.update(f.read())
    hdr_digest = hd.digest()
    srcs = sources()
    if not srcs:
        raise RuntimeError("no sources under csrc/")

    def one(src):
        relp = os.path.relpath(src, CSRC).replace(os.sep, "/")
        fflags = flags + file_flags().get(relp, [])
        rel = relp.replace("/", "_")
        obj = os.path.join(OBJ_DIR, f"{rel}.{_hash(src, fflags, hdr_digest)}.o")
        if os.path.exists(obj) and not force:
            return obj, None
        cmd = [hipcc()] + fflags + ["-c", src, "-o", obj + ".tmp"]
        if src.endswith(".hip"):
            cmd[1:1] = ["-x", "hip"]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            return None, f"compile failed: {src}\n{r.stdout}\n{r.stderr}"
        os.replace(obj + ".tmp", obj)
        return obj, None

    jobs = jobs or min(8, os.cpu_count() or 4)
    with ThreadPoolExecutor(max_workers=jobs) as ex:
        results = list(ex.map(one, srcs))
    errs = [e for _, e in results if e]
    if errs:
        raise RuntimeError("\n".join(errs))
    objs = [o for o, _ in results]

    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    out = out or os.path.join(PKG, "_C" + suffix)
    os.makedirs(os.path.dirname(out), exist_ok=True)
    link = ([hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", out + ".tmp"] + objs +
            [f"-L{lib}", "-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python", "-lc10_hip",
             "-ltorch_hip", "-lamdhip64", "-lrccl", f"-Wl,-rpath,{lib}"])
    if verbose:
        print(" ".join(link), flush=True)
    r = subprocess.run(link, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    os.replace(out + ".tmp", out)
    # drop stale objects of sources that no longer exist / older hashes
    keep = set(objs)
    variant = custom_out or any(os.environ.get(k) for k in
                                     ("PDM_STAMPS", "PDM_DEBUG_BOUNDS", "PDM_HIPCC_FLAGS",
                                      "PDM_FILE_FLAGS"))
    for o in glob.glob(os.path.join(OBJ_DIR, "*.o")) if not variant else []:
        if o not in keep:
            try:
                os.unlink(o)
            except OSError:
                pass
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--out", default=None, help="output .so path (default: in-tree _C*.so)")
    a = ap.parse_args(argv)
    out = build(force=a.force, jobs=a.jobs, verbose=a.verbose, out=a.out)
    print(f"built {out}")


if __name__ == "__main__":
    main(sys.argv[1:])
