#!/usr/bin/env python3
"""Build the in-tree native extensions for gfx950 (MI355X).

Host C++ (.cpp) is compiled with g++ (-fopenmp -> libgomp, the same OpenMP
runtime PyTorch uses, so the two never clash in one process); HIP sources
(.hip) are compiled with hipcc --offload-arch=gfx950; everything is linked
into one pybind11 module per component that lands inside the package, so the
.so travels with the repo snapshot to the GPU box.

Usage: python tools/build_native.py [--jobs N] [--force] [--only NAME]
"""
from __future__ import annotations

import argparse
import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
ARCH = os.environ.get("SML_OFFLOAD_ARCH", "gfx950")
BUILD = ROOT / "build" / "native"


def _py_includes() -> list[str]:
    import pybind11

    return [f"-I{sysconfig.get_paths()['include']}", f"-I{pybind11.get_include()}"]


# module name -> (source dir, sources, extra link libs)
MODULES = {
    "_gbdt": (
        "csrc/gbdt",
        [
            "config.cpp",
            "dataset.cpp",
            "tree.cpp",
            "objective.cpp",
            "backend_cpu.cpp",
            "booster.cpp",
            "comm_rccl.cpp",
            "dev_pool.cpp",
            "bindings.cpp",
            "backend_gpu.hip",
            "valid_gpu.hip",
            "predict_gpu.hip",
            "comm_p2p.hip",
            "bin_encode.hip",
            "metric_gpu.hip",
        ],
        ["-lrccl", "-lrocprofiler-sdk-roctx"],
    ),
    # plain C ABI (no Python): csrc/gbdt/c_api.cpp over the same engine objects -> synapseml_amd/lib/
    "libsml_gbdt": (
        "csrc/gbdt",
        ["config.cpp", "dataset.cpp", "tree.cpp", "objective.cpp", "backend_cpu.cpp", "booster.cpp", "comm_rccl.cpp",
         "dev_pool.cpp", "backend_gpu.hip", "valid_gpu.hip", "predict_gpu.hip", "metric_gpu.hip", "bin_encode.hip",
         "comm_p2p.hip", "c_api.cpp"],
        ["-lrccl", "-lrocprofiler-sdk-roctx", "-Wl,-z,defs"],
    ),
    "_vw": (
        "csrc/vw",
        ["vw_core.cpp", "vw_bindings.cpp", "vw_gpu.hip", "../gbdt/dev_pool.cpp"],
        ["-lrccl"],
    ),
    "_image": (
        "csrc/image",
        ["image_bindings.cpp", "image_ops.cpp", "jpeg_decode.cpp", "image_gpu.hip"],
        [],
    ),
    "_nn": (
        "csrc/nn",
        ["nn_bindings.cpp", "nn_ops.hip", "conv_mfma.hip", "gemm_mfma.hip", "conv_direct.hip"],
        [],
    ),
}

CXXFLAGS = ["-O3", "-fPIC", "-std=c++17", "-Wall", "-Wno-unused-function", "-Wno-sign-compare"]
HOST_DEFS = ["-D__HIP_PLATFORM_AMD__=1", f"-I{ROCM}/include"]


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(" ".join(cmd) + "\n" + r.stdout + r.stderr)
        raise SystemExit(f"compile failed: {cmd[-1]}")


def _obj_for(src: Path, flags: list[str]) -> Path:
    h = hashlib.sha1()
    h.update(src.read_bytes())
    # headers of the same directory invalidate every object (small projects)
    for hdr in sorted(src.parent.glob("*.h")):
        h.update(hdr.read_bytes())
    h.update(" ".join(flags).encode())
    return BUILD / f"{src.stem}.{src.suffix[1:]}.{h.hexdigest()[:12]}.o"


def compile_one(src: Path, inc: list[str]) -> Path:
    if src.suffix == ".hip":
        flags = [str(ROCM / "bin" / "hipcc"), f"--offload-arch={ARCH}", "-x", "hip", *CXXFLAGS,
                 "-munsafe-fp-atomics", *inc]
    else:
        flags = ["g++", "-fopenmp", *CXXFLAGS, *HOST_DEFS, *inc]
    obj = _obj_for(src, flags)
    if not obj.exists():
        _run([*flags, "-c", str(src), "-o", str(obj)])
    return obj


def build(jobs: int = 8, force: bool = False, only: str | None = None) -> list[Path]:
    BUILD.mkdir(parents=True, exist_ok=True)
    if force:
        shutil.rmtree(BUILD)
        BUILD.mkdir(parents=True)
    ext = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    out_paths = []
    for name, (d, srcs, libs) in MODULES.items():
        if only and name != only:
            continue
        src_dir = ROOT / d
        sources = [src_dir / s for s in srcs if (src_dir / s).exists()]
        if not sources:
            continue
        inc = [f"-I{src_dir}", f"-I{ROOT / 'csrc'}", *_py_includes()]
        with ThreadPoolExecutor(max_workers=jobs) as ex:
            objs = list(ex.map(lambda s: compile_one(s, inc), sources))
        if name.startswith("lib"):
            (ROOT / "synapseml_amd" / "lib").mkdir(exist_ok=True)
            out = ROOT / "synapseml_amd" / "lib" / f"{name}.so"
        else:
            out = ROOT / "synapseml_amd" / f"{name}{ext}"
        link = ["g++", "-shared", "-fopenmp", "-o", str(out), *map(str, objs), f"-L{ROCM}/lib",
                "-lamdhip64", *libs, f"-Wl,-rpath,{ROCM}/lib"]
        _run(link)
        out_paths.append(out)
    return out_paths


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--only", default=None)
    a = ap.parse_args()
    for p in build(a.jobs, a.force, a.only):
        print("built", p.relative_to(ROOT))


if __name__ == "__main__":
    main()
