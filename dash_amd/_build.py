"""Native build driver for dash_amd.

Compiles the host C++ core (amdclang++) and the HIP kernels for gfx950
(hipcc --offload-arch=gfx950) into one in-tree extension module
``dash_amd/_dash_native*.so``. No torch headers are involved. A full rebuild
takes 2.5-4.5 minutes with 8 jobs (the per-K chain units dominate,
docs/BUILD.md); incremental rebuilds only recompile changed translation
units.

Usage:  python -m dash_amd._build [--clean] [--jobs N] [--debug]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
BUILD = Path(os.environ.get("DASH_BUILD_DIR", str(PKG.parent / "build" / "native")))
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
ARCH = os.environ.get("DASH_GPU_ARCH", "gfx950")

HOST_SOURCES = ["core.cpp", "gadgets.cpp", "garbler.cpp", "evaluator.cpp", "serialize.cpp", "onnx.cpp", "dataloader.cpp", "bind.cpp"]
# kernels_mrs_a.hip (K = 7, the headline) first: the longest units start first in the parallel build
HIP_SOURCES = ["hip/kernels_mrs_a.hip", "hip/kernels_gadget.hip", "hip/garble_gpu.hip", "hip/runtime.hip",
               "hip/kernels_mrs_b.hip", "hip/kernels_mrs_c.hip", "hip/kernels_mrs_d.hip", "hip/kernels_mrs_e.hip",
               "hip/kernels_mrs_f.hip", "hip/kernels_label.hip", "hip/kernels_gemm.hip", "hip/guard.hip"]


def ext_suffix() -> str:
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def target_path() -> Path:
    return PKG / ("_dash_native" + ext_suffix())


def _includes() -> list[str]:
    import pybind11

    return [f"-I{CSRC}", f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}"]


def _host_cmd(src: Path, obj: Path, debug: bool) -> list[str]:
    cxx = str(ROCM / "llvm" / "bin" / "clang++")
    if not Path(cxx).exists():
        cxx = "g++"
    opt = ["-O1", "-g"] if debug else ["-O3"]
    return [cxx, "-std=c++17", "-fPIC", "-fvisibility=hidden", "-maes", "-msse4.2", "-mavx2", "-mpclmul",
            *opt, "-Wall", "-Wno-unused-function", *_includes(), "-MMD", "-MF", str(obj) + ".d", "-c", str(src),
            "-o", str(obj)]


def _hip_cmd(src: Path, obj: Path, debug: bool) -> list[str]:
    hipcc = str(ROCM / "bin" / "hipcc")
    opt = ["-O1", "-g"] if debug else ["-O3"]
    extra = os.environ.get("DASH_HIP_FLAGS", "").split()  # e.g. -DDASH_AES_BLOCK=512 for A/B builds
    return [hipcc, "-std=c++17", "-fPIC", "-fvisibility=hidden", f"--offload-arch={ARCH}", "-maes", "-msse4.2",
            *opt, "-Wno-unused-result", *extra, *_includes(), "-MMD", "-MF", str(obj) + ".d", "-c", "-x", "hip",
            str(src), "-o", str(obj)]


def _dep_headers(obj: Path) -> list[Path] | None:
    """In-tree headers the object was compiled from (the compiler's -MMD file), or None without one."""
    d = Path(str(obj) + ".d")
    if not d.exists():
        return None
    text = d.read_text().replace("\\\n", " ")
    _, _, deps = text.partition(":")
    out = []
    for tok in deps.split():
        p = Path(tok)
        if p.suffix in (".h", ".cuh", ".hpp") and str(p).startswith(str(CSRC)):
            out.append(p)
    return out


def _deps_newer(obj: Path, src: Path) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    if src.stat().st_mtime > t:
        return True
    hdrs = _dep_headers(obj)
    if hdrs is None:  # no dependency file yet: any in-tree header may be included
        hdrs = list(CSRC.glob("*.h")) + list(CSRC.glob("hip/*.h")) + list(CSRC.glob("hip/*.cuh"))
    for h in hdrs:
        if not h.exists() or h.stat().st_mtime > t:
            return True
    return False


def build(jobs: int | None = None, debug: bool = False, clean: bool = False, verbose: bool = False) -> Path:
    if clean and BUILD.exists():
        shutil.rmtree(BUILD)
    BUILD.mkdir(parents=True, exist_ok=True)
    jobs = jobs or min(8, os.cpu_count() or 4)
    tasks = []
    objs = []
    for s in HOST_SOURCES:
        src = CSRC / s
        obj = BUILD / (s.replace("/", "_") + ".o")
        objs.append(obj)
        if _deps_newer(obj, src):
            tasks.append(_host_cmd(src, obj, debug))
    for s in HIP_SOURCES:
        src = CSRC / s
        if not src.exists():
            continue
        obj = BUILD / (s.replace("/", "_") + ".o")
        objs.append(obj)
        if _deps_newer(obj, src):
            tasks.append(_hip_cmd(src, obj, debug))

    def run(cmd):
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        if r.stderr.strip() and verbose:
            print(r.stderr, file=sys.stderr)
        return cmd[-1]

    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        for f in cf.as_completed([ex.submit(run, t) for t in tasks]):
            f.result()

    out = target_path()
    newest = max(o.stat().st_mtime for o in objs)
    if tasks or not out.exists() or out.stat().st_mtime < newest:
        tmp = out.with_suffix(".tmp.so")
        link = [str(ROCM / "bin" / "hipcc"), "-shared", "-fPIC", f"--offload-arch={ARCH}", *map(str, objs), "-o",
                str(tmp), f"-L{ROCM / 'lib'}", f"-Wl,-rpath,{ROCM / 'lib'}", "-lamdhip64",
                "-lrocprofiler-sdk-roctx", "-lpthread"]
        if verbose:
            print(" ".join(link), flush=True)
        r = subprocess.run(link, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, out)
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("--jobs", type=int, default=None)
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args()
    p = build(jobs=a.jobs, debug=a.debug, clean=a.clean, verbose=a.verbose)
    print(p)


if __name__ == "__main__":
    main()
