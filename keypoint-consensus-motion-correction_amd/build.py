"""Build libkcmc.so (HIP kernels for gfx950 + the C ABI) in-tree with hipcc.

Usage: ``python -m kcmc_amd.build`` or ``kcmc_amd.build.build()``; also driven by
``__graft_entry__.build()``.  Objects are compiled in parallel, then linked into
``<package>/libkcmc.so`` (git-ignored; travels to the GPU box with the snapshot).
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG_DIR, "csrc")
REPO = os.path.dirname(PKG_DIR)
LIB_PATH = os.path.join(PKG_DIR, "libkcmc.so")
OFFLOAD_ARCH = os.environ.get("KCMC_OFFLOAD_ARCH", "gfx950")
SOURCES = ["capi.cpp", "consensus.hip", "hostalg.cpp", "match.hip", "match_f32.hip", "match_hamming.hip", "normalize.hip", "orb.hip", "pyramid.hip", "ransac.hip", "ransac_model.hip", "warp.hip"]
HEADERS = ["kcmc_internal.h", "ransac_common.h", os.path.join("..", "..", "include", "kcmc.h")]

COMMON_FLAGS = [
    f"--offload-arch={OFFLOAD_ARCH}",
    "-O3",
    "-fPIC",
    "-std=c++17",
    "-ffp-contract=off",  # reproduce the reference's operation-by-operation rounding
    "-Wall",
    "-Wno-unused-function",
    f"-I{os.path.join(REPO, 'include')}",
]


def hipcc() -> str:
    p = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(p):
        raise RuntimeError("hipcc not found: the kcmc HIP library cannot be built")
    return p


def _newest_input_mtime() -> float:
    paths = [os.path.join(CSRC, s) for s in SOURCES] + [os.path.join(CSRC, h) for h in HEADERS]
    paths.append(os.path.abspath(__file__))
    return max(os.path.getmtime(p) for p in paths)


def up_to_date() -> bool:
    return os.path.exists(LIB_PATH) and os.path.getmtime(LIB_PATH) >= _newest_input_mtime()


# Per-source flags.  match.hip: MFMA results in VGPRs (the K1 epilogue reads every
# accumulator once; the AGPR form added a v_accvgpr_read per distance).
EXTRA_FLAGS = {"match.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form"]}


def _compile(src: str, obj: str) -> None:
    cmd = [hipcc(), *COMMON_FLAGS, *EXTRA_FLAGS.get(src, []), "-c", os.path.join(CSRC, src), "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")


def build(force: bool = False, verbose: bool = True) -> str:
    """Compile and link libkcmc.so if any source changed; return its path."""
    if not force and up_to_date():
        return LIB_PATH
    objdir = os.path.join(PKG_DIR, "build")
    os.makedirs(objdir, exist_ok=True)
    objs = [os.path.join(objdir, os.path.splitext(s)[0] + ".o") for s in SOURCES]
    jobs = min(len(SOURCES), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)), 8)
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        list(ex.map(lambda so: _compile(*so), zip(SOURCES, objs)))
    tmp = LIB_PATH + ".tmp"
    cmd = [hipcc(), f"--offload-arch={OFFLOAD_ARCH}", "-shared", "-fPIC", "-o", tmp, *objs, "-lpthread"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, LIB_PATH)
    if verbose:
        print(f"[kcmc] built {LIB_PATH}", file=sys.stderr)
    return LIB_PATH


if __name__ == "__main__":
    build(force="--force" in sys.argv)
