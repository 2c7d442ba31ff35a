"""Build the HIP C-ABI library ``libptv_amd.so`` in-tree for gfx950.

Plain ``hipcc`` (no torch extension machinery): each translation unit is
compiled to an object with ``--offload-arch=gfx950`` and linked into one
shared library next to this file, so the snapshot that travels to the GPU
box carries it.  ``-ffp-contract=off`` is load-bearing: the k-NN epilogue
reproduces numpy's rounding sequence (no fused multiply-adds).
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
INCLUDE = os.path.join(os.path.dirname(HERE), "include")
LIB = os.path.join(HERE, "libptv_amd.so")
BUILD = os.path.join(HERE, "csrc", "_build")
# the k-NN kernel's list lengths compile in parallel (ptv_knn_k*.hip instantiate ptv_knn_impl.hpp)
KNN_PARTS = ["ptv_knn_k" + g + ".hip" for g in "abcdefgh"]
SOURCES = (["ptv_api.cpp", "ptv_bin.hip", "ptv_knn.hip"] + KNN_PARTS +
           ["ptv_rbf.hip"] + ["ptv_rbf_ns_" + g + ".hip" for g in "abcd"] +
           ["ptv_div.hip", "ptv_mask.hip", "ptv_filter.hip", "ptv_linear.hip", "ptv_knn_big.hip"])
ARCH = os.environ.get("PTV_OFFLOAD_ARCH", "gfx950")
# per-file extras: the local-RBF kernel keeps each voxel's system row in registers, so every
# loop over the row must unroll fully (a partial unroll turns the row into scratch memory)
EXTRA = {f: ["-mllvm", "-pragma-unroll-threshold=1000000"] for f in ["ptv_rbf.hip"] + ["ptv_rbf_ns_" + g + ".hip" for g in "abcd"]}
# the null-space kernel's persistent quad loop: machine LICM would hoist every VGPR constant (the
# log polynomial, LDS offsets) out of it, live across the whole solve (~30 VGPRs, spills at 32 slots)
for _f in ["ptv_rbf.hip"] + ["ptv_rbf_ns_" + g + ".hip" for g in "abcd"]:  # k_rbf_spd16 loops the same way
    EXTRA[_f] += ["-mllvm", "-disable-machine-licm"]

COMMON = ["-O3", "-fPIC", "-std=c++17", "-ffp-contract=off", f"--offload-arch={ARCH}",
          "-I", INCLUDE, "-I", CSRC, "-Wno-unused-result"]
# dev A/B builds: PTV_EXTRA_FLAGS="-DPTV_KNN_WAVES=5" PTV_BUILD_TAG=w5 builds ab/libptv_w5.so
# (own object directory) without touching the shipped library
EXTRA_FLAGS = os.environ.get("PTV_EXTRA_FLAGS", "").split()
TAG = os.environ.get("PTV_BUILD_TAG", "")
if TAG:
    LIB = os.path.join(os.path.dirname(HERE), "ab", f"libptv_{TAG}.so")
    BUILD = os.path.join(HERE, "csrc", "_build_" + TAG)
    EXTRA_FLAGS.append("-DPTV_DEV_KNOBS=1")  # only dev builds read the PTV_* tuning variables


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build libptv_amd.so)")


def _stale(obj: str, deps) -> bool:
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(d) > t for d in deps)


def build(verbose: bool = False, force: bool = False) -> str:
    os.makedirs(BUILD, exist_ok=True)
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    cc = hipcc()
    headers = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hpp", ".h"))]
    headers.append(os.path.join(INCLUDE, "ptv_api.h"))
    jobs = []
    objs = []
    for src in SOURCES:
        sp = os.path.join(CSRC, src)
        obj = os.path.join(BUILD, src + ".o")
        objs.append(obj)
        if force or _stale(obj, [sp, __file__] + headers):
            lang = ["-x", "hip"]
            jobs.append([cc, *COMMON, *EXTRA_FLAGS, *EXTRA.get(src, []), *lang, "-c", sp, "-o", obj])

    def run(cmd):
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        return r

    workers = int(os.environ.get("PTV_BUILD_JOBS", str(min(16, os.cpu_count() or 4))))
    # longest translation units first
    jobs.sort(key=lambda cmd: -os.path.getsize(cmd[-3]))
    with ThreadPoolExecutor(max_workers=max(1, min(workers, len(jobs)))) as ex:
        list(ex.map(run, jobs))
    if force or jobs or _stale(LIB, objs):
        run([cc, "-shared", "-fPIC", "-pthread", f"--offload-arch={ARCH}", *objs, "-o", LIB])
    return LIB


if __name__ == "__main__":
    print(build(verbose=True, force="--force" in sys.argv))
