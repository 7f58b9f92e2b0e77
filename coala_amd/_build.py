"""Build the in-tree HIP shared library (gfx950) that backs the codec's C ABI (include/coalac.h).

The library is compiled straight with hipcc — no torch extension, no JIT cache — so the `.so` lands in
coala_amd/lib/ and travels with the repo snapshot to the GPU box (it is git-ignored, not gpurun-ignored).
"""
import os
import shutil
import subprocess

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
SRC = os.path.join(PKG, "csrc", "coalac.hip")
HDR = os.path.join(REPO, "include", "coalac.h")
LIB = os.path.join(PKG, "lib", "libcoalac.so")
ARCH = os.environ.get("COALAC_ARCH", "gfx950")

HIPCC_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", f"--offload-arch={ARCH}"]


def hipcc():
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (set HIPCC or install ROCm)")


def stale():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(p) > t for p in (SRC, HDR, __file__))


def build(force=False, verbose=False):
    """Compile coala_amd/lib/libcoalac.so for gfx950 if missing or older than its sources."""
    if not force and not stale():
        return LIB
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    tmp = LIB + ".tmp"
    cmd = [hipcc(), *HIPCC_FLAGS, "-o", tmp, SRC]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force=True, verbose=True))
