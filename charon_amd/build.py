"""Build the HIP engine for gfx950 in-tree: charon_amd/libhipbls.so (C-ABI, include/hipbls.h)."""
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "libhipbls.so")
ARCH = os.environ.get("HIPBLS_ARCH", "gfx950")


def _sources():
    hdrs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".h", ".hip"))]
    return hdrs + [os.path.join(ROOT, "include", "hipbls.h")]


def stale(lib=LIB):
    if not os.path.exists(lib):
        return True
    t = os.path.getmtime(lib)
    return any(os.path.getmtime(s) > t for s in _sources())


def build(force=False, verbose=True, extra=(), out=LIB):
    """Build the library; `extra` adds compiler flags (e.g. -D variants) and `out` names another file for A/B
    measurements (loaded with HIPBLS_LIB=<path>); the product is the default in-tree build."""
    if not force and out == LIB and not stale():
        return LIB
    cmd = ["hipcc", "--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-shared",
           "-I" + CSRC, "-I" + os.path.join(ROOT, "include"),
           "-o", out + ".tmp", os.path.join(CSRC, "hipbls.hip"), os.path.join(CSRC, "verify_lat.hip"),
           os.path.join(CSRC, "verify_hex.hip"),
           "-L/opt/rocm/lib", "-lhsa-runtime64"] + list(extra)
    if verbose:
        print("[hipbls] " + " ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    # scratch budget per lane (charon_amd/codeobj.py): a deeper kernel fails the build here instead of
    # exhausting the hardware queues' scratch under load (HSA_STATUS_ERROR_OUT_OF_RESOURCES aborts the process)
    from charon_amd import codeobj
    try:
        codeobj.check_budget(out + ".tmp")
    except Exception:
        os.remove(out + ".tmp")
        raise
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    build(force="--force" in sys.argv)
