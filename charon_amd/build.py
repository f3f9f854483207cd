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
    # the three translation units compile in parallel (each a separate code object; the link combines them), then link
    srcs = [os.path.join(CSRC, f) for f in ("hipbls.hip", "verify_lat.hip", "verify_hex.hip")]
    flags = ["--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-I" + CSRC, "-I" + os.path.join(ROOT, "include")]
    flags += list(extra)
    objs = [out + "." + os.path.splitext(os.path.basename(src))[0] + ".o" for src in srcs]
    procs = []
    for src, obj in zip(srcs, objs):
        cmd = ["hipcc"] + flags + ["-c", "-o", obj, src]
        if verbose:
            print("[hipbls] " + " ".join(cmd), flush=True)
        procs.append(subprocess.Popen(cmd))
    rcs = [p.wait() for p in procs]
    if any(rcs):
        for obj in objs:
            if os.path.exists(obj):
                os.remove(obj)
        raise subprocess.CalledProcessError(max(rcs), "hipcc")
    cmd = ["hipcc", "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", out + ".tmp"] + objs + [
        "-L/opt/rocm/lib", "-lhsa-runtime64"]
    if verbose:
        print("[hipbls] " + " ".join(cmd), flush=True)
    try:
        subprocess.check_call(cmd)
    finally:
        for obj in objs:
            if os.path.exists(obj):
                os.remove(obj)
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
