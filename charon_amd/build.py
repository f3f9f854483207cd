"""Build the HIP engine for gfx950 in-tree: charon_amd/libhipbls.so (C-ABI, include/hipbls.h)."""
import hashlib
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
    return sorted(hdrs) + [os.path.join(ROOT, "include", "hipbls.h")]


def _base_flags():
    return ["--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-I" + CSRC, "-I" + os.path.join(ROOT, "include")]


def source_digest():
    """SHA-256 over every source the library is compiled from (charon_amd/csrc/*.h|.hip and include/hipbls.h, by
    path relative to the repo root and content): compiled into the library as its build id (hipbls_build_id), and
    recomputed by smoke(), the GPU test session and bench.py from the sources shipped beside the binary."""
    h = hashlib.sha256()
    for f in _sources():
        h.update(os.path.relpath(f, ROOT).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    return h.hexdigest()


def flags_digest(extra=()):
    """SHA-256 of the compile flags (paths relative to the repo root, so a copy of the tree gives the same digest)."""
    flags = [x.replace(ROOT, ".") for x in _base_flags() + list(extra)]
    return hashlib.sha256(" ".join(flags).encode()).hexdigest()


_MARK = b"HIPBLS_BUILD_ID src="


def embedded_id(lib=LIB):
    """(src digest, flags digest) compiled into a built library, read from its bytes without loading it; None when
    the file is missing or carries no build id."""
    if not os.path.exists(lib):
        return None
    with open(lib, "rb") as fh:
        data = fh.read()
    i = data.find(_MARK)
    if i < 0:
        return None
    j = data.index(b"\0", i)
    fields = dict(kv.split("=", 1) for kv in data[i + len(b"HIPBLS_BUILD_ID "):j].decode().split())
    return fields.get("src"), fields.get("flags")


def stale(lib=LIB, extra=()):
    """A library is stale when its compiled-in digests differ from the sources' and the flags' (not by mtime: a copied
    tree keeps no meaningful mtimes)."""
    return embedded_id(lib) != (source_digest(), flags_digest(extra))


def verify(lib=None):
    """Raise when the library a process loads was not built from the sources beside it.  The
    product library must also carry the default flags; an A/B build (HIPBLS_LIB) only needs the same sources.
    Returns the source digest."""
    lib = lib or os.environ.get("HIPBLS_LIB") or LIB
    got = embedded_id(lib)
    want = source_digest()
    if got is None:
        raise RuntimeError("%s carries no build id: rebuild with charon_amd/build.py" % lib)
    if got[0] != want:
        raise RuntimeError("%s was built from other sources (build id %s, sources %s): rebuild with "
                           "charon_amd/build.py" % (lib, got[0][:16], want[:16]))
    if not os.environ.get("HIPBLS_LIB") and got[1] != flags_digest():
        raise RuntimeError("%s was built with non-default flags: rebuild with charon_amd/build.py" % lib)
    return want


def build(force=False, verbose=True, extra=(), out=LIB):
    """Build the library; `extra` adds compiler flags (e.g. -D variants) and `out` names another file for A/B
    measurements (loaded with HIPBLS_LIB=<path>); the product is the default in-tree build."""
    if not force and out == LIB and not stale(extra=extra):
        return LIB
    # the five translation units compile in parallel (each a separate code object; the link combines them), then link
    srcs = [os.path.join(CSRC, f) for f in ("hipbls.hip", "verify_lat.hip", "verify_hex.hip", "rlc_wide.hip", "fav_wide.hip")]
    flags = _base_flags() + list(extra)
    # the build id (hipbls_build_id): digests of the sources and of the flags, checked before any GPU run
    flags += ['-DHIPBLS_SRC_SHA="%s"' % source_digest(), '-DHIPBLS_FLAGS_SHA="%s"' % flags_digest(extra)]
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
