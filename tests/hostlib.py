"""ctypes loader for tests/native/libhost_ops.so (host build of the kernel arithmetic; test-only)."""
import ctypes
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "native", "host_ops.cpp")
LIB = os.path.join(HERE, "native", "libhost_ops.so")
CSRC = os.path.join(os.path.dirname(HERE), "charon_amd", "csrc")


def _stale():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [SRC] + [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    deps.append(os.path.join(os.path.dirname(HERE), "include", "hipbls.h"))
    return any(os.path.getmtime(d) > t for d in deps)


def build():
    if _stale():
        subprocess.check_call(["g++", "-std=c++17", "-O2", "-fPIC", "-shared", "-o", LIB, SRC])


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        _lib = ctypes.CDLL(LIB)
    return _lib


def buf(n):
    return ctypes.create_string_buffer(n)
