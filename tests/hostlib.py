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


CB_SRC = os.path.join(HERE, "native", "cpu_baseline.cpp")
CB_LIB = os.path.join(HERE, "native", "libcpu_baseline.so")


def build():
    """The g++ artefacts only (host arithmetic, CPU baseline): CPU tests reach this through lib() and must not need
    ROCm.  The gfx950 test library is built by build_gpu_units(), called from __graft_entry__.build()."""
    if _stale():
        subprocess.check_call(["g++", "-std=c++17", "-O2", "-fPIC", "-shared", "-o", LIB, SRC])
    build_cpu_baseline()


GU_SRC = os.path.join(HERE, "native", "gpu_units.hip")
GU_LIB = os.path.join(HERE, "native", "libgpu_units.so")


def build_gpu_units():
    """Test-only device entry points into single kernel building blocks (tests/test_gpu_units.py), gfx950."""
    deps = [GU_SRC] + [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    if not os.path.exists(GU_LIB) or any(os.path.getmtime(d) > os.path.getmtime(GU_LIB) for d in deps):
        subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                               "-I" + CSRC, "-I" + os.path.join(os.path.dirname(HERE), "include"),
                               "-o", GU_LIB + ".tmp", GU_SRC])
        os.replace(GU_LIB + ".tmp", GU_LIB)


def gpu_units_lib():
    """ctypes handle on tests/native/libgpu_units.so (built by __graft_entry__.build(); -m gpu tests only)."""
    if not os.path.exists(GU_LIB):
        raise RuntimeError("tests/native/libgpu_units.so not built (run __graft_entry__.build())")
    return ctypes.CDLL(GU_LIB)


def build_cpu_baseline():
    """-O3, portable x86-64 (the .so built here runs on the GPU box's host CPU), one thread per core at run time."""
    deps = [CB_SRC] + [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    if not os.path.exists(CB_LIB) or any(os.path.getmtime(d) > os.path.getmtime(CB_LIB) for d in deps):
        subprocess.check_call(["g++", "-std=c++17", "-O3", "-fPIC", "-shared", "-pthread", "-o", CB_LIB, CB_SRC])


def cpu_baseline_lib():
    """ctypes handle on tests/native/libcpu_baseline.so (bench.py's cpu_baseline leg only)."""
    if not os.path.exists(CB_LIB):
        build_cpu_baseline()
    lib = ctypes.CDLL(CB_LIB)
    lib.cb_verify_batch.restype = ctypes.c_double
    lib.cb_threshold_aggregate_batch.restype = ctypes.c_double
    return lib


_lib = None
# HIPBLS_HOST_CONTRACT=1 (tests/test_operand_contract.py): lib() is the BLS_CONTRACT_CHECK build, which counts every
# product / add / sub whose operands break the device routines' contracts (field.h BLS_CONTRACT); at exit the count
# and the first violation go to HIPBLS_HOST_CONTRACT_OUT.
CONTRACT = os.environ.get("HIPBLS_HOST_CONTRACT") == "1"
CT_LIB = os.path.join(HERE, "native", "libhost_ops_contract.so")


def _contract_lib():
    deps = [SRC] + [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    if not os.path.exists(CT_LIB) or any(os.path.getmtime(d) > os.path.getmtime(CT_LIB) for d in deps):
        subprocess.check_call(["g++", "-std=c++17", "-O2", "-fPIC", "-shared", "-DBLS_CONTRACT_CHECK", "-o",
                               CT_LIB + ".tmp", SRC])
        os.replace(CT_LIB + ".tmp", CT_LIB)
    L = ctypes.CDLL(CT_LIB)
    L.ht_contract_violations.restype = ctypes.c_uint64
    L.ht_contract_first.restype = ctypes.c_char_p
    L.ht_contract_lazy_operands.restype = ctypes.c_uint64
    out = os.environ.get("HIPBLS_HOST_CONTRACT_OUT")
    if out:
        import atexit
        import json

        def dump():
            first = L.ht_contract_first()
            with open(out, "w") as f:
                json.dump({"violations": L.ht_contract_violations(), "first": first.decode() if first else None,
                           "lazy_operands": L.ht_contract_lazy_operands()}, f)
        atexit.register(dump)
    return L


def lib():
    global _lib
    if _lib is None:
        if CONTRACT:
            _lib = _contract_lib()
        else:
            build()
            _lib = ctypes.CDLL(LIB)
    return _lib


def buf(n):
    return ctypes.create_string_buffer(n)
