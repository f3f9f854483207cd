"""C-ABI boundary checks that need no GPU: the library loads, exports every function that
include/hipbls.h declares, and the ctypes mirror (charon_amd/tbls.py) declares exactly that set.
No compute entry point is called here (there is no device in this container)."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "hipbls.h")
LIB = os.path.join(ROOT, "charon_amd", "libhipbls.so")


def header_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(hipbls_[a-z0-9_]+)\s*\(", text)))


def test_header_parses():
    fns = header_functions()
    assert "hipbls_verify_batch" in fns and "hipbls_threshold_aggregate_batch" in fns
    assert len(fns) >= 18


@pytest.mark.skipif(not os.path.exists(LIB), reason="libhipbls.so not built (run __graft_entry__.build())")
def test_library_exports_every_declared_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (hipbls_[a-z0-9_]+)$", out, flags=re.M))
    missing = [f for f in header_functions() if f not in exported]
    assert not missing, missing


@pytest.mark.skipif(not os.path.exists(LIB), reason="libhipbls.so not built (run __graft_entry__.build())")
def test_ctypes_mirror_declares_header_set():
    from charon_amd import tbls
    assert sorted(tbls.exported_symbols()) == header_functions()
    lib = tbls.load_library()
    assert lib.hipbls_abi_version() == 12


def test_no_cpu_fallback_without_library(tmp_path):
    """The product path fails loudly when the HIP library is absent (no oracle/CPU fallback)."""
    from charon_amd import tbls
    saved = tbls._lib
    tbls._lib = None
    try:
        with pytest.raises(RuntimeError, match="not built"):
            tbls.load_library(str(tmp_path / "missing.so"))
    finally:
        tbls._lib = saved


def test_product_never_imports_oracle():
    for dirpath, _, files in os.walk(os.path.join(ROOT, "charon_amd")):
        for f in files:
            if f.endswith((".py", ".h", ".hip", ".cpp")):
                src = open(os.path.join(dirpath, f), errors="replace").read()
                assert "oracle" not in re.findall(r"(?:import|from|#include)\s+[\"<]?([a-z_./]+)", src), f


@pytest.mark.skipif(not os.path.exists(LIB), reason="libhipbls.so not built (run __graft_entry__.build())")
def test_plan_ranges_tiles_exactly():
    """hipbls_plan_ranges (the batch split across devices, host code): ranges tile [0, n) in order, are balanced,
    and with run keys (a validator's message index) no run straddles two ranges unless it is longer than half a
    share (then the bound stays at the equal split)."""
    import random
    from charon_amd.tbls import plan_ranges
    rng = random.Random(3)
    for n in (0, 1, 7, 64, 1000, 1048576, 262144 * 4 + 128):
        for parts in (1, 2, 3, 8):
            b = plan_ranges(n, parts)
            assert b[0] == 0 and b[-1] == n and all(b[i] <= b[i + 1] for i in range(parts))
            if n >= parts:
                sizes = [b[i + 1] - b[i] for i in range(parts)]
                assert max(sizes) - min(sizes) <= 1
    for trial in range(40):
        n = rng.randrange(1, 5000)
        runs = []
        while sum(runs) < n:
            runs.append(rng.choice([1, 4, 4, 7, 10, 600]))
        keys = []
        for k, r in enumerate(runs):
            keys += [k] * r
        keys = keys[:n]
        parts = rng.choice([2, 3, 4, 8])
        b = plan_ranges(n, parts, keys)
        assert b[0] == 0 and b[-1] == n and all(b[i] <= b[i + 1] for i in range(parts))
        share = n // parts
        for k in range(1, parts):
            x = n * k // parts
            y = b[k]
            if y in (0, n) or keys[y] != keys[y - 1]:
                assert x <= y <= x + share // 2 or y == n or y == x, (x, y)
            else:  # the run is longer than the window: the bound stays at the equal split
                assert y == max(x, b[k - 1])
        # C4 shape: 4 partials per validator -> every inner bound starts a validator
        keys4 = [i // 4 for i in range(4 * 1000)]
        b4 = plan_ranges(4000, 8, keys4)
        assert all(x % 4 == 0 for x in b4)


def test_build_id_is_the_shipped_sources():
    """The in-tree library carries the digests of the sources and default flags it was built from (VERDICT r05 next
    3), both in its bytes (read without loading) and through hipbls_build_id()."""
    from charon_amd import build, tbls
    assert build.embedded_id() == (build.source_digest(), build.flags_digest())
    assert tbls.build_id() == {"src": build.source_digest(), "flags": build.flags_digest()}
    assert build.verify() == build.source_digest()


def test_build_id_detects_other_sources(tmp_path, monkeypatch):
    from charon_amd import build
    fake = tmp_path / "lib.so"
    fake.write_bytes(b"\x7fELF...HIPBLS_BUILD_ID src=" + b"0" * 64 + b" flags=" + b"1" * 64 + b"\0tail")
    assert build.embedded_id(str(fake)) == ("0" * 64, "1" * 64)
    assert build.stale(str(fake))
    with pytest.raises(RuntimeError, match="other sources"):
        build.verify(str(fake))
    (tmp_path / "none.so").write_bytes(b"\x7fELF no id")
    with pytest.raises(RuntimeError, match="no build id"):
        build.verify(str(tmp_path / "none.so"))
