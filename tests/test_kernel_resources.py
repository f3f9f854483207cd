"""The built library's kernel resources, read from its gfx950 code object on the CPU (charon_amd/codeobj.py).

The per-lane private segment (scratch) of the deepest kernel sizes every hardware queue's scratch block (x 64 lanes x
32 wave slots x 256 CUs); all queues of a process share one 32 GiB region per device.  The build
refuses a library above PRIVATE_SEGMENT_BUDGET, derived so the library's four queues plus one more of the same depth
fit the region; this test holds the shipped .so to the same bound, checks that the runtime's kernel table (the
scratch budget hipbls_scratch_budget computes at init) names every kernel of the code objects, and checks the
metadata the roofline and occupancy arguments use (VGPRs, the LDS-resident Miller slot).
"""
import os

import pytest

from charon_amd import codeobj

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "charon_amd", "libhipbls.so")

pytestmark = pytest.mark.skipif(not os.path.exists(LIB), reason="libhipbls.so not built (run __graft_entry__.build())")


def test_budget_is_the_scratch_arithmetic():
    """PRIVATE_SEGMENT_BUDGET is the largest per-lane segment whose 2 MiB-aligned block (x 64 x 32 x 256) fits five
    times (the library's four queues + one) in the 32 GiB region: measured per-queue blocks 1,040 B -> 520 MiB and
    12,480 B -> 6,240 MiB (profiles/r05/r05_scratch_probe.txt, r05_scratch_layout.txt)."""
    b = codeobj.PRIVATE_SEGMENT_BUDGET
    assert b == 13104
    blk = lambda p: -(-p * codeobj.WAVE_SLOTS // codeobj.BLOCK_ALIGN) * codeobj.BLOCK_ALIGN
    assert blk(1040) == 520 << 20 and blk(12480) == 6240 << 20
    assert 5 * blk(b) <= codeobj.SCRATCH_REGION < 5 * blk(b + 16) + 5 * codeobj.BLOCK_ALIGN
    # round 3's 17,880 B/lane: four queues alone exceed the region (the round-3 aborts)
    assert 4 * blk(17880) > codeobj.SCRATCH_REGION


def test_runtime_kernel_table_names_every_kernel():
    import ctypes
    lib = ctypes.CDLL(LIB)
    lib.hipbls_kernel_names.restype = ctypes.c_char_p
    table = lib.hipbls_kernel_names().decode().split()
    assert len(table) == len(set(table))
    co = {r[0] for r in codeobj.resource_table(LIB)}
    assert set(table) == co - {"k_scratch_reserve"}


def test_reserve_kernels_cover_the_deepest_kernel():
    """The init-time reserve kernels (one dispatch per library stream) reach at least the deepest kernel's segment and
    stop at the budget."""
    rows = codeobj.resource_table(LIB)
    res = sorted(r[1] for r in rows if r[0] == "k_scratch_reserve")
    deepest = max(r[1] for r in rows if r[0] != "k_scratch_reserve")
    assert res and res[-1] == codeobj.PRIVATE_SEGMENT_BUDGET
    assert any(deepest <= x < deepest + 256 for x in res)


def test_every_kernel_within_scratch_budget():
    rows = codeobj.check_budget(LIB)
    assert len(rows) >= 30
    names = {r[0] for r in rows}
    for k in ("k_verify_fused", "k_verify_pair_lq4", "k_rlcb_items", "k_tagg_scale", "k_msm_run"):
        assert k in names, k
    assert max(r[1] for r in rows) <= codeobj.PRIVATE_SEGMENT_BUDGET


def test_budget_check_rejects_deeper_kernels():
    deepest = codeobj.resource_table(LIB)[0]
    with pytest.raises(RuntimeError, match="budget"):
        codeobj.check_budget(LIB, budget=deepest[1] - 1)


def test_lds_slot_kernels_fit_four_workgroups_per_cu():
    """The LDS-resident Miller f (576 B/lane x 64 lanes = 36 KiB per workgroup) must leave room for the four one-wave
    workgroups a CU runs at this register count: 4 x LDS <= 160 KiB."""
    for name, scratch, vgpr, lds in codeobj.resource_table(LIB):
        if name in ("k_verify_fused", "k_verify_keys", "k_rlc_window", "k_rlcb_chunks"):
            assert lds == 36864, name
            assert 4 * lds <= 160 * 1024


def test_race_polls_use_zero_extended_word_address(tmp_path):
    """Every mid-program `s_endpgm` of the latency code object is a replica-race poll (verify_lat.hip bls_race::poll).
    Its word address is rebuilt from two readfirstlane halves; readfirstlane returns int, and round 5's first race build
    sign-extended the low half over the high one (`s_bfe_i64`), a wild address for half of all buffers.  The fixed code
    builds the address with no sign extension and polls with a `global_load_dword ... sc1` (the first build's flat_ loads
never saw another XCD's word), checked on the disassembly."""
    import re
    import subprocess
    objdump = "/opt/rocm/lib/llvm/bin/llvm-objdump"
    if not os.path.exists(objdump) or not os.path.exists(LIB):
        pytest.skip("llvm-objdump or the library missing")
    polls = 0
    for i, co in enumerate(codeobj.code_objects(LIB)):
        f = tmp_path / ("co%d.elf" % i)
        f.write_bytes(co)
        lines = subprocess.run([objdump, "-d", "--no-show-raw-insn", str(f)], check=True, capture_output=True,
                               text=True).stdout.splitlines()
        for j, ln in enumerate(lines):
            # a poll: `s_cbranch_scc1` over one `s_endpgm`, more code after it (other kernels' early exits differ)
            if "s_endpgm" not in ln or j + 1 >= len(lines) or not re.search(r"s_cbranch_scc1 1\s", lines[j - 1]):
                continue
            if not lines[j + 1].strip() or lines[j + 1].strip().startswith(("0", "<")):
                continue
            window = lines[max(0, j - 30):j]
            polls += 1
            assert not any("s_bfe_i64" in w or "s_ashr_i32" in w for w in window), "\n".join(window)
            # a flag written on another XCD is seen by global/buffer sc1 loads, never flat ones (MI355X_MICROARCH.md)
            assert not any("flat_load" in w for w in window), "\n".join(window)
            assert any("global_load_dword" in w and "sc1" in w for w in window), "\n".join(window)
    assert polls > 0
