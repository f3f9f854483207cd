"""The built library's kernel resources, read from its gfx950 code object on the CPU (charon_amd/codeobj.py).

The per-lane private segment (scratch) of the deepest kernel sizes every hardware queue's scratch allocation; round 3
saw HSA_STATUS_ERROR_OUT_OF_RESOURCES aborts once kernels reached ~17.9 KB/lane.  The build refuses
a library above PRIVATE_SEGMENT_BUDGET; this test holds the shipped .so to the same bound and checks the metadata the
roofline and occupancy arguments use (VGPRs, the LDS-resident Miller slot).
"""
import os

import pytest

from charon_amd import codeobj

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "charon_amd", "libhipbls.so")

pytestmark = pytest.mark.skipif(not os.path.exists(LIB), reason="libhipbls.so not built (run __graft_entry__.build())")


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
