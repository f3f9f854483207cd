"""BASELINE configs C4 and C5 at full size on one GPU, through the C-ABI (VERDICT r02 "Next round" 1a/1b).

C2 (65,536 Verify) and C3 (10,000 x 7-of-10) run at full size in tests/test_gpu_r02.py.  Here:

* C4 (configs[3]): the 262,144-validator x 4-partial node batch (1,048,576 partials) through
  `hipbls_batch_verify_rlc` (host buffers, the drop-in call) in both root layouts -- (i) one root per validator,
  (ii) 2,048 committee roots -- and an all-valid stream, under every RLC mode (AUTO, WINDOWS, BATCH) and with the
  resident pubshare table.  The bitmap must equal the seeded corruption set (bench.py's construction), every mode
  must give the same statuses, and a seeded sample (corrupted items included) must equal the oracle's Verify
  (oracle/bls12381.py, herumi.go:285-301).
* C5 (configs[4]): the slot mix in one go -- C4(i) plus 32 x 4 proposer partials through the device RLC call on one
  stream, overlapped with the 512-key sync-committee FastAggregateVerify on another; the FAV verdict is checked by
  the oracle as well.

Sizes are the BASELINE ones; inputs are bench.py's (every item a function of (seed, config, index)).
"""
import ctypes
import os
import random

import pytest

pytestmark = pytest.mark.gpu

V = 262144  # validators in the C4 node batch (x 4 partials = 1,048,576)


@pytest.fixture(scope="module")
def impl():
    from charon_amd.tbls import HipBLS
    return HipBLS()


@pytest.fixture(scope="module")
def keys4(impl):
    import bench
    return bench.share_keys(impl, 4096, "c4")


def _rlc_host(impl, pks, sigs, midx, roots, seed):
    """hipbls_batch_verify_rlc on host buffers (the message table is already distinct, items adjacent by root)."""
    from charon_amd.tbls import _check, _offsets
    n = len(pks)
    blob, offs = _offsets(roots)
    idx = (ctypes.c_uint32 * n)(*midx)
    st = (ctypes.c_int32 * n)()
    _check(impl.lib.hipbls_batch_verify_rlc(b"".join(pks), b"".join(sigs), idx, n, blob, offs, len(roots), seed, st),
           impl.lib)
    return list(st)


def _rlc_keys_host(impl, kidx, sigs, midx, roots, seed):
    from charon_amd.tbls import _check, _offsets
    n = len(kidx)
    blob, offs = _offsets(roots)
    idx = (ctypes.c_uint32 * n)(*midx)
    k = (ctypes.c_uint32 * n)(*kidx)
    st = (ctypes.c_int32 * n)()
    _check(impl.lib.hipbls_batch_verify_rlc_keys(k, b"".join(sigs), idx, n, blob, offs, len(roots), seed, st),
           impl.lib)
    return list(st)


def _oracle_sample(pks, sigs, midx, roots, bad, st, seed, k_bad=6, k_good=6):
    from oracle import bls12381 as bls
    rng = random.Random(seed)
    sample = rng.sample(sorted(bad), min(k_bad, len(bad))) + rng.sample(range(len(pks)), k_good)
    for i in sample:
        assert st[i] == bls.verify_status(pks[i], roots[midx[i]], sigs[i]), i


@pytest.mark.parametrize("variant", ["i_root_per_validator", "ii_committee_roots"])
def test_c4_full_node_batch_every_mode(impl, keys4, variant):
    import bench
    from charon_amd.tbls import RLC_AUTO, RLC_BATCH, RLC_WINDOWS
    tag, n_roots = ("c4i", 0) if variant.startswith("i_") else ("c4ii", V // 128)
    pks, sigs, midx, roots, bad = bench.make_c4(impl, keys4, tag, 0, V, V, n_roots)
    assert len(pks) == 4 * V and len(roots) == (n_roots or V) and bad == bench.c4_node_bad(tag, V, 4096)
    seed = os.urandom(32)
    results = {}
    try:
        for name, mode in (("windows", RLC_WINDOWS), ("batch", RLC_BATCH), ("auto", RLC_AUTO)):
            impl.set_rlc_mode(mode)
            a0, p0, _ = impl.rlc_batch_stats()
            st = _rlc_host(impl, pks, sigs, midx, roots, seed)
            a1, p1, last = impl.rlc_batch_stats()
            assert {i for i, s in enumerate(st) if s != 0} == bad, name
            if name == "batch":  # the batch-wide check ran and failed (1 % invalid): the windows decided
                assert a1 - a0 == 1 and p1 == p0 and last == 0
            results[name] = st
        assert results["windows"] == results["batch"] == results["auto"]
        # the resident pubshare table gives the same statuses
        impl.set_rlc_mode(RLC_AUTO)
        table = list(dict.fromkeys(pks))
        assert set(impl.load_pubshares(table)) == {0}
        pos = {p: j for j, p in enumerate(table)}
        assert _rlc_keys_host(impl, [pos[p] for p in pks], sigs, midx, roots, seed) == results["windows"]
    finally:
        impl.set_rlc_mode(RLC_AUTO)
    _oracle_sample(pks, sigs, midx, roots, bad, results["windows"], 0xC4 + len(roots))


@pytest.mark.parametrize("variant", ["i_root_per_validator", "ii_committee_roots"])
def test_c4_all_valid_node_batch_decided_by_batch_check(impl, keys4, variant):
    """An all-valid 1M-partial node batch, one root per validator (i) or 2,048 committee roots (ii): the batch-wide
    Pippenger check alone passes it (no window pairing work); WINDOWS gives the same all-zero bitmap."""
    import bench
    from charon_amd.tbls import RLC_AUTO, RLC_BATCH, RLC_WINDOWS
    tag, n_roots = ("c4h", 0) if variant.startswith("i_") else ("c4hii", V // 128)
    pks, sigs, midx, roots, bad = bench.make_c4(impl, keys4, tag, 0, V, V, n_roots, corrupt=False)
    assert len(roots) == (n_roots or V)
    assert not bad
    seed = os.urandom(32)
    try:
        impl.set_rlc_mode(RLC_BATCH)
        a0, p0, _ = impl.rlc_batch_stats()
        st = _rlc_host(impl, pks, sigs, midx, roots, seed)
        a1, p1, last = impl.rlc_batch_stats()
        assert set(st) == {0} and a1 - a0 == 1 and p1 - p0 == 1 and last == 1
        assert impl.rlc_stats()[1:] == (0, 0)  # no window failed, nothing re-verified
        impl.set_rlc_mode(RLC_WINDOWS)
        assert set(_rlc_host(impl, pks, sigs, midx, roots, seed)) == {0}
    finally:
        impl.set_rlc_mode(RLC_AUTO)
    _oracle_sample(pks, sigs, midx, roots, set(), st, 0xC4A, k_bad=0, k_good=4)


def test_c5_slot_mix_overlapped(impl, keys4):
    """The full-slot mix: RLC over C4(i) + 32 x 4 proposer partials on one stream while the 512-key sync-committee
    FastAggregateVerify runs on another; bitmap == construction, FAV == oracle, sample == oracle."""
    import torch

    import bench
    from oracle import bls12381 as bls
    pks, sigs, midx, roots, bad = bench.make_c4(impl, keys4, "c4i", 0, V, V, 0)
    ppks, psigs, pmidx, proots, pbad = bench.make_c4(impl, bench.share_keys(impl, 128, "c5p"), "c5p", 0, 32, 32)
    base, off = len(pks), len(roots)
    pks, sigs, roots = pks + ppks, sigs + psigs, roots + proots
    midx = midx + [m + off for m in pmidx]
    bad = bad | {base + i for i in pbad}
    sync_sks = [bench._scalar("c5sync", k).to_bytes(32, "big") for k in range(512)]
    sync_pks, _ = impl.secret_to_public_key_batch(sync_sks)
    sync_root = bench._hb("c5sync", "root")
    ssigs, _ = impl.sign_batch(sync_sks, [sync_root] * 512)
    sync_agg = impl.aggregate(ssigs)
    dev = torch.device("cuda", 0)

    def u8(blobs):
        return torch.frombuffer(bytearray(b"".join(blobs)), dtype=torch.uint8).to(dev)

    n = len(pks)
    d_pk, d_sig, d_msg = u8(pks), u8(sigs), u8(roots)
    d_midx = torch.tensor(midx, dtype=torch.int32).to(dev)
    d_off = torch.arange(0, 32 * (len(roots) + 1), 32, dtype=torch.int64).to(dev)
    d_st = torch.full((n,), -7, dtype=torch.int32, device=dev)
    d_spk, d_ssig, d_smsg = u8(sync_pks), u8([sync_agg, sync_agg]), u8([sync_root, sync_root[::-1]])
    d_skoff = torch.tensor([0, 512, 1024], dtype=torch.int64).to(dev)
    d_spk2 = torch.cat([d_spk, d_spk])
    d_smoff = torch.tensor([0, 32, 64], dtype=torch.int64).to(dev)
    d_sst = torch.full((2,), -7, dtype=torch.int32, device=dev)
    s_rlc, s_fav = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    torch.cuda.synchronize(dev)
    lib = impl.lib
    rc = lib.hipbls_verify_aggregate_batch_device(d_spk2.data_ptr(), 1024, d_skoff.data_ptr(), 2, d_ssig.data_ptr(),
                                                  d_smsg.data_ptr(), d_smoff.data_ptr(), d_sst.data_ptr(),
                                                  ctypes.c_void_p(s_fav.cuda_stream))
    assert rc == 0
    rc = lib.hipbls_batch_verify_rlc_device(d_pk.data_ptr(), d_sig.data_ptr(), d_midx.data_ptr(), n, d_msg.data_ptr(),
                                            d_off.data_ptr(), len(roots), os.urandom(32), d_st.data_ptr(),
                                            ctypes.c_void_p(s_rlc.cuda_stream))
    assert rc == 0
    torch.cuda.synchronize(dev)
    st = d_st.cpu().tolist()
    assert {i for i, s in enumerate(st) if s != 0} == bad
    assert d_sst.cpu().tolist() == [0, 3]
    bls.verify_aggregate(sync_pks, sync_agg, sync_root)  # the oracle accepts the honest sync aggregate (raises if not)
    with pytest.raises(bls.BLSError):
        bls.verify_aggregate(sync_pks, sync_agg, sync_root[::-1])
    _oracle_sample(pks, sigs, midx, roots, bad, st, 0xC5, k_bad=4, k_good=4)
    # the proposer partials (own roots, at the end of the batch) against the oracle too
    for i in range(base, base + 8):
        assert st[i] == bls.verify_status(pks[i], roots[midx[i]], sigs[i])
