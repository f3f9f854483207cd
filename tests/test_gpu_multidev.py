"""One process, several device contexts (VERDICT r02 "Next round" 2).

charon is one process per node (/root/reference/app/app.go:127) with one global tbls implementation
(tbls/tbls.go:11-14), so the library drives every GPU of the node itself: hipbls_init_devices binds K contexts and
each host-buffer batch is split into K contiguous ranges (whole validators for RLC), run concurrently, with the
results written straight into the caller's arrays.

The box has one GPU, so the child process binds K = 3 contexts all on device 0: every split path runs (three ranges,
three host threads, three streams, per-context tables, caches and queues) and must return exactly what this process
returns unsplit on its single context -- statuses, aggregates, signatures and keys byte for byte.
"""
import os
import random
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
K = 3


@pytest.fixture(scope="module")
def impl():
    from charon_amd.tbls import HipBLS
    return HipBLS()


def _u8(blobs):
    return np.frombuffer(b"".join(blobs), dtype=np.uint8)


def test_three_contexts_equal_unsplit(impl, tmp_path):
    import bench
    from charon_amd.tbls import _check, _offsets
    import ctypes
    rng = random.Random(0x3D)
    # Verify: 12,288 items (3 ranges of 4,096), ~1% corrupted
    keys2 = bench.share_keys(impl, 256, "md2")
    pks, roots, sigs, bad = bench.make_c2(impl, keys2, 0, 12288)
    objs = [rng.randbytes(32) for _ in range(len(pks))]
    doms = [rng.randbytes(32) for _ in range(len(pks))]
    # RLC: 12,288 validators x 4 partials (3 ranges of 16,384), ~1% corrupted
    keys4 = bench.share_keys(impl, 512, "md4")
    rp, rs, rm, rroots, rbad = bench.make_c4(impl, keys4, "md4", 0, 12288, 12288)
    # RLC with committee roots (the batch-wide check's G1 MSM per root in every range): 2,048 validators x 4 over
    # 24 roots, ~1% corrupted, in the batch-wide mode
    cp, cs, cm, croots, cbad = bench.make_c4(impl, keys4, "md4c", 0, 2048, 2048, 24)
    # ThresholdAggregate: 3,072 validators x 3-of-5, with a few failing groups
    t_sig, t_ids, t_off, t_dvpk, t_root = [], [], [0], [], []
    for g in range(3072):
        secret = rng.randrange(1, R_ORDER)
        poly = [secret, rng.randrange(R_ORDER), rng.randrange(R_ORDER)]
        ids = rng.sample(range(1, 6), 3)
        root = rng.randbytes(32)
        shares = []
        for i in ids:
            acc = 0
            for c in reversed(poly):
                acc = (acc * i + c) % R_ORDER
            shares.append(acc.to_bytes(32, "big"))
        t_ids += ids
        t_off.append(len(t_ids))
        t_root.append(root)
        t_dvpk.append(secret.to_bytes(32, "big"))
        t_sig.append(shares)
    # sign all groups' partials in one batch
    flat_sk = [s for sh in t_sig for s in sh]
    flat_msg = [t_root[g] for g in range(3072) for _ in range(3)]
    flat_sig, st = impl.sign_batch(flat_sk, flat_msg)
    assert set(st) == {0}
    flat_sig = list(flat_sig)
    flat_sig[5] = bytes(96)          # undecodable partial in group 1
    t_ids[9] = 0                     # id 0 in group 3
    dvpks, _ = impl.secret_to_public_key_batch(t_dvpk)
    dvpks = list(dvpks)
    dvpks[7] = dvpks[8]              # wrong root key for group 7
    # Sign / SecretToPublicKey: 12,288
    s_sk = [rng.randrange(1, R_ORDER).to_bytes(32, "big") for _ in range(12288)]
    s_msg = [rng.randbytes(32) for _ in range(12288)]
    # FastAggregateVerify: 192 groups of 4 keys, every 5th over the wrong root
    fsk = [rng.randrange(1, R_ORDER).to_bytes(32, "big") for _ in range(768)]
    fpk, _ = impl.secret_to_public_key_batch(fsk)
    f_msg = [rng.randbytes(32) for _ in range(192)]
    fs, _ = impl.sign_batch(fsk, [f_msg[i // 4] for i in range(768)])
    f_sig = [impl.aggregate(fs[4 * g:4 * g + 4]) for g in range(192)]
    f_msg_used = [m if g % 5 else m[::-1] for g, m in enumerate(f_msg)]
    # Aggregate: 196,608 signatures (3 ranges of 65,536)
    good = [s for i, s in enumerate(sigs) if i not in bad]
    a_sig = (good * 17)[:196608]
    np.savez(tmp_path / "in.npz", v_pk=_u8(pks), v_msg=_u8(roots), v_sig=_u8(sigs), v_obj=_u8(objs), v_dom=_u8(doms),
             r_pk=_u8(rp), r_sig=_u8(rs), r_midx=np.array(rm, dtype=np.uint32), r_roots=_u8(rroots),
             c_pk=_u8(cp), c_sig=_u8(cs), c_midx=np.array(cm, dtype=np.uint32), c_roots=_u8(croots),
             t_sig=_u8(flat_sig), t_ids=np.array(t_ids, dtype=np.int64), t_off=np.array(t_off, dtype=np.int64),
             t_dvpk=_u8(dvpks), t_root=_u8(t_root), s_sk=_u8(s_sk), s_msg=_u8(s_msg), f_pk=_u8(fpk),
             f_off=np.arange(0, 769, 4, dtype=np.int64), f_sig=_u8(f_sig), f_msg=_u8(f_msg_used), a_sig=_u8(a_sig))
    # the unsplit results on this process's one context
    want = {}
    want["verify"] = impl.batch_verify_status(pks, roots, sigs)
    assert {i for i, s in enumerate(want["verify"]) if s} == bad
    n = len(rp)
    blob, offs = _offsets(rroots)
    st = (ctypes.c_int32 * n)()
    _check(impl.lib.hipbls_batch_verify_rlc(b"".join(rp), b"".join(rs), (ctypes.c_uint32 * n)(*rm), n, blob, offs,
                                            len(rroots), os.urandom(32), st), impl.lib)
    want["rlc"] = list(st)
    assert {i for i, s in enumerate(want["rlc"]) if s} == rbad
    want["rlc_keys"] = want["rlc"]
    from charon_amd.tbls import RLC_AUTO, RLC_BATCH
    impl.set_rlc_mode(RLC_BATCH)
    try:
        want["rlc_committee"] = impl.batch_verify_rlc_status(cp, [croots[m] for m in cm], cs)
    finally:
        impl.set_rlc_mode(RLC_AUTO)
    assert {i for i, s in enumerate(want["rlc_committee"]) if s} == cbad
    want["verify_keys"] = want["rlc"][:12288]
    groups = [dict(zip(t_ids[t_off[g]:t_off[g + 1]], flat_sig[t_off[g]:t_off[g + 1]])) for g in range(3072)]
    res = impl.batch_threshold_aggregate(groups)
    want["tagg"] = b"".join(r if isinstance(r, bytes) else bytes(96) for r in res)
    res2, vst = impl.batch_threshold_aggregate_verify(groups, dvpks, t_root)
    want["tagg_v"] = b"".join(r if isinstance(r, bytes) else bytes(96) for r in res2)
    want["tagg_vst"] = vst
    assert vst[1] == 2 and vst[3] == 5 and vst[7] == 3 and vst.count(0) == 3072 - 3
    sg, _ = impl.sign_batch(s_sk, s_msg)
    want["sign"] = b"".join(sg)
    pk_, _ = impl.secret_to_public_key_batch(s_sk)
    want["pk"] = b"".join(pk_)
    want["fav"] = impl.batch_verify_aggregate_status([(fpk[4 * g:4 * g + 4], f_sig[g], f_msg_used[g])
                                                      for g in range(192)])
    assert want["fav"] == [3 if g % 5 == 0 else 0 for g in range(192)]
    want["agg"] = impl.aggregate(a_sig)
    want["signed"] = impl.verify_signed_data_status(pks[:9000], objs[:9000], doms[:9000], sigs[:9000])
    want["queue"] = want["rlc"][:2048]
    # the split run
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tests", "multidev_child.py"),
                        str(tmp_path / "in.npz"), str(tmp_path / "out.npz"), str(K)],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    got = np.load(tmp_path / "out.npz", allow_pickle=False)
    for key in ("verify", "rlc", "rlc_keys", "rlc_committee", "verify_keys", "tagg_vst", "fav", "signed", "queue"):
        assert got[key].tolist() == list(want[key]), key
    for key in ("tagg", "tagg_v", "sign", "pk", "agg"):
        assert got[key].tobytes() == want[key], key
    # the window statistics of the split RLC call cover the whole batch; the queue's batches ran keyed
    assert got["rlc_stats"][0] >= (n + 7) // 8
    assert got["queue_keyed"][0] > 0
    assert got["streams"][0] == 4  # three contexts on device 0, one set of library streams
