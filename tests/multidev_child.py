"""Child process of tests/test_gpu_multidev.py: binds the library to K device contexts (all on device 0 when the box
has one GPU) so that every host-buffer batch is split into K ranges, runs the same calls the parent ran unsplit on
one context, and writes the results.  Usage: multidev_child.py IN.npz OUT.npz K
"""
import ctypes
import os
import sys
import threading

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def rows(a, w):
    b = a.tobytes()
    return [b[w * i:w * i + w] for i in range(len(b) // w)]


def main():
    src, dst, k = sys.argv[1], sys.argv[2], int(sys.argv[3])
    from charon_amd.tbls import HipBLS, _check, _offsets
    d = np.load(src, allow_pickle=False)
    impl = HipBLS(devices=[0] * k)
    assert impl.device_slots() == [0] * k
    out = {}
    pks, msgs, sigs = rows(d["v_pk"], 48), rows(d["v_msg"], 32), rows(d["v_sig"], 96)
    out["verify"] = np.array(impl.batch_verify_status(pks, msgs, sigs), dtype=np.int32)
    # RLC with a validator-shaped message index (4 partials per root)
    rp, rs, rm = rows(d["r_pk"], 48), rows(d["r_sig"], 96), d["r_midx"].astype(np.uint32)
    roots = rows(d["r_roots"], 32)
    n = len(rp)
    blob, offs = _offsets(roots)
    st = (ctypes.c_int32 * n)()
    idx = (ctypes.c_uint32 * n)(*rm.tolist())
    _check(impl.lib.hipbls_batch_verify_rlc(b"".join(rp), b"".join(rs), idx, n, blob, offs, len(roots), os.urandom(32),
                                            st), impl.lib)
    out["rlc"] = np.array(list(st), dtype=np.int32)
    w, wf, fb = impl.rlc_stats()
    out["rlc_stats"] = np.array([w, wf, fb], dtype=np.int64)
    table = list(dict.fromkeys(rp))
    assert set(impl.load_pubshares(table)) == {0}
    pos = {p: j for j, p in enumerate(table)}
    kidx = (ctypes.c_uint32 * n)(*[pos[p] for p in rp])
    st2 = (ctypes.c_int32 * n)()
    _check(impl.lib.hipbls_batch_verify_rlc_keys(kidx, b"".join(rs), idx, n, blob, offs, len(roots), os.urandom(32),
                                                 st2), impl.lib)
    out["rlc_keys"] = np.array(list(st2), dtype=np.int32)
    # committee roots in the batch-wide mode: each context's range takes the G1 MSM per root
    from charon_amd.tbls import RLC_AUTO, RLC_BATCH
    cp, cs, cm, croots = rows(d["c_pk"], 48), rows(d["c_sig"], 96), d["c_midx"].tolist(), rows(d["c_roots"], 32)
    impl.set_rlc_mode(RLC_BATCH)
    out["rlc_committee"] = np.array(impl.batch_verify_rlc_status(cp, [croots[m] for m in cm], cs), dtype=np.int32)
    impl.set_rlc_mode(RLC_AUTO)
    m12 = [roots[m] for m in rm[:12288].tolist()]
    out["verify_keys"] = np.array(impl.batch_verify_keys_status([pos[p] for p in rp[:12288]], m12, rs[:12288]),
                                  dtype=np.int32)
    # ThresholdAggregate (+ the fused aggregate Verify)
    tsig, tid, toff = rows(d["t_sig"], 96), d["t_ids"].tolist(), d["t_off"].tolist()
    groups = [dict(zip(tid[toff[g]:toff[g + 1]], tsig[toff[g]:toff[g + 1]])) for g in range(len(toff) - 1)]
    res = impl.batch_threshold_aggregate(groups)
    out["tagg"] = np.frombuffer(b"".join(r if isinstance(r, bytes) else bytes(96) for r in res), dtype=np.uint8)
    res2, vst = impl.batch_threshold_aggregate_verify(groups, rows(d["t_dvpk"], 48), rows(d["t_root"], 32))
    out["tagg_v"] = np.frombuffer(b"".join(r if isinstance(r, bytes) else bytes(96) for r in res2), dtype=np.uint8)
    out["tagg_vst"] = np.array(vst, dtype=np.int32)
    # Sign / SecretToPublicKey
    sks = rows(d["s_sk"], 32)
    s_sigs, _ = impl.sign_batch(sks, rows(d["s_msg"], 32))
    out["sign"] = np.frombuffer(b"".join(s_sigs), dtype=np.uint8)
    s_pks, _ = impl.secret_to_public_key_batch(sks)
    out["pk"] = np.frombuffer(b"".join(s_pks), dtype=np.uint8)
    # FastAggregateVerify groups
    fpk, foff, fsig, fmsg = rows(d["f_pk"], 48), d["f_off"].tolist(), rows(d["f_sig"], 96), rows(d["f_msg"], 32)
    fg = [(fpk[foff[g]:foff[g + 1]], fsig[g], fmsg[g]) for g in range(len(fsig))]
    out["fav"] = np.array(impl.batch_verify_aggregate_status(fg), dtype=np.int32)
    # Aggregate over ranges
    out["agg"] = np.frombuffer(impl.aggregate(rows(d["a_sig"], 96)), dtype=np.uint8)
    # eth2util/signing.Verify
    out["signed"] = np.array(impl.verify_signed_data_status(pks[:9000], rows(d["v_obj"], 32)[:9000],
                                                            rows(d["v_dom"], 32)[:9000], sigs[:9000]), dtype=np.int32)
    # the submission queues: n = 1 calls from 32 threads over the RLC items (keys in the table, 4 partials per
    # root), routed by message hash
    qn = 2048
    got = [None] * qn

    def worker(t):
        for i in range(t, qn, 32):
            got[i] = impl.verify_queued(rp[i], m12[i], rs[i])

    th = [threading.Thread(target=worker, args=(t,)) for t in range(32)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    out["queue"] = np.array(got, dtype=np.int32)
    out["queue_keyed"] = np.array([impl.queue_keyed_batches()], dtype=np.int64)
    # K contexts on one device share the device's library streams: at most 4, not 4 K
    out["streams"] = np.array([impl.lib.hipbls_device_streams(0)], dtype=np.int64)
    np.savez(dst, **out)
    print("multidev child: %d contexts ok" % k)


if __name__ == "__main__":
    main()
