"""GPU tests added in round 5 (VERDICT r04 "Next round" 1).

The round-4 abort (HSA_STATUS_ERROR_OUT_OF_RESOURCES when a high-priority stream ran the library's kernels beside a
C5 step) came from the scratch arithmetic measured in profiles/r05/r05_scratch_probe.txt and
r05_scratch_layout.txt: every hardware queue that dispatches a kernel holds a block of (private segment) x 64 x 32 x
256 CUs from one 32 GiB region per device, placed first fit; queues grown in stages leave holes, and a priority stream
is a queue of its own.  The library now reserves its four queues' blocks at init, refuses a device where they do not
fit, and runs a *_device call on a priority stream on its own library stream instead (StreamJoin).  Here:

* the budget the library computed at init equals the code objects' arithmetic (hipbls_scratch_budget);
* a C5-sized RLC call on a HIGH-priority caller stream beside a FastAggregateVerify on a LOW-priority one (two
  hardware queues the library does not hold): the statuses equal the construction, both calls were joined to the
  library stream, and the device's free memory does not drop by a scratch block (6.1 GiB);
* the submission queue's worker polls a batch in flight from its expected end on, not every 20 us from its start.
"""
import ctypes
import os

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "charon_amd", "libhipbls.so")
V = 262144  # C4/C5 node batch: 262,144 validators x 4 partials


@pytest.fixture(scope="module")
def impl():
    from charon_amd.tbls import HipBLS
    return HipBLS()


def _budget(impl, dev=0):
    pl, pq, lim = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
    q = ctypes.c_uint32()
    assert impl.lib.hipbls_scratch_budget(dev, ctypes.byref(pl), ctypes.byref(pq), ctypes.byref(lim),
                                          ctypes.byref(q)) == 0
    return pl.value, pq.value, lim.value, q.value


def _joins(impl):
    n = ctypes.c_uint64()
    assert impl.lib.hipbls_stream_joins(ctypes.byref(n)) == 0
    return n.value


def test_scratch_budget_matches_code_objects(impl):
    from charon_amd import codeobj
    impl.batch_verify_status([b"\xc0" + bytes(47)], [b"x"], [b"\xc0" + bytes(95)])  # binds the device
    per_lane, per_queue, limit, queues = _budget(impl)
    deepest = max(r[1] for r in codeobj.resource_table(LIB) if r[0] != "k_scratch_reserve")
    assert per_lane == deepest
    assert per_queue == -(-per_lane * codeobj.WAVE_SLOTS // codeobj.BLOCK_ALIGN) * codeobj.BLOCK_ALIGN
    assert limit == codeobj.SCRATCH_REGION  # 32 GiB on MI355X
    assert queues == int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))
    assert impl.lib.hipbls_device_streams(0) == 4
    # the four library queues plus one more of the same depth fit the region (the build's budget)
    assert 5 * per_queue <= limit
    print("scratch: %d B/lane, %.2f GiB per queue, limit %.1f GiB" % (per_lane, per_queue / 2**30, limit / 2**30))


def test_priority_streams_beside_c5_run_on_library_queues(impl):
    import torch

    import bench
    from oracle import bls12381 as bls
    keys4 = bench.share_keys(impl, 4096, "c4")
    pks, sigs, midx, roots, bad = bench.make_c4(impl, keys4, "c4i", 0, V, V, 0)
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
    d_spk2 = torch.cat([u8(sync_pks), u8(sync_pks)])
    d_ssig, d_smsg = u8([sync_agg, sync_agg]), u8([sync_root, sync_root[::-1]])
    d_skoff = torch.tensor([0, 512, 1024], dtype=torch.int64).to(dev)
    d_smoff = torch.tensor([0, 32, 64], dtype=torch.int64).to(dev)
    d_sst = torch.full((2,), -7, dtype=torch.int32, device=dev)
    lib = impl.lib

    def run(s_rlc, s_fav):
        d_st.fill_(-7)
        d_sst.fill_(-7)
        torch.cuda.synchronize(dev)
        assert lib.hipbls_verify_aggregate_batch_device(d_spk2.data_ptr(), 1024, d_skoff.data_ptr(), 2,
                                                        d_ssig.data_ptr(), d_smsg.data_ptr(), d_smoff.data_ptr(),
                                                        d_sst.data_ptr(), ctypes.c_void_p(s_fav.cuda_stream)) == 0
        assert lib.hipbls_batch_verify_rlc_device(d_pk.data_ptr(), d_sig.data_ptr(), d_midx.data_ptr(), n,
                                                  d_msg.data_ptr(), d_off.data_ptr(), len(roots), os.urandom(32),
                                                  d_st.data_ptr(), ctypes.c_void_p(s_rlc.cuda_stream)) == 0
        # the caller's streams are ordered after the calls: reading on them sees the results
        with torch.cuda.stream(s_rlc):
            st = d_st.cpu()
        with torch.cuda.stream(s_fav):
            sst = d_sst.cpu()
        torch.cuda.synchronize(dev)
        assert {i for i, s in enumerate(st.tolist()) if s != 0} == bad
        assert sst.tolist() == [0, 3]

    # warm-up on normal-priority streams: workspaces allocated, no join
    j0 = _joins(impl)
    run(torch.cuda.Stream(dev), torch.cuda.Stream(dev))
    assert _joins(impl) == j0
    torch.cuda.synchronize(dev)
    free0, _ = torch.cuda.mem_get_info(dev)
    hi = torch.cuda.Stream(dev, priority=-1)
    # torch clamps priorities to [-1, 0]: the least priority (+1 on this runtime, its own hardware queue as well,
    # profiles/r05/r05_scratch_probe.txt) comes from HIP directly
    hip = ctypes.CDLL("libamdhip64.so")
    least, greatest = ctypes.c_int(), ctypes.c_int()
    assert hip.hipDeviceGetStreamPriorityRange(ctypes.byref(least), ctypes.byref(greatest)) == 0
    raw = ctypes.c_void_p()
    assert hip.hipStreamCreateWithPriority(ctypes.byref(raw), 1, least) == 0  # hipStreamNonBlocking
    lo = torch.cuda.ExternalStream(raw.value, device=dev)
    assert least.value != 0 and hi.priority != 0
    run(hi, lo)
    free1, _ = torch.cuda.mem_get_info(dev)
    joined = _joins(impl) - j0
    assert joined == 2
    _, per_queue, _, _ = _budget(impl)
    drop = free0 - free1
    print("priority streams: %d calls joined, free memory drop %.3f GiB (a queue's block: %.2f GiB)"
          % (joined, drop / 2**30, per_queue / 2**30))
    assert drop < per_queue // 4
    bls.verify_aggregate(sync_pks, sync_agg, sync_root)


def test_queue_worker_polls_from_expected_end(impl):
    import bench
    pks, roots, sigs, bad = bench.make_c2(impl, bench.share_keys(impl, 64, "c2q"), 0, 64)
    st = impl.batch_verify_status(pks, roots, sigs)
    assert {i for i, s in enumerate(st) if s} == bad
    w0, b0 = ctypes.c_uint64(), ctypes.c_uint64()
    impl.verify_queued(pks[0], roots[0], sigs[0])  # starts the worker; learns the n = 1 batch time
    assert impl.lib.hipbls_queue_worker_stats(ctypes.byref(w0), ctypes.byref(b0)) == 0
    for j in range(1, 33):
        assert impl.verify_queued(pks[j], roots[j], sigs[j]) == st[j]
    w1, b1 = ctypes.c_uint64(), ctypes.c_uint64()
    assert impl.lib.hipbls_queue_worker_stats(ctypes.byref(w1), ctypes.byref(b1)) == 0
    per_batch = (w1.value - w0.value) / max(1, b1.value - b0.value)
    print("queue worker: %.1f completion polls per n = 1 batch" % per_batch)
    # a ~12 ms batch polled every 20 us from its launch would take ~600 polls
    assert per_batch < 250


def test_host_sigagg_calls_from_two_threads_overlap_and_match(impl):
    """The host-buffer sigagg call holds the context lock only while it enqueues (two slots), so two
    threads' calls run side by side on the GPU -- what two goroutines with consecutive sigagg duties do.  Every result
    of 6 concurrent calls (3 per thread, different validator sets, two with a bad partial) equals the same call made
    alone, and the aggregates equal Sign(secret)."""
    import threading

    from tests.test_gpu_r04 import _make_c3
    sets = []
    for k in range(6):
        groups, secrets_, roots, dv_pks, _ = _make_c3(impl, G=1200, seed=0x5A + k)
        gmaps = [dict(g) for g in groups]
        if k in (1, 4):  # one partial of group 7 replaced by another group's: the aggregate fails Verify
            key = next(iter(gmaps[7]))
            gmaps[7][key] = groups[8][0][1]
        sets.append((gmaps, dv_pks, roots, secrets_))
    alone = [impl.batch_threshold_aggregate_verify(g, p, r) for g, p, r, _ in sets]
    got = [None] * 6

    def worker(ks):
        for k in ks:
            g, p, r, _ = sets[k]
            got[k] = impl.batch_threshold_aggregate_verify(g, p, r)

    th = [threading.Thread(target=worker, args=(ks,)) for ks in ((0, 2, 4), (1, 3, 5))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert got == alone
    for k, (g, p, r, secrets_) in enumerate(sets):
        aggs, vst = got[k]
        want, st = impl.sign_batch([s.to_bytes(32, "big") for s in secrets_], r)
        assert set(st) == {0}
        for j in range(len(g)):
            if k in (1, 4) and j == 7:
                assert vst[j] == 3  # HIPBLS_ERR_VERIFY
            else:
                assert vst[j] == 0 and aggs[j] == want[j], (k, j)


def test_raced_small_batches_across_workspace_growth(impl):
    """Batches of at most 8 items run as replicas that race (verify_lat.hip bls_race) through words at the tail of
    the Verify workspace.  The workspace moves every time a larger batch grows it, so small batches alternate with
    larger ones here: every workspace address the sequence produces carries raced calls, and their statuses equal
    the same items' statuses from one large call, with the race off (replicas = 1) and on (8).  Round 5's first race
    build built the word's address from two sign-extended halves and read a wild address for half of all buffers."""
    import bench
    N = 20000
    pks, roots, sigs, bad = bench.make_c2(impl, bench.share_keys(impl, 4096, "c2race"), 0, N)
    want = impl.batch_verify_status(pks, roots, sigs)
    assert {i for i, s in enumerate(want) if s} == bad
    bad_l = sorted(bad)
    good_l = [i for i in range(N) if i not in bad][:64]
    small = [[bad_l[0]], [good_l[0]], [good_l[1], bad_l[1], good_l[2]], good_l[3:11], [bad_l[2]] + good_l[11:18]]
    prev = impl.lib.hipbls_set_latency_replicas(8)
    try:
        for grow in (1, 700, 3000, 9000, N):
            lo = (grow * 7) % max(1, N - grow)
            got = impl.batch_verify_status(pks[lo:lo + grow], roots[lo:lo + grow], sigs[lo:lo + grow])
            assert got == want[lo:lo + grow]
            for reps in (8, 1, 8):
                impl.lib.hipbls_set_latency_replicas(reps)
                for idx in small:
                    got = impl.batch_verify_status([pks[i] for i in idx], [roots[i] for i in idx],
                                                   [sigs[i] for i in idx])
                    assert got == [want[i] for i in idx], (grow, reps, idx)
    finally:
        impl.lib.hipbls_set_latency_replicas(prev)


def test_sixteen_lane_check_takes_small_batches(impl):
    """AUTO runs batches of at most four items on the sixteen-lane check (verify_hex.hip), five to eight on the octet
    check; the forced OCTETS mode keeps eight lanes.  Statuses agree everywhere (the layout-parity tests in
    tests/test_gpu_lg2.py compare the modes on mixed batches and the fixtures)."""
    import bench
    from charon_amd.tbls import PAIR_AUTO, PAIR_OCTETS

    def launches(name):
        a, c = ctypes.c_double(), ctypes.c_uint64()
        impl.lib.hipbls_kernel_timing(name, ctypes.byref(a), ctypes.byref(c))
        return c.value

    pks, roots, sigs, bad = bench.make_c2(impl, bench.share_keys(impl, 64, "c2hex"), 0, 64)
    want = impl.batch_verify_status(pks, roots, sigs)
    impl.lib.hipbls_set_timing(1)
    try:
        for mode, n, lq16, lq8 in ((PAIR_AUTO, 1, 1, 0), (PAIR_AUTO, 4, 1, 0), (PAIR_AUTO, 5, 0, 1),
                                   (PAIR_OCTETS, 3, 0, 1)):
            impl.set_pair_mode(mode)
            b16, b8 = launches(b"verify_pair_lq16"), launches(b"verify_pair_lq8")
            lo = 7 * n
            assert impl.batch_verify_status(pks[lo:lo + n], roots[lo:lo + n], sigs[lo:lo + n]) == want[lo:lo + n]
            assert (launches(b"verify_pair_lq16") - b16, launches(b"verify_pair_lq8") - b8) == (lq16, lq8), (mode, n)
    finally:
        impl.set_pair_mode(PAIR_AUTO)
        impl.lib.hipbls_set_timing(0)


def test_raced_calls_from_many_threads(impl):
    """Raced small batches from eight threads at once, direct batch calls (the context's workspace) mixed with queued
    n = 1 calls (the queue's slot workspaces): every call's race words and epochs are its own, so every status equals
    the one large call's."""
    import random
    import threading

    import bench
    N = 512
    pks, roots, sigs, bad = bench.make_c2(impl, bench.share_keys(impl, 256, "c2thr"), 0, N)
    want = impl.batch_verify_status(pks, roots, sigs)
    errors = []

    def worker(seed):
        rng = random.Random(seed)
        try:
            for _ in range(12):
                n = rng.randint(1, 8)
                lo = rng.randrange(0, N - n)
                if rng.random() < 0.5:
                    got = impl.batch_verify_status(pks[lo:lo + n], roots[lo:lo + n], sigs[lo:lo + n])
                    if got != want[lo:lo + n]:
                        errors.append(("batch", lo, n, got))
                else:
                    got = impl.verify_queued(pks[lo], roots[lo], sigs[lo])
                    if got != want[lo]:
                        errors.append(("queued", lo, got))
        except Exception as e:  # noqa: BLE001 -- reported by the assertion below
            errors.append(("exception", repr(e)))

    th = [threading.Thread(target=worker, args=(k,)) for k in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors[:5]


def test_fav_octet_and_sixteen_lane_layouts_match_fav_batch(impl):
    """FastAggregateVerify for at most 16 groups runs on the drop-in path's layouts (verify_lat.hip k_fav_prep8, then
    verify_hex.hip k_fav_pair_lq16); PAIR_SINGLE keeps k_fav_batch.  Same statuses on: honest groups, a wrong message,
    a signature / key encoding error, empty, identity key, keys summing to infinity (P, -P), small-order signatures
    (alone and with a bad key: the signature's error wins), a small-order key, a 512-key sync-committee group, and a
    17-group batch (over the limit: k_fav_batch in AUTO too)."""
    import json
    import random

    from charon_amd.tbls import PAIR_AUTO, PAIR_SINGLE

    def launches(name):
        a, c = ctypes.c_double(), ctypes.c_uint64()
        impl.lib.hipbls_kernel_timing(name, ctypes.byref(a), ctypes.byref(c))
        return c.value

    with open(os.path.join(ROOT, "tests", "golden", "fixtures.json")) as f:
        so = json.load(f)["small_order"]
    h = bytes.fromhex
    rng = random.Random(55)
    sks = [rng.randrange(1, 2 ** 254).to_bytes(32, "big") for _ in range(512)]
    pks, st = impl.secret_to_public_key_batch(sks)
    assert set(st) == {0}
    msg = b"sync committee root".ljust(32, b"\0")
    sigs, _ = impl.sign_batch(sks, [msg] * 512)
    agg3, agg512 = impl.aggregate(sigs[:3]), impl.aggregate(sigs)
    bad_sig = bytearray(agg3)
    bad_sig[0] &= 0x7F
    neg0 = bytearray(pks[0])
    neg0[0] ^= 0x20  # the sign flag: -P
    small_sig, small_pk = h(so["verify"][0]["sig"]), h(so["verify"][16]["pk"])
    groups = [
        (pks[:3], agg3, msg),                        # 0
        (pks[:3], agg3, msg[::-1]),                  # 3
        (pks[:3], bytes(bad_sig), msg),              # 2
        ([pks[0], bytes(48), pks[2]], agg3, msg),    # 1
        ([], agg3, msg),                             # 3
        (pks[:3] + [bytes([0xC0]) + bytes(47)], agg3, msg),  # 3
        ([pks[0], bytes(neg0)], agg3, msg),          # 3: the key sum is the identity
        (pks[:3], small_sig, msg),                   # 2
        ([pks[0], bytes(48)], small_sig, msg),       # 2: the signature's membership error before the key's
        (pks[:3] + [small_pk], agg3, msg),           # 1
        (pks, agg512, msg),                          # 0
        (pks[:511], agg512, msg),                    # 3
    ]
    want = [0, 3, 2, 1, 3, 3, 3, 2, 2, 1, 0, 3]
    impl.lib.hipbls_set_timing(1)
    try:
        for mode, batch, hexl in ((PAIR_SINGLE, groups, 0), (PAIR_AUTO, groups, 1), (PAIR_AUTO, groups * 2, 0)):
            impl.set_pair_mode(mode)
            before = launches(b"fav_lq16")
            assert impl.batch_verify_aggregate_status(batch) == want * (len(batch) // len(groups)), (mode, len(batch))
            assert launches(b"fav_lq16") - before == hexl, (mode, len(batch))
        impl.set_pair_mode(PAIR_AUTO)
        for g, w in zip(groups, want):  # one group per call, as the sync-committee duty sends it
            assert impl.batch_verify_aggregate_status([g]) == [w]
    finally:
        impl.set_pair_mode(PAIR_AUTO)
        impl.lib.hipbls_set_timing(0)


@pytest.mark.parametrize("rlc_mode", ["windows", "batch"])
def test_c5_partial_wave_windows_go_to_item_checks(impl, rlc_mode):
    """C5's 131,088 windows are 2 x 1,024.1 waves at one lane per window on 1,024 SIMDs: the two partial last waves'
    windows (8 per sub-batch) skip the window check and their items go straight to the per-item checks
    (kernels.h k_rlc_window wdirect), on the windows path and on a failed batch-wide check's windows.  Bitmap ==
    construction; the statistics count those items as re-checked, not their windows as failed."""
    import bench
    from charon_amd.tbls import RLC_BATCH, RLC_WINDOWS
    keys4 = bench.share_keys(impl, 4096, "c4")
    pks, sigs, midx, roots, bad = bench.make_c4(impl, keys4, "c4i", 0, V, V, 0)
    ppks, psigs, pmidx, proots, pbad = bench.make_c4(impl, bench.share_keys(impl, 128, "c5p"), "c5p", 0, 32, 32)
    base, off = len(pks), len(roots)
    pks, sigs, roots = pks + ppks, sigs + psigs, roots + proots
    midx = midx + [m + off for m in pmidx]
    bad = bad | {base + i for i in pbad}
    prev = impl.set_rlc_mode({"windows": RLC_WINDOWS, "batch": RLC_BATCH}[rlc_mode])
    try:
        st = impl.batch_verify_rlc_status(pks, [roots[m] for m in midx], sigs, seed=bytes(range(32)))
        assert {i for i, s in enumerate(st) if s != 0} == bad
        w, wf, fb = impl.rlc_stats()
        assert w == (len(pks) + 7) // 8
        assert fb >= wf + 96  # >= 1 item per failed window + the direct windows' (16 windows, 128 items, few invalid)
    finally:
        impl.set_rlc_mode(prev)
