#!/usr/bin/env python3
"""Benchmark: charon's BLS hot path on MI355X (BASELINE.json metric).

  python bench.py --gpus N --steps K --warmup W
  (N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...)

Step = one pass of the hot path over one batch: tbls.Verify of the configs[1] workload (C2:
65,536 partial signatures over distinct 32-byte signing roots, 1% corrupted) through the C-ABI
device entry point, inputs already resident in HBM.  Multi-GPU is weak scaling: every rank owns its
own validator-index shard of the same size (no data-path collective).  Threshold aggregation (C3:
10,000 validators x 7-of-10 + Verify of each aggregate) is timed after the main loop and reported as
an extra field.  Rank 0 prints ONE JSON line.
"""
import argparse
import ctypes
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

SEED = 0x636861726F6E
R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
METRIC = "verified BLS partial sigs/sec (node) + threshold aggregates/sec, 1/2/4/8 GPU"

# Algorithmic work per honest Verify of a 32-byte root, in Fp-multiplication equivalents
# (one 381-bit Montgomery product, fp_mul or fp_sqr, = 12x12 CIOS = 300 32x32->64 multiply-adds).
# Counted by the instrumented host build of the same kernels (tests/test_work_counts.py keeps
# this in sync).  See DESIGN.md "Roofline".
FPMUL_PER_VERIFY = 28880
MADS_PER_FPMUL = 300
# RLC BatchVerify stages (charon_amd/csrc/rlc.h), same unit and source (tests/test_work_counts.py):
# stage 1 per item, stage 2 per distinct message, stage 3 per window of 8 with 2 messages (one per
# 4-partial validator) or 1 message (committee root), stage 4 per item re-checked after a failed window.
RLC_FPMUL = {"item": 5832, "hash": 6689, "window_2msg": 24842, "window_1msg": 19962, "fallback": 20004}
# gfx950 32x32->64 integer multiply-add peak (v_mad_u64_u32): 256 CU x 4 SIMD x 32 lanes x 2.4 GHz
# at half rate (measured: profiles/r01_mad_probe.txt) = 39.3e12 MAD/s.
MAD_PEAK_T = 39.3


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--n", type=int, default=65536, help="verifies per GPU per step (C2: 65,536)")
    ap.add_argument("--tagg-groups", type=int, default=10000, help="C3 validators per GPU (0 = skip)")
    ap.add_argument("--tagg-steps", type=int, default=2)
    ap.add_argument("--cpu-sample", type=int, default=4096,
                    help="C2 items verified by the C++ CPU baseline, one thread per core (0 = skip)")
    ap.add_argument("--rlc-validators", type=int, default=32768,
                    help="C4 validators per GPU (x4 partials; 32,768 = the 1M-partial node batch / 8 GPUs; 0 = skip)")
    ap.add_argument("--rlc-steps", type=int, default=3)
    ap.add_argument("--c5", type=int, default=1, help="time the C5 full-slot mix (0 = skip)")
    ap.add_argument("--keys", type=int, default=1, help="also time C2 / C4 with the resident pubshare table (0 = skip)")
    ap.add_argument("--rlc-big-validators", type=int, default=262144,
                    help="also time one GPU on the whole C4 node batch (262,144 x 4 = 1M partials; 0 = skip)")
    return ap.parse_args()


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def make_c2(impl, n, rng):
    """n partial signatures by 4,096 share keys over distinct roots; 1% corrupted at seeded spots."""
    nkeys = min(4096, n)
    sks = [rng.randrange(1, R_ORDER).to_bytes(32, "big") for _ in range(nkeys)]
    pks, st = impl.secret_to_public_key_batch(sks)
    assert set(st) == {0}
    roots = [rng.randbytes(32) for _ in range(n)]
    owner = [i % nkeys for i in range(n)]
    sigs, st = impl.sign_batch([sks[o] for o in owner], roots)
    assert set(st) == {0}
    pk_list = [pks[o] for o in owner]
    bad = sorted(rng.sample(range(n), max(1, n // 100)))
    for j, i in enumerate(bad):
        kind = j % 3
        if kind == 0:    # wrong root
            roots[i] = bytes(32 - len(roots[i][:1])) + roots[i][:1]
        elif kind == 1:  # swapped share (another validator's pubshare)
            pk_list[i] = pks[(owner[i] + 1) % nkeys]
        else:            # flipped bit in the signature
            s = bytearray(sigs[i])
            s[40] ^= 0x04
            sigs[i] = bytes(s)
    return pk_list, roots, sigs, set(bad)


def make_c3(impl, groups, rng, t=7, n=10):
    """groups DVs, each split t-of-n; a random t-subset of partials per DV; DV pubkeys + one root each."""
    secrets_ = [rng.randrange(1, R_ORDER) for _ in range(groups)]
    roots = [rng.randbytes(32) for _ in range(groups)]
    part_sks, part_msgs, part_ids, offs = [], [], [], [0]
    for g in range(groups):
        poly = [secrets_[g]] + [rng.randrange(R_ORDER) for _ in range(t - 1)]
        ids = sorted(rng.sample(range(1, n + 1), t))
        for i in ids:
            acc = 0
            for c in reversed(poly):
                acc = (acc * i + c) % R_ORDER
            part_sks.append(acc.to_bytes(32, "big"))
            part_msgs.append(roots[g])
            part_ids.append(i)
        offs.append(len(part_ids))
    psigs, st = impl.sign_batch(part_sks, part_msgs)
    assert set(st) == {0}
    dv_pks, st = impl.secret_to_public_key_batch([s.to_bytes(32, "big") for s in secrets_])
    assert set(st) == {0}
    return psigs, part_ids, offs, dv_pks, roots


def make_c4(impl, n_dv, rng, shared_roots=0, shares=4, nkeys=4096):
    """C4 shard: n_dv validators x `shares` partials, items grouped by validator.  One root per
    validator (variant i) or `shared_roots` committee roots (variant ii).  1% corrupted."""
    n = n_dv * shares
    sks = [rng.randrange(1, R_ORDER).to_bytes(32, "big") for _ in range(nkeys)]
    keys, st = impl.secret_to_public_key_batch(sks)
    assert set(st) == {0}
    if shared_roots:
        roots = [rng.randbytes(32) for _ in range(shared_roots)]
        dv_root = [d * shared_roots // n_dv for d in range(n_dv)]  # contiguous committees
    else:
        roots = [rng.randbytes(32) for _ in range(n_dv)]
        dv_root = list(range(n_dv))
    owner = [rng.randrange(nkeys) for _ in range(n)]
    midx = [dv_root[i // shares] for i in range(n)]
    sigs, st = impl.sign_batch([sks[o] for o in owner], [roots[m] for m in midx])
    assert set(st) == {0}
    pks = [keys[o] for o in owner]
    bad = sorted(rng.sample(range(n), max(1, n // 100)))
    for j, i in enumerate(bad):
        if j % 2 == 0:  # swapped share
            pks[i] = keys[(owner[i] + 1) % nkeys]
        else:           # flipped bit in the signature
            s = bytearray(sigs[i])
            s[40] ^= 0x04
            sigs[i] = bytes(s)
    return pks, sigs, midx, roots, set(bad)


def traffic_from_pmc(path=os.path.join(ROOT, "profiles", "r01_pmc_verify.json")):
    """HBM bytes per k_verify_fused launch from the committed rocprofv3 PMC passes of this build
    (FETCH_SIZE + WRITE_SIZE, scripts/pmc_summary.py); None when absent.  Almost all of it is
    scratch (register-spill) traffic, ~8000x the 188 B/verify of algorithmic input."""
    try:
        with open(path) as f:
            return json.load(f).get("hbm_bytes_per_launch_raw")
    except (OSError, ValueError):
        return None


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_threads():
    """One thread per host core this job may use: the box exports OMP_NUM_THREADS = its CPU share."""
    n = os.cpu_count() or 1
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        n = min(n, int(env))
    return n


def cpu_baseline(impl, c2, n_sample, rng):
    """SURVEY.md §8d(2) / BASELINE.md: the repo's C++ restatement of the same per-item operations
    (tests/native/cpu_baseline.cpp over charon_amd/csrc/ops.h, -O3, 6 x 64-bit Montgomery product), one
    thread per host core, timed on this box.  kind 'port' -- NOT herumi (no Go toolchain or herumi module
    here).  Two samples: (1) n_sample C2 items (the bench's own inputs) -> verifies/s, the `value`; (2) the
    C1 workload (BASELINE configs[0]): 250 DVs x 4-of-6 -> 1,000 partial Verify + 250 ThresholdAggregate +
    250 Verify of the aggregates, inputs made by the GPU engine, statuses checked."""
    from tests.hostlib import cpu_baseline_lib
    cb = cpu_baseline_lib()
    threads = cpu_threads()
    pks, roots, sigs, bad = c2
    n = min(n_sample, len(pks))
    offs = (ctypes.c_uint64 * (n + 1))(*[32 * i for i in range(n + 1)])
    st = (ctypes.c_int32 * n)()
    dt = cb.cb_verify_batch(b"".join(pks[:n]), b"".join(roots[:n]), offs, b"".join(sigs[:n]), n, st, threads)
    assert {i for i in range(n) if st[i] != 0} == {i for i in bad if i < n}, "CPU baseline bitmap mismatch"
    # C1: 250 DVs x 4-of-6
    G, t, nsh = 250, 4, 6
    secrets_ = [rng.randrange(1, R_ORDER) for _ in range(G)]
    droots = [rng.randbytes(32) for _ in range(G)]
    psks, pmsg, pids, poffs = [], [], [], [0]
    for g in range(G):
        poly = [secrets_[g]] + [rng.randrange(R_ORDER) for _ in range(t - 1)]
        for i in sorted(rng.sample(range(1, nsh + 1), t)):
            acc = 0
            for c in reversed(poly):
                acc = (acc * i + c) % R_ORDER
            psks.append(acc.to_bytes(32, "big"))
            pmsg.append(droots[g])
            pids.append(i)
        poffs.append(len(pids))
    ppks, _ = impl.secret_to_public_key_batch(psks)
    psig, _ = impl.sign_batch(psks, pmsg)
    dpk, _ = impl.secret_to_public_key_batch([s.to_bytes(32, "big") for s in secrets_])
    np_ = len(psks)
    o1 = (ctypes.c_uint64 * (np_ + 1))(*[32 * i for i in range(np_ + 1)])
    s1 = (ctypes.c_int32 * np_)()
    t_ver = cb.cb_verify_batch(b"".join(ppks), b"".join(pmsg), o1, b"".join(psig), np_, s1, threads)
    ids = (ctypes.c_int64 * np_)(*pids)
    go = (ctypes.c_uint64 * (G + 1))(*poffs)
    agg = ctypes.create_string_buffer(96 * G)
    s2 = (ctypes.c_int32 * G)()
    t_agg = cb.cb_threshold_aggregate_batch(b"".join(psig), ids, go, G, agg, s2, threads)
    aggs = [agg.raw[96 * g:96 * g + 96] for g in range(G)]
    o3 = (ctypes.c_uint64 * (G + 1))(*[32 * i for i in range(G + 1)])
    s3 = (ctypes.c_int32 * G)()
    t_aver = cb.cb_verify_batch(b"".join(dpk), b"".join(droots), o3, b"".join(aggs), G, s3, threads)
    assert set(s1) == {0} and set(s2) == {0} and set(s3) == {0}, "CPU baseline C1 statuses"
    gpu_aggs = impl.batch_threshold_aggregate([dict(zip(pids[poffs[g]:poffs[g + 1]], psig[poffs[g]:poffs[g + 1]]))
                                               for g in range(G)])
    assert gpu_aggs == aggs, "CPU and GPU threshold aggregates differ"
    c1 = t_ver + t_agg + t_aver
    return {"value": round(n / dt, 1), "unit": "verified partial sigs/s", "cores": threads, "kind": "port",
            "label": "cpu-restatement, not herumi",
            "cpu_model": _cpu_model(),
            "sample": "%d C2 items (the bench's own 32-byte-root inputs, 1%% corrupted) through "
                      "tests/native/cpu_baseline.cpp (charon_amd/csrc/ops.h compiled -O3 for x86-64, 6x64-bit "
                      "Montgomery product), %d threads; herumi/Go absent on the box (SURVEY.md 8c)" % (n, threads),
            "c1_workload": {"config": "BASELINE configs[0]: 250 DVs x 4-of-6: 1,000 Verify + 250 ThresholdAggregate "
                                      "+ 250 Verify of the aggregates",
                            "seconds": round(c1, 4), "verify_s": round(t_ver, 4), "threshold_aggregate_s": round(t_agg, 4),
                            "aggregate_verify_s": round(t_aver, 4),
                            "verified_partial_sigs_per_s": round(np_ / t_ver, 1),
                            "threshold_aggregates_per_s": round(G / t_agg, 1)}}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:  # "nccl" is RCCL on ROCm
        dist.init_process_group(backend="nccl", device_id=dev)

    from charon_amd.shard import gather_bitmaps, pack_bitmap, unpack_bitmap
    from charon_amd.tbls import HipBLS, load_library
    impl = HipBLS(device=local)
    lib = load_library()
    lib.hipbls_set_timing(1)  # per-kernel HIP events for the roofline (off by default in the library)

    rng = random.Random(SEED * 1000003 + rank)  # validator-index shard of this rank
    t0 = time.time()
    pks, roots, sigs, bad = make_c2(impl, args.n, rng)
    log("rank %d: C2 data (%d items) in %.1fs" % (rank, args.n, time.time() - t0))

    n = args.n
    d_pk = torch.frombuffer(bytearray(b"".join(pks)), dtype=torch.uint8).to(dev)
    d_sig = torch.frombuffer(bytearray(b"".join(sigs)), dtype=torch.uint8).to(dev)
    d_msg = torch.frombuffer(bytearray(b"".join(roots)), dtype=torch.uint8).to(dev)
    d_off = torch.arange(0, 32 * (n + 1), 32, dtype=torch.int64).to(dev)
    d_st = torch.full((n,), -1, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)
    gathered = [None]

    def step():
        rc = lib.hipbls_verify_batch_device(d_pk.data_ptr(), d_msg.data_ptr(), d_off.data_ptr(), d_sig.data_ptr(),
                                            n, d_st.data_ptr(), ctypes.c_void_p(stream.cuda_stream))
        if rc != 0:
            raise RuntimeError("hipbls_verify_batch_device rc=%d %s" % (rc, lib.hipbls_last_error()))
        if world > 1:  # the only collective: all-gather of the per-rank verify bitmaps (RCCL/xGMI)
            gathered[0] = gather_bitmaps(pack_bitmap(d_st))

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    lib.hipbls_kernel_timing_reset()
    barrier()
    torch.cuda.synchronize(dev)
    t_start = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    barrier()
    elapsed = time.perf_counter() - t_start

    st = d_st.cpu().tolist()
    fails = {i for i, s in enumerate(st) if s != 0}
    assert fails == bad, "verify bitmap mismatch: %d unexpected, %d missed" % (len(fails - bad), len(bad - fails))
    if world > 1:  # my row of the gathered node bitmap equals my local result
        mine = unpack_bitmap(gathered[0][rank], n).cpu()
        assert {i for i in range(n) if not mine[i]} == bad, "gathered bitmap mismatch"
    avg_ms = ctypes.c_double()
    launches = ctypes.c_uint64()
    lib.hipbls_kernel_timing(b"verify", ctypes.byref(avg_ms), ctypes.byref(launches))

    t_max = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
    elapsed = float(t_max.item())
    total = n * args.steps * world
    value = total / elapsed

    # ---- C2 with the resident pubshare table (extra field): same items, keys by index
    keys_rate = None
    if args.keys:
        table = list(dict.fromkeys(pks))
        pos = {k: j for j, k in enumerate(table)}
        assert set(impl.load_pubshares(table)) == {0}
        d_kidx = torch.tensor([pos[p] for p in pks], dtype=torch.int32).to(dev)
        d_kst = torch.full((n,), -1, dtype=torch.int32, device=dev)

        def kstep():
            rc = lib.hipbls_verify_batch_keys_device(d_kidx.data_ptr(), d_msg.data_ptr(), d_off.data_ptr(),
                                                     d_sig.data_ptr(), n, d_kst.data_ptr(),
                                                     ctypes.c_void_p(stream.cuda_stream))
            assert rc == 0

        kstep()
        torch.cuda.synchronize(dev)
        barrier()
        ts = time.perf_counter()
        for _ in range(args.steps):
            kstep()
        torch.cuda.synchronize(dev)
        barrier()
        tk = time.perf_counter() - ts
        assert d_kst.cpu().tolist() == st, "key-table bitmap differs from wire-format Verify"
        tt = torch.tensor([tk], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        keys_rate = n * args.steps * world / float(tt.item())

    # ---- C3: threshold aggregation + Verify of the aggregate (extra field)
    tagg = None
    if args.tagg_groups > 0:
        t0 = time.time()
        psigs, pids, poffs, dv_pks, droots = make_c3(impl, args.tagg_groups, rng)
        log("rank %d: C3 data (%d groups) in %.1fs" % (rank, args.tagg_groups, time.time() - t0))
        G = args.tagg_groups
        d_psig = torch.frombuffer(bytearray(b"".join(psigs)), dtype=torch.uint8).to(dev)
        d_pid = torch.tensor(pids, dtype=torch.int64).to(dev)
        d_poff = torch.tensor(poffs, dtype=torch.int64).to(dev)
        d_agg = torch.zeros(G * 96, dtype=torch.uint8, device=dev)
        d_gst = torch.full((G,), -1, dtype=torch.int32, device=dev)
        d_dpk = torch.frombuffer(bytearray(b"".join(dv_pks)), dtype=torch.uint8).to(dev)
        d_dmsg = torch.frombuffer(bytearray(b"".join(droots)), dtype=torch.uint8).to(dev)
        d_doff = torch.arange(0, 32 * (G + 1), 32, dtype=torch.int64).to(dev)
        d_vst = torch.full((G,), -1, dtype=torch.int32, device=dev)

        def tstep():
            rc = lib.hipbls_threshold_aggregate_batch_device(d_psig.data_ptr(), d_pid.data_ptr(), d_poff.data_ptr(), G,
                                                             len(pids), d_agg.data_ptr(), d_gst.data_ptr(),
                                                             ctypes.c_void_p(stream.cuda_stream))
            assert rc == 0
            rc = lib.hipbls_verify_batch_device(d_dpk.data_ptr(), d_dmsg.data_ptr(), d_doff.data_ptr(),
                                                d_agg.data_ptr(), G, d_vst.data_ptr(),
                                                ctypes.c_void_p(stream.cuda_stream))
            assert rc == 0

        tstep()
        torch.cuda.synchronize(dev)
        barrier()
        ts = time.perf_counter()
        for _ in range(args.tagg_steps):
            tstep()
        torch.cuda.synchronize(dev)
        barrier()
        tel = time.perf_counter() - ts
        assert set(d_gst.cpu().tolist()) == {0} and set(d_vst.cpu().tolist()) == {0}, "aggregate mismatch"
        tt = torch.tensor([tel], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        tagg = G * args.tagg_steps * world / float(tt.item())

    # ---- C4: random-linear-combination BatchVerify of this rank's shard (extra fields)
    rlc = {}
    if args.rlc_validators > 0:
        variants = [("i_root_per_validator", args.rlc_validators, 0),
                    ("ii_committee_roots", args.rlc_validators, max(1, args.rlc_validators // 128))]
        if args.rlc_big_validators > 0:
            variants.append(("i_node_batch_on_each_gpu", args.rlc_big_validators, 0))
        for variant, n_dv, shared in variants:
            t0 = time.time()
            pks4, sigs4, midx4, roots4, bad4 = make_c4(impl, n_dv, rng, shared_roots=shared)
            n4 = len(pks4)
            log("rank %d: C4(%s) data (%d items, %d roots) in %.1fs" % (rank, variant, n4, len(roots4), time.time() - t0))
            d_pk4 = torch.frombuffer(bytearray(b"".join(pks4)), dtype=torch.uint8).to(dev)
            d_sig4 = torch.frombuffer(bytearray(b"".join(sigs4)), dtype=torch.uint8).to(dev)
            d_midx4 = torch.tensor(midx4, dtype=torch.int32).to(dev)
            d_msg4 = torch.frombuffer(bytearray(b"".join(roots4)), dtype=torch.uint8).to(dev)
            d_off4 = torch.arange(0, 32 * (len(roots4) + 1), 32, dtype=torch.int64).to(dev)
            d_st4 = torch.full((n4,), -7, dtype=torch.int32, device=dev)
            seed = os.urandom(32)

            def rstep():
                rc = lib.hipbls_batch_verify_rlc_device(d_pk4.data_ptr(), d_sig4.data_ptr(), d_midx4.data_ptr(), n4,
                                                        d_msg4.data_ptr(), d_off4.data_ptr(), len(roots4), seed,
                                                        d_st4.data_ptr(), ctypes.c_void_p(stream.cuda_stream))
                if rc != 0:
                    raise RuntimeError("hipbls_batch_verify_rlc_device rc=%d" % rc)

            rstep()
            torch.cuda.synchronize(dev)
            lib.hipbls_kernel_timing_reset()
            barrier()
            torch.cuda.synchronize(dev)
            ts = time.perf_counter()
            for _ in range(args.rlc_steps):
                rstep()
            torch.cuda.synchronize(dev)
            barrier()
            tel = time.perf_counter() - ts
            st4 = d_st4.cpu().tolist()
            assert {i for i, x in enumerate(st4) if x != 0} == bad4, "RLC bitmap mismatch"
            w = ctypes.c_uint64()
            wf = ctypes.c_uint64()
            fb = ctypes.c_uint64()
            lib.hipbls_rlc_stats(ctypes.byref(w), ctypes.byref(wf), ctypes.byref(fb))
            kms = {}
            for k in ("rlc_items", "rlc_hash", "rlc_window", "rlc_window_lg2", "rlc_fallback", "rlc_fallback_lg2"):
                a = ctypes.c_double()
                c = ctypes.c_uint64()
                lib.hipbls_kernel_timing(k.encode(), ctypes.byref(a), ctypes.byref(c))
                if c.value:  # lane-pair (_lg2) or one-lane kernels, whichever HIPBLS_PAIR_AUTO picked
                    kms[k] = round(a.value, 3)
            tt = torch.tensor([tel], dtype=torch.float64, device=dev)
            if world > 1:
                dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            per_win = RLC_FPMUL["window_1msg"] if shared else RLC_FPMUL["window_2msg"]
            fpmul = (RLC_FPMUL["item"] * n4 + RLC_FPMUL["hash"] * len(roots4) + per_win * w.value
                     + RLC_FPMUL["fallback"] * fb.value)
            ach = fpmul * MADS_PER_FPMUL * args.rlc_steps / float(tt.item()) / 1e12
            rlc[variant] = {"verified_partial_sigs_per_s": round(n4 * args.rlc_steps * world / float(tt.item()), 1),
                            "fpmul_per_item": round(fpmul / n4, 1),
                            "pipeline_roofline": {"achieved": round(ach, 3), "peak": MAD_PEAK_T, "unit": "Tmad/s",
                                                  "frac": round(ach / MAD_PEAK_T, 4),
                                                  "note": "whole 4-stage pipeline over wall time (not one kernel)"},
                            "items_per_gpu": n4, "distinct_roots_per_gpu": len(roots4),
                            "ms_per_batch": round(1000 * float(tt.item()) / args.rlc_steps, 3),
                            "windows": w.value, "windows_failed": wf.value, "items_fallback": fb.value,
                            "kernel_avg_ms": kms}
            if args.keys and variant == "i_root_per_validator":
                # same batch with pubshares from the resident table
                table4 = list(dict.fromkeys(pks4))
                pos4 = {k: j for j, k in enumerate(table4)}
                assert set(impl.load_pubshares(table4)) == {0}
                d_k4 = torch.tensor([pos4[p] for p in pks4], dtype=torch.int32).to(dev)

                def rkstep():
                    rc = lib.hipbls_batch_verify_rlc_keys_device(d_k4.data_ptr(), d_sig4.data_ptr(),
                                                                 d_midx4.data_ptr(), n4, d_msg4.data_ptr(),
                                                                 d_off4.data_ptr(), len(roots4), seed,
                                                                 d_st4.data_ptr(), ctypes.c_void_p(stream.cuda_stream))
                    assert rc == 0

                rkstep()
                torch.cuda.synchronize(dev)
                barrier()
                ts = time.perf_counter()
                for _ in range(args.rlc_steps):
                    rkstep()
                torch.cuda.synchronize(dev)
                barrier()
                tk = time.perf_counter() - ts
                assert d_st4.cpu().tolist() == st4, "RLC key-table bitmap differs"
                tt = torch.tensor([tk], dtype=torch.float64, device=dev)
                if world > 1:
                    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
                rlc[variant]["verified_partial_sigs_per_s_pubshare_table"] = round(
                    n4 * args.rlc_steps * world / float(tt.item()), 1)
            del d_pk4, d_sig4, d_midx4, d_msg4, d_off4, d_st4

    # ---- C5: full-slot mix on this rank's shard: RLC over the C4 shard + 32 validators x 4 proposer
    # partials (own roots), concurrently with a 512-key sync-committee FastAggregateVerify
    c5 = None
    if args.c5 and args.rlc_validators > 0:
        t0 = time.time()
        pks5, sigs5, midx5, roots5, bad5 = make_c4(impl, args.rlc_validators, rng)
        ppks, psigs, pmidx, proots, pbad = make_c4(impl, 32, rng, nkeys=128)
        off = len(roots5)
        base = len(pks5)
        pks5 += ppks
        sigs5 += psigs
        midx5 += [m + off for m in pmidx]
        roots5 += proots
        bad5 |= {base + i for i in pbad}
        n5 = len(pks5)
        sync_sks = [rng.randrange(1, R_ORDER).to_bytes(32, "big") for _ in range(512)]
        sync_pks, _ = impl.secret_to_public_key_batch(sync_sks)
        sync_root = rng.randbytes(32)
        ssigs, _ = impl.sign_batch(sync_sks, [sync_root] * 512)
        sync_agg = impl.aggregate(ssigs)
        log("rank %d: C5 data (%d partials + 512-key sync aggregate) in %.1fs" % (rank, n5, time.time() - t0))
        d_pk5 = torch.frombuffer(bytearray(b"".join(pks5)), dtype=torch.uint8).to(dev)
        d_sig5 = torch.frombuffer(bytearray(b"".join(sigs5)), dtype=torch.uint8).to(dev)
        d_midx5 = torch.tensor(midx5, dtype=torch.int32).to(dev)
        d_msg5 = torch.frombuffer(bytearray(b"".join(roots5)), dtype=torch.uint8).to(dev)
        d_off5 = torch.arange(0, 32 * (len(roots5) + 1), 32, dtype=torch.int64).to(dev)
        d_st5 = torch.full((n5,), -7, dtype=torch.int32, device=dev)
        d_spk = torch.frombuffer(bytearray(b"".join(sync_pks)), dtype=torch.uint8).to(dev)
        d_skoff = torch.tensor([0, 512], dtype=torch.int64).to(dev)
        d_ssig = torch.frombuffer(bytearray(sync_agg), dtype=torch.uint8).to(dev)
        d_smsg = torch.frombuffer(bytearray(sync_root), dtype=torch.uint8).to(dev)
        d_smoff = torch.tensor([0, 32], dtype=torch.int64).to(dev)
        d_sst = torch.full((1,), -7, dtype=torch.int32, device=dev)
        seed5 = os.urandom(32)

        def c5step():
            # the sync-committee check goes on the library's own stream (NULL) and overlaps the RLC
            rc = lib.hipbls_verify_aggregate_batch_device(d_spk.data_ptr(), 512, d_skoff.data_ptr(), 1,
                                                          d_ssig.data_ptr(), d_smsg.data_ptr(), d_smoff.data_ptr(),
                                                          d_sst.data_ptr(), None)
            assert rc == 0
            rc = lib.hipbls_batch_verify_rlc_device(d_pk5.data_ptr(), d_sig5.data_ptr(), d_midx5.data_ptr(), n5,
                                                    d_msg5.data_ptr(), d_off5.data_ptr(), len(roots5), seed5,
                                                    d_st5.data_ptr(), ctypes.c_void_p(stream.cuda_stream))
            assert rc == 0

        c5step()
        torch.cuda.synchronize()
        barrier()
        ts = time.perf_counter()
        for _ in range(args.rlc_steps):
            c5step()
        torch.cuda.synchronize()
        barrier()
        t5 = time.perf_counter() - ts
        assert {i for i, x in enumerate(d_st5.cpu().tolist()) if x != 0} == bad5, "C5 bitmap mismatch"
        assert d_sst.cpu().tolist() == [0], "sync-committee FastAggregateVerify failed"
        tt = torch.tensor([t5], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t5 = float(tt.item())
        c5 = {"workload": "C5 (BASELINE configs[4]) per GPU: RLC BatchVerify of the C4 shard (%d validators x 4, "
                          "one root each) + 32 validators x 4 proposer partials (own roots), 1%% corrupted, with a "
                          "512-key sync-committee FastAggregateVerify (hash-to-G2 of its root) overlapped"
                          % args.rlc_validators,
              "partials_per_slot_per_gpu": n5, "ms_per_slot": round(1000 * t5 / args.rlc_steps, 3),
              "verified_partial_sigs_per_s": round(n5 * args.rlc_steps * world / t5, 1),
              "sync_aggregate_verifies_per_s": round(args.rlc_steps * world / t5, 3)}
        del d_pk5, d_sig5, d_midx5, d_msg5, d_off5, d_st5

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "verified partial sigs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000 * elapsed / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic: seeded share keys, distinct 32-byte roots, 1% corrupted (wrong root / swapped "
                    "share / flipped sig bit); signatures made by the engine's own sign kernel",
            "config": {"workload": "C2 (BASELINE.json configs[1]): individual tbls.Verify of %d partial sigs per GPU, "
                                   "distinct messages" % n,
                       "items_per_gpu": n, "parallelism": "shard-by-validator-index x %d" % world},
            "pairings_per_s": round(2 * value, 1),
            "verified_partial_sigs_per_s_pubshare_table": round(keys_rate, 1) if keys_rate else None,
            "threshold_aggregates_per_s": round(tagg, 1) if tagg else None,
            "threshold_aggregate_workload": "C3: %d validators x 7-of-10 Lagrange in G2 + Verify of each aggregate per GPU"
                                            % args.tagg_groups if tagg else None,
        }
        if c5:
            out["full_slot_mix"] = c5
        if rlc:
            out["rlc_batch_verify"] = dict(rlc, workload="C4 (BASELINE configs[3]): validators x 4 partials per GPU, "
                                                        "items grouped by validator, 1%% corrupted (swapped share / "
                                                        "flipped sig bit), windows of 8 items, per-item bitmap == "
                                                        "tbls.Verify; i/ii = the 1M-partial node batch sharded over 8 "
                                                        "GPUs (%d validators per GPU), node_batch = all 1M on every GPU"
                                                        % args.rlc_validators)
        k_ms = avg_ms.value
        if k_ms > 0:
            achieved = FPMUL_PER_VERIFY * MADS_PER_FPMUL * n / (k_ms * 1e-3) / 1e12
            out["roofline"] = {
                "bound": "valu-int (32x32->64 v_mad_u64_u32; no HBM or MFMA bound: ~190 B in per verify)",
                "kernel": "k_verify_fused",
                "achieved": round(achieved, 3),
                "peak": MAD_PEAK_T,
                "unit": "Tmad/s",
                "frac": round(achieved / MAD_PEAK_T, 4),
                "traffic": traffic_from_pmc(),
                "algorithmic_unit": "%d Fp-mul-equivalents x %d MADs per verify" % (FPMUL_PER_VERIFY, MADS_PER_FPMUL),
                "kernel_avg_ms": round(k_ms, 3),
                "kernel_launches": int(launches.value),
            }
        if world == 1 and args.cpu_sample > 0:
            out["cpu_baseline"] = cpu_baseline(impl, (pks, roots, sigs, bad), args.cpu_sample, random.Random(SEED))
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
