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
import hashlib
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
# this in sync).  Inversions are binary-GCD divsteps (field.h fp_inv), which are not products and are not
# counted: ~33k VALU each, about 49 products' worth of issue time.  See DESIGN.md "Roofline".
FPMUL_PER_VERIFY = 24247
MADS_PER_FPMUL = 300
# HIPBLS_RLC_AUTO after a failed batch-wide check: kRlcbBackoff (8) calls on windows only, then the check again
# (charon_amd/csrc/hipbls.hip use_rlc_batch), so a stream with invalid partials pays one failed check per 9 calls
RLC_AUTO_PERIOD = 9
# RLC BatchVerify stages (charon_amd/csrc/rlc.h), same unit and source (tests/test_work_counts.py):
# stage 1 per item, stage 2 per distinct message, stage 3 per window of 8 with 2 messages (one per
# 4-partial validator) or 1 message (committee root), stage 4 per item re-checked after a failed window.
RLC_FPMUL = {"item": 5495, "hash": 4790, "window_2msg": 21906, "window_1msg": 17485, "fallback": 17021}
# Batch-wide check (charon_amd/csrc/rlcb.h), same unit and source: stage 1 per item, the Pippenger MSM per item
# (2 points x 2 windows of mixed additions; the bucket/segment folds add ~15 per item at 1M items and are left
# out), and one multi-Miller loop per 16-item chunk with 4 message runs (one root per 4-partial validator) or with one
# run (committee roots, C4(ii)).
RLCB_FPMUL = {"item": 4306, "msm_per_item": 116, "chunk_4runs": 18948, "chunk_1run": 6909,
              # the G1 MSM per committee root (g1msm.h) at 512 items per root: stage 1 without the per-item Shamir
              # multiplication, the bucket + fold work per item, one Miller pair per root
              "item_g1slot": 3702, "g1msm_per_item_512": 207, "g1miller_per_root": 6977}
# sigagg in one call (C3), per aggregate of 7 partials, same unit and source (tests/native/host_ops.cpp
# ht_count_tagg_verify, tests/test_work_counts.py): the 7 partials' decode + subgroup test + c_k sig_k (k_tagg_scale),
# the sum S (k_tagg_sum_s), [L^-1] S + compress (k_tagg_unscale), the root key's decode + subgroup test + [L] pk +
# hash_to_G2 (k_tv_prep_pk), and the pairing check on S against [L] pk (k_verify_pair_lq4).
TAGG_FPMUL = {"scale_7": 17209, "sum": 274, "unscale": 4071, "key_prep": 6493, "pairing": 17012}
# gfx950 32x32->64 integer multiply-add peak (v_mad_u64_u32): 256 CU x 4 SIMD x 32 lanes x 2.4 GHz
# at half rate (measured: profiles/r01_mad_probe.txt) = 39.3e12 MAD/s.
MAD_PEAK_T = 39.3


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--c2-items", dest="n", type=int, default=65536,
                    help="C2 verifies per GPU per step (65,536); node batch = items x world")
    ap.add_argument("--tagg-groups", type=int, default=10000,
                    help="C3 validators per GPU (0 = skip); node batch = groups x world")
    ap.add_argument("--tagg-steps", type=int, default=2)
    ap.add_argument("--tagg-two-streams", type=int, default=1,
                    help="also time C3 with consecutive calls alternating between two streams (0 = skip)")
    ap.add_argument("--cpu-sample", type=int, default=4096,
                    help="C2 items verified by the C++ CPU baseline, one thread per core (0 = skip)")
    ap.add_argument("--rlc-node-validators", type=int, default=262144,
                    help="C4 node batch in validators (x4 partials; 262,144 = 1M partials), sliced over the ranks "
                         "with shard_range (0 = skip)")
    ap.add_argument("--rlc-steps", type=int, default=3)
    ap.add_argument("--rlc-variants", default="i,ii,all_valid,ii_all_valid",
                    help="C4 variants to time: i (one root per validator), ii (committee roots), all_valid (i, no "
                         "invalid partial), ii_all_valid (ii, no invalid partial)")
    ap.add_argument("--c5", type=int, default=1, help="time the C5 full-slot mix (0 = skip)")
    ap.add_argument("--keys", type=int, default=1, help="also time C2 / C4 with the resident pubshare table (0 = skip)")
    ap.add_argument("--host-path", type=int, default=1,
                    help="time the host-buffer calls charon's Go code makes (C2 hipbls_verify_batch[_keys], C3 "
                         "hipbls_threshold_aggregate_verify_batch), PCIe copies included; rank 0 (0 = skip)")
    ap.add_argument("--latency-calls", type=int, default=1000,
                    help="synchronous n = 1 tbls.Verify calls (hipbls_verify on an idle queue) timed one after another, "
                         "the unpatched parsigex loop's shape (0 = skip; rank 0 only)")
    return ap.parse_args()


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


# ---------------------------------------------------------------- synthetic node batches
# Every item of a node batch is a pure function of (SEED, config tag, global index), so each rank builds exactly its
# shard_range slice of the same node batch and can recompute the node-wide expected bitmap after the all-gather.
def _hb(*parts) -> bytes:
    return hashlib.sha256(("%x|" % SEED + "|".join(str(p) for p in parts)).encode()).digest()


def _hi(*parts) -> int:
    return int.from_bytes(_hb(*parts)[:8], "big")


def _scalar(*parts) -> int:
    """Uniform-ish secret in [1, r)."""
    return int.from_bytes(_hb(*parts), "big") % (R_ORDER - 1) + 1


def share_keys(impl, nkeys, tag):
    sks = [_scalar(tag, "sk", k).to_bytes(32, "big") for k in range(nkeys)]
    pks, st = impl.secret_to_public_key_batch(sks)
    assert set(st) == {0}
    return sks, pks


def c2_is_bad(i):
    r = _hi("c2", "bad", i)
    return r % 100 == 0, (r >> 32) % 3


def make_c2(impl, keys, lo, hi):
    """Items [lo, hi) of the C2 node batch: partial signatures by 4,096 share keys over distinct roots, ~1% corrupted
    (wrong root / swapped share / flipped signature bit).  Returns local lists + the set of local bad indices."""
    sks, pks = keys
    nk = len(sks)
    idx = range(lo, hi)
    roots = [_hb("c2", "root", i) for i in idx]
    owner = [i % nk for i in idx]
    sigs, st = impl.sign_batch([sks[o] for o in owner], roots)
    assert set(st) <= {0}
    pk_list = [pks[o] for o in owner]
    bad = set()
    for j, i in enumerate(idx):
        is_bad, kind = c2_is_bad(i)
        if not is_bad:
            continue
        bad.add(j)
        if kind == 0:
            roots[j] = _hb("c2", "wrong-root", i)
        elif kind == 1:
            pk_list[j] = pks[(owner[j] + 1) % nk]
        else:
            s = bytearray(sigs[j])
            s[40] ^= 0x04
            sigs[j] = bytes(s)
    return pk_list, roots, sigs, bad


def make_c3(impl, g_lo, g_hi, t=7, n=10):
    """Validators [g_lo, g_hi) of the C3 node batch: each split t-of-n, a seeded t-subset of partials, the DV pubkey
    and one root each."""
    part_sks, part_msgs, part_ids, offs, secrets_, roots = [], [], [], [0], [], []
    for v in range(g_lo, g_hi):
        secret = _scalar("c3", "sk", v)
        poly = [secret] + [_scalar("c3", "poly", v, k) - 1 for k in range(t - 1)]
        ids = sorted(random.Random(_hi("c3", "ids", v)).sample(range(1, n + 1), t))
        root = _hb("c3", "root", v)
        secrets_.append(secret)
        roots.append(root)
        for i in ids:
            acc = 0
            for c in reversed(poly):
                acc = (acc * i + c) % R_ORDER
            part_sks.append(acc.to_bytes(32, "big"))
            part_msgs.append(root)
            part_ids.append(i)
        offs.append(len(part_ids))
    psigs, st = impl.sign_batch(part_sks, part_msgs)
    assert set(st) <= {0}
    dv_pks, st = impl.secret_to_public_key_batch([s.to_bytes(32, "big") for s in secrets_])
    assert set(st) <= {0}
    return psigs, part_ids, offs, dv_pks, roots, secrets_


# Invalid partials per 1,000 in the C4 / C5 batches (BASELINE's ~1 %: 10).  BENCH_C4_BAD_PER_MILLE changes it for the
# fallback-size measurements of DESIGN.md 9 (round 6); the default line always uses 10.
C4_BAD_PER_MILLE = int(os.environ.get("BENCH_C4_BAD_PER_MILLE", "10"))


def c4_item(tag, v, j, nk, corrupt=True):
    """(owner key, bad?, kind) of partial j of validator v; corrupt=False: an all-valid node batch."""
    r = _hi(tag, v, j)
    bad = (r >> 20) % 100 == 0 if C4_BAD_PER_MILLE == 10 else (r >> 20) % 1000 < C4_BAD_PER_MILLE
    return r % nk, corrupt and bad, (r >> 40) & 1


def make_c4(impl, keys, tag, v_lo, v_hi, v_node, n_roots_node=0, shares=4, corrupt=True):
    """Validators [v_lo, v_hi) of a C4 node batch of v_node validators x `shares` partials, items grouped by
    validator.  One root per validator (n_roots_node = 0, variant i) or n_roots_node committee roots over the node
    batch, contiguous committees (variant ii).  ~1% corrupted (swapped share / flipped signature bit)."""
    sks, pks = keys
    nk = len(sks)
    if n_roots_node:
        root_of = [v * n_roots_node // v_node for v in range(v_lo, v_hi)]
    else:
        root_of = list(range(v_lo, v_hi))
    first = root_of[0] if root_of else 0
    roots = [_hb(tag, "root", g) for g in range(first, (root_of[-1] + 1) if root_of else 0)]
    owner, midx, bad, kinds = [], [], set(), {}
    for dv, v in enumerate(range(v_lo, v_hi)):
        for j in range(shares):
            o, is_bad, kind = c4_item(tag, v, j, nk, corrupt)
            if is_bad:
                bad.add(len(owner))
                kinds[len(owner)] = kind
            owner.append(o)
            midx.append(root_of[dv] - first)
    sigs, st = impl.sign_batch([sks[o] for o in owner], [roots[m] for m in midx])
    assert set(st) <= {0}
    pk_list = [pks[o] for o in owner]
    for i, kind in kinds.items():
        if kind == 0:
            pk_list[i] = pks[(owner[i] + 1) % nk]
        else:
            s = bytearray(sigs[i])
            s[40] ^= 0x04
            sigs[i] = bytes(s)
    return pk_list, sigs, midx, roots, bad


def c4_node_bad(tag, v_node, nk, shares=4, corrupt=True):
    return {v * shares + j for v in range(v_node) for j in range(shares) if c4_item(tag, v, j, nk, corrupt)[1]}


def pmc_summary(path=None):
    """k_verify_fused counters from the committed rocprofv3 --pmc passes over this build's bench (scripts/gpu_pmc.sh
    WL=c2, scripts/pmc_commit_r04.py): HBM bytes per launch (FETCH_SIZE + WRITE_SIZE), their ratio to the 188 B/verify
    of algorithmic input, VALU utilisation (SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES at one wave per SIMD), the fraction
    of wave cycles spent waiting, VALU and 64-bit integer VALU (the v_mad_u64_u32 stream) instructions per wave, and
    the commit the counters were taken at.  {} when absent.  The newest round's passes are read."""
    if path is None:
        for rnd in ("r06", "r05", "r04"):
            path = os.path.join(ROOT, "profiles", rnd, "pmc_verify.json")
            if os.path.exists(path):
                break
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return {}
    return {"hbm_bytes_per_launch": d.get("hbm_bytes_per_launch_raw"), "traffic_ratio": d.get("traffic_ratio"),
            "valu_util": d.get("valu_util"), "wait_any_frac": d.get("wait_any_frac"),
            "valu_insts_per_wave": d.get("valu_insts_per_wave"),
            "int64_valu_insts_per_wave": d.get("int64_valu_insts_per_wave"),
            "taken_at": d.get("taken_at"), "source": os.path.relpath(path, ROOT)}


def attainable_products(path=None):
    """The product routines' own rate on every SIMD (profiles/<round>/ceiling_probe.json, written from
    charon_amd/tools/ceiling_probe's output); {} when absent."""
    if path is None:
        path = os.path.join(ROOT, "profiles", "r06", "ceiling_probe.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return {}
    d["source_file"] = os.path.relpath(path, ROOT)
    return d


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


def timed_loop(step, steps, dev, barrier, world):
    """barrier + synchronize, `steps` calls, synchronize + barrier; max over ranks (seconds)."""
    import torch
    import torch.distributed as dist
    torch.cuda.synchronize(dev)
    barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize(dev)
    barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    else:
        t = torch.tensor([el], dtype=torch.float64)
    return float(t.item())


def kernel_stats(lib, name):
    a = ctypes.c_double()
    c = ctypes.c_uint64()
    lib.hipbls_kernel_timing(name.encode(), ctypes.byref(a), ctypes.byref(c))
    return a.value, c.value


def stage_fracs(lib, work, calls):
    """Per-stage roofline fraction: algorithmic Fp products of the stage over `calls` calls x 300 MADs, over the
    stage's summed kernel time (all its launches, from HIP events on the launch streams), against MAD_PEAK_T."""
    out = {}
    for k, fpmul in work.items():
        avg, n = kernel_stats(lib, k)
        if n and fpmul:
            out[k] = round(fpmul * calls * MADS_PER_FPMUL / (avg * n * 1e-3) / 1e12 / MAD_PEAK_T, 4)
    return out


def kernel_ms(lib, names):
    out = {}
    for k in names:
        a = ctypes.c_double()
        c = ctypes.c_uint64()
        lib.hipbls_kernel_timing(k.encode(), ctypes.byref(a), ctypes.byref(c))
        if c.value:  # lane-pair (_lg2) or one-lane kernels, whichever HIPBLS_PAIR_AUTO picked
            out[k] = round(a.value, 3)
    return out


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one rank per GPU; more ranks than GPUs only in a rehearsal (HIPBLS_BENCH_BACKEND=gloo on a one-GPU box)
    local_dev = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local_dev)
    dev = torch.device("cuda", local_dev)
    if world > 1:  # "nccl" is RCCL on ROCm: the production path
        backend = os.environ.get("HIPBLS_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group(backend="nccl", device_id=dev)
        else:
            dist.init_process_group(backend=backend)

    from charon_amd.shard import gather_aggregates, gather_bitmap_rows, gather_node_bitmap, shard_range, unpack_bitmap
    from charon_amd import build as hb
    from charon_amd.tbls import RLC_AUTO, RLC_BATCH, RLC_WINDOWS, HipBLS, load_library
    build_src = hb.verify()  # the binary measured is the one built from the sources beside it
    impl = HipBLS(device=local_dev)
    lib = load_library()
    lib.hipbls_set_timing(1)  # per-kernel HIP events for the roofline (off by default in the library)
    # A stream of our own, made current: the library's *_device calls enqueue on it, and the bitmap packing and the
    # collectives that read their results run after them on the same stream.  (The default stream's handle is 0,
    # which the library reads as "my own stream": nothing would order the gathers behind its kernels.)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    sp = ctypes.c_void_p(stream.cuda_stream)

    def barrier():
        if world > 1:
            dist.barrier()

    def u8(blobs):
        return torch.frombuffer(bytearray(b"".join(blobs)), dtype=torch.uint8).to(dev)

    # ---- C2 (headline): the node batch is n x world items; this rank verifies its shard_range slice, then the
    # per-rank bitmaps are all-gathered over RCCL inside the timed step (the only collective)
    t0 = time.time()
    keys2 = share_keys(impl, 4096, "c2")
    n_node = args.n * world
    lo, hi = shard_range(n_node, rank, world)
    n = hi - lo
    pks, roots, sigs, bad = make_c2(impl, keys2, lo, hi)
    log("rank %d: C2 slice [%d, %d) of %d in %.1fs" % (rank, lo, hi, n_node, time.time() - t0))
    d_pk, d_sig, d_msg = u8(pks), u8(sigs), u8(roots)
    d_off = torch.arange(0, 32 * (n + 1), 32, dtype=torch.int64).to(dev)
    d_st = torch.full((n,), -1, dtype=torch.int32, device=dev)
    node_ok = [None]

    def step():
        rc = lib.hipbls_verify_batch_device(d_pk.data_ptr(), d_msg.data_ptr(), d_off.data_ptr(), d_sig.data_ptr(),
                                            n, d_st.data_ptr(), sp)
        if rc != 0:
            raise RuntimeError("hipbls_verify_batch_device rc=%d %s" % (rc, lib.hipbls_last_error()))
        if world > 1:
            node_ok[0] = gather_node_bitmap(d_st, n_node)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    lib.hipbls_kernel_timing_reset()
    elapsed = timed_loop(step, args.steps, dev, barrier, world)
    st = d_st.cpu().tolist()
    assert {i for i, s in enumerate(st) if s != 0} == bad, "verify bitmap mismatch"
    if world > 1:  # the gathered node bitmap equals the node batch's construction
        want = {i for i in range(n_node) if c2_is_bad(i)[0]}
        got = node_ok[0].cpu()
        assert {i for i in range(n_node) if not got[i]} == want, "gathered node bitmap mismatch"
    avg_ms = ctypes.c_double()
    launches = ctypes.c_uint64()
    lib.hipbls_kernel_timing(b"verify", ctypes.byref(avg_ms), ctypes.byref(launches))
    value = n_node * args.steps / elapsed

    # ---- drop-in latency: the unpatched callers run tbls.Verify one item at a time, synchronously
    # (core/parsigex/parsigex.go:86-91 verifies a peer's set in series, validatorapi.go:246-283 every attestation):
    # each call is one n = 1 batch through the submission queue, so the serial rate is 1 / latency.  Rank 0, untimed
    # by the step loop (it is a latency, not a throughput).
    latency = None
    if args.latency_calls > 0 and rank == 0:
        k = min(args.latency_calls, n)
        assert impl.verify_queued(pks[0], roots[0], sigs[0]) == st[0]  # starts the queue worker
        lat = []
        w0, b0 = ctypes.c_uint64(), ctypes.c_uint64()
        lib.hipbls_queue_worker_stats(ctypes.byref(w0), ctypes.byref(b0))
        cpu0 = time.process_time()
        t0 = time.perf_counter()
        for j in range(k):
            a = time.perf_counter()
            got = impl.verify_queued(pks[j], roots[j], sigs[j])
            lat.append(time.perf_counter() - a)
            assert got == st[j], "queued Verify differs from the batch call"
        tot = time.perf_counter() - t0
        cpu = time.process_time() - cpu0
        w1, b1 = ctypes.c_uint64(), ctypes.c_uint64()
        lib.hipbls_queue_worker_stats(ctypes.byref(w1), ctypes.byref(b1))
        lat.sort()
        latency = {"calls": k, "p50_ms": round(1000 * lat[k // 2], 3), "p90_ms": round(1000 * lat[(9 * k) // 10], 3),
                   "min_ms": round(1000 * lat[0], 3), "serial_verifies_per_s": round(k / tot, 1),
                   "seconds_per_1000_serial": round(1000 * tot / k, 2),
                   "path": "hipbls_verify (submission queue, n = 1 batch: eight-lane prep (verify_lat.hip) + "
                           "sixteen-lane pairing check (verify_hex.hip); each stage raced by 8 replicas, one per XCD)",
                   # the queue worker's completion polls per batch (CPU inside the charon process) and the
                   # whole process's CPU time per call (the calling thread's ctypes round trip included)
                   "worker_polls_per_batch": round((w1.value - w0.value) / max(1, b1.value - b0.value), 1),
                   "process_cpu_ms_per_call": round(1000 * cpu / k, 3)}
        # the same calls without the replica race (hipbls_set_latency_replicas(1)), for comparison
        k1 = min(200, k)
        prev = lib.hipbls_set_latency_replicas(1)
        lat1 = []
        for j in range(k1):
            a = time.perf_counter()
            got = impl.verify_queued(pks[j], roots[j], sigs[j])
            lat1.append(time.perf_counter() - a)
            assert got == st[j], "queued Verify differs from the batch call"
        lib.hipbls_set_latency_replicas(prev)
        lat1.sort()
        latency["no_replicas"] = {"calls": k1, "p50_ms": round(1000 * lat1[k1 // 2], 3),
                                  "p90_ms": round(1000 * lat1[(9 * k1) // 10], 3)}

    # ---- C2 with the resident pubshare table (extra field): same items, keys by index
    keys_rate = None
    if args.keys:
        table = list(dict.fromkeys(pks))
        pos = {k: j for j, k in enumerate(table)}
        assert set(impl.load_pubshares(table)) <= {0}
        d_kidx = torch.tensor([pos[p] for p in pks], dtype=torch.int32).to(dev)
        d_kst = torch.full((n,), -1, dtype=torch.int32, device=dev)

        def kstep():
            rc = lib.hipbls_verify_batch_keys_device(d_kidx.data_ptr(), d_msg.data_ptr(), d_off.data_ptr(),
                                                     d_sig.data_ptr(), n, d_kst.data_ptr(), sp)
            assert rc == 0

        kstep()
        tk = timed_loop(kstep, args.steps, dev, barrier, world)
        assert d_kst.cpu().tolist() == st, "key-table bitmap differs from wire-format Verify"
        keys_rate = n_node * args.steps / tk

    # ---- C3: threshold aggregation + Verify of each aggregate; node batch = groups x world validators, this rank's
    # slice; the 96-byte aggregates and the verify bitmap are all-gathered inside the timed step
    tagg = None
    tagg2 = None
    tagg_kms = {}
    tagg_roofline = None
    if args.tagg_groups > 0:
        t0 = time.time()
        G_node = args.tagg_groups * world
        g_lo, g_hi = shard_range(G_node, rank, world)
        G = g_hi - g_lo
        psigs, pids, poffs, dv_pks, droots, dsecrets = make_c3(impl, g_lo, g_hi)
        log("rank %d: C3 slice [%d, %d) of %d validators in %.1fs" % (rank, g_lo, g_hi, G_node, time.time() - t0))
        d_psig = u8(psigs)
        d_pid = torch.tensor(pids, dtype=torch.int64).to(dev)
        d_poff = torch.tensor(poffs, dtype=torch.int64).to(dev)
        d_agg = torch.zeros(G * 96, dtype=torch.uint8, device=dev)
        d_gst = torch.full((G,), -1, dtype=torch.int32, device=dev)
        d_dpk, d_dmsg = u8(dv_pks), u8(droots)
        d_doff = torch.arange(0, 32 * (G + 1), 32, dtype=torch.int64).to(dev)
        d_vst = torch.full((G,), -1, dtype=torch.int32, device=dev)
        node_aggs = [None, None]

        def tstep():  # sigagg in one call: aggregate + Verify of each aggregate against the DV root key
            rc = lib.hipbls_threshold_aggregate_verify_batch_device(
                d_psig.data_ptr(), d_pid.data_ptr(), d_poff.data_ptr(), G, len(pids), d_dpk.data_ptr(),
                d_dmsg.data_ptr(), d_doff.data_ptr(), d_agg.data_ptr(), d_gst.data_ptr(), d_vst.data_ptr(), sp)
            assert rc == 0
            if world > 1:
                node_aggs[0] = gather_aggregates(d_agg, G_node)
                node_aggs[1] = gather_node_bitmap(d_vst, G_node)

        tstep()
        torch.cuda.synchronize(dev)
        lib.hipbls_kernel_timing_reset()
        tel = timed_loop(tstep, args.tagg_steps, dev, barrier, world)
        tagg_kms = kernel_ms(lib, ("tv_phase_a", "tagg_sum", "tv_check_unscale", "tagg_scale", "tagg_unscale",
                                   "tv_prep_pk", "verify_pair_lg2", "verify_pair_single"))
        assert set(d_gst.cpu().tolist()) == {0} and set(d_vst.cpu().tolist()) == {0}, "aggregate mismatch"
        # the 96-byte aggregates themselves (herumi.go:244-283 returns exactly these bytes, sigagg.go:149-154 injects
        # them): each equals Sign(secret) made by the separate sign kernel
        want_aggs, st_s = impl.sign_batch([s.to_bytes(32, "big") for s in dsecrets], droots)
        assert set(st_s) <= {0}
        assert bytes(d_agg.cpu().numpy().tobytes()) == b"".join(want_aggs), "C3 aggregate bytes != Sign(secret)"
        if world > 1:
            assert torch.equal(node_aggs[0][96 * g_lo:96 * g_hi], d_agg), "gathered aggregates differ from local"
            bad_g = (~node_aggs[1]).nonzero().flatten().tolist()
            assert not bad_g, "an aggregate of the node batch failed Verify: %d groups, first %s (this rank's slice " \
                              "[%d, %d))" % (len(bad_g), bad_g[:8], g_lo, g_hi)
        tagg = G_node * args.tagg_steps / tel
        # The same calls with two in flight: consecutive calls alternate between this stream and a second one (each
        # with its own outputs), as consecutive sigagg duties would; the library starts a call's phase A once the
        # previous call's is done, so it runs in the SIMDs the previous call's quad check leaves idle.  No gathers in
        # this measurement (two streams' collectives on one communicator are not ordered); outputs checked after.
        if args.tagg_two_streams:
            stream_b = torch.cuda.Stream(device=dev)
            sp_b = ctypes.c_void_p(stream_b.cuda_stream)
            d_agg_b = torch.zeros_like(d_agg)
            d_gst_b = torch.full_like(d_gst, -1)
            d_vst_b = torch.full_like(d_vst, -1)

            def tcall(spx, agg, gst, vst):
                rc = lib.hipbls_threshold_aggregate_verify_batch_device(
                    d_psig.data_ptr(), d_pid.data_ptr(), d_poff.data_ptr(), G, len(pids), d_dpk.data_ptr(),
                    d_dmsg.data_ptr(), d_doff.data_ptr(), agg.data_ptr(), gst.data_ptr(), vst.data_ptr(), spx)
                assert rc == 0

            def tstep2():  # two calls, one per stream
                tcall(sp, d_agg, d_gst, d_vst)
                tcall(sp_b, d_agg_b, d_gst_b, d_vst_b)

            tstep2()
            torch.cuda.synchronize(dev)
            tel2 = timed_loop(tstep2, args.tagg_steps, dev, barrier, world)
            for agg, gst, vst in ((d_agg, d_gst, d_vst), (d_agg_b, d_gst_b, d_vst_b)):
                assert set(gst.cpu().tolist()) == {0} and set(vst.cpu().tolist()) == {0}, "two-stream C3 statuses"
                assert bytes(agg.cpu().numpy().tobytes()) == b"".join(want_aggs), "two-stream C3 aggregate bytes"
            tagg2 = 2 * G_node * args.tagg_steps / tel2
        # C3 roofline: the counted per-aggregate unit over the whole call's wall time (the pipeline), and per stage over
        # its kernel's average launch time (HIP events on the launch stream)
        unit = sum(TAGG_FPMUL.values())
        ach = unit * MADS_PER_FPMUL * G * args.tagg_steps / tel / 1e12

        def kfrac(name, fpmul):
            a, c = kernel_stats(lib, name)
            return round(fpmul * MADS_PER_FPMUL / (a * 1e-3) / 1e12 / MAD_PEAK_T, 4) if c else None

        tagg_roofline = {
            "algorithmic_unit": "%d Fp-mul-equivalents x %d MADs per aggregate (7 partials + Verify)" % (unit,
                                                                                                     MADS_PER_FPMUL),
            "achieved": round(ach, 3), "peak": MAD_PEAK_T, "unit": "Tmad/s", "frac": round(ach / MAD_PEAK_T, 4),
            "note": "whole sigagg call (4 kernels on the caller's stream) over wall time, one call in flight",
            "stage_frac": {"tv_phase_a": kfrac("tv_phase_a", (TAGG_FPMUL["scale_7"] + TAGG_FPMUL["key_prep"]) * G),
                           "tv_check_unscale": kfrac("tv_check_unscale",
                                                     (TAGG_FPMUL["pairing"] + TAGG_FPMUL["unscale"]) * G)}}
        if tagg2:
            tagg_roofline["frac_two_streams"] = round(unit * MADS_PER_FPMUL * (tagg2 / world) / 1e12 / MAD_PEAK_T, 4)
        ceil = attainable_products()
        if ceil:  # the product routines' own rate on every SIMD (roofline.attainable)
            a = ceil["attainable_g_products_per_s_one_wave"]
            tagg_roofline["attainable"] = {"g_products_per_s": a,
                                           "achieved_g_products_per_s": round(unit * (tagg / world) / 1e9, 2),
                                           "frac": round(unit * (tagg / world) / 1e9 / a, 4),
                                           "frac_two_streams": round(unit * (tagg2 / world) / 1e9 / a, 4)
                                           if tagg2 else None, "source": ceil["source_file"]}

    # ---- the host-buffer calls charon's Go side makes (INTEGRATION.md "What charon reaches"): tbls.BatchVerify ->
    # hipbls_verify_batch, or hipbls_verify_batch_keys once app loaded the pubshare table; sigagg.NewFused ->
    # hipbls_threshold_aggregate_verify_batch.  Inputs copied in and statuses / aggregates copied out inside every call
    # (the PCIe-inclusive rate; `value` stays the resident-input rate).  Rank 0, this rank's items, untimed by the step
    # loop's barrier.
    host_path = None
    if args.host_path and rank == 0:
        from charon_amd.tbls import _offsets
        host_path = {"note": "host buffers in and out per call (cgo's path), rank 0's items, synchronous calls"}
        blob, offs = _offsets(roots)
        c_pk, c_sig = b"".join(pks), b"".join(sigs)
        c_st = (ctypes.c_int32 * n)()

        def hstep():
            assert lib.hipbls_verify_batch(c_pk, blob, offs, c_sig, n, c_st) == 0

        hstep()
        th = timed_loop(hstep, args.steps, dev, lambda: None, 1)
        assert list(c_st) == st, "host-buffer C2 statuses differ from the device call"
        host_path["c2_verify_batch_per_s"] = round(n * args.steps / th, 1)
        if args.keys:
            kidx = (ctypes.c_uint32 * n)(*[pos[p] for p in pks])

            def hkstep():
                assert lib.hipbls_verify_batch_keys(kidx, blob, offs, c_sig, n, c_st) == 0

            hkstep()
            thk = timed_loop(hkstep, args.steps, dev, lambda: None, 1)
            assert list(c_st) == st, "host-buffer keyed C2 statuses differ"
            host_path["c2_verify_batch_keys_per_s"] = round(n * args.steps / thk, 1)
        if args.tagg_groups > 0:
            gblob, goffs = _offsets(droots)
            c_psig, c_dpk = b"".join(psigs), b"".join(dv_pks)
            c_pid = (ctypes.c_int64 * len(pids))(*pids)
            c_poff = (ctypes.c_uint64 * len(poffs))(*poffs)
            c_out = ctypes.create_string_buffer(96 * G)
            c_ast, c_vst = (ctypes.c_int32 * G)(), (ctypes.c_int32 * G)()

            def hc3():
                assert lib.hipbls_threshold_aggregate_verify_batch(c_psig, c_pid, c_poff, G, c_dpk, gblob, goffs, c_out,
                                                                   c_ast, c_vst) == 0

            hc3()
            th3 = timed_loop(hc3, args.tagg_steps, dev, lambda: None, 1)
            assert set(c_ast) == {0} and set(c_vst) == {0} and c_out.raw == b"".join(want_aggs), "host C3"
            host_path["c3_threshold_aggregate_verify_batch_per_s"] = round(G * args.tagg_steps / th3, 1)
            # two threads each making the same calls (two goroutines with consecutive sigagg duties): the host call
            # holds the context lock only while it enqueues, so the second call's copies and phase A run beside the
            # first call's checks
            import threading
            outs2 = [(ctypes.create_string_buffer(96 * G), (ctypes.c_int32 * G)(), (ctypes.c_int32 * G)())
                     for _ in range(2)]

            k3 = max(4, args.tagg_steps)

            def hc3_thread(o):
                for _ in range(k3):
                    assert lib.hipbls_threshold_aggregate_verify_batch(c_psig, c_pid, c_poff, G, c_dpk, gblob, goffs,
                                                                       o[0], o[1], o[2]) == 0

            t0 = time.perf_counter()
            ths = [threading.Thread(target=hc3_thread, args=(o,)) for o in outs2]
            for t in ths:
                t.start()
            for t in ths:
                t.join()
            t2 = time.perf_counter() - t0
            for o in outs2:
                assert set(o[1]) == {0} and set(o[2]) == {0} and o[0].raw == b"".join(want_aggs), "host C3 x2"
            host_path["c3_two_threads_per_s"] = round(2 * G * k3 / t2, 1)

    # ---- C4: RLC BatchVerify of the 1M-partial node batch, validator-index slices over the ranks (strong scaling:
    # the node batch is fixed); node bitmap all-gathered inside the timed step
    rlc = {}
    c4i = None
    if args.rlc_node_validators > 0:
        V = args.rlc_node_validators
        v_lo, v_hi = shard_range(V, rank, world)
        keys4 = share_keys(impl, 4096, "c4")
        chosen = set(args.rlc_variants.split(","))
        for variant, tag, n_roots, corrupt in (("i_root_per_validator", "c4i", 0, True),
                                               ("ii_committee_roots", "c4ii", max(1, V // 128), True),
                                               ("i_all_valid", "c4h", 0, False),
                                               ("ii_all_valid", "c4hii", max(1, V // 128), False)):
            if {"i_root_per_validator": "i", "ii_committee_roots": "ii", "i_all_valid": "all_valid",
                "ii_all_valid": "ii_all_valid"}[variant] not in chosen:
                continue
            # the mode HIPBLS_RLC_AUTO settles on for each stream: windows while invalid partials keep arriving
            # (its batch-wide check keeps failing), the batch-wide check for an all-valid stream
            impl.set_rlc_mode(RLC_BATCH if not corrupt else RLC_WINDOWS)
            t0 = time.time()
            pks4, sigs4, midx4, roots4, bad4 = make_c4(impl, keys4, tag, v_lo, v_hi, V, n_roots, corrupt=corrupt)
            n4 = len(pks4)
            log("rank %d: C4(%s) validators [%d, %d) of %d: %d items, %d roots in %.1fs"
                % (rank, variant, v_lo, v_hi, V, n4, len(roots4), time.time() - t0))
            d_pk4, d_sig4, d_msg4 = u8(pks4), u8(sigs4), u8(roots4)
            d_midx4 = torch.tensor(midx4, dtype=torch.int32).to(dev)
            d_off4 = torch.arange(0, 32 * (len(roots4) + 1), 32, dtype=torch.int64).to(dev)
            d_st4 = torch.full((n4,), -7, dtype=torch.int32, device=dev)
            seed = os.urandom(32)
            node4 = [None]

            def rstep():
                rc = lib.hipbls_batch_verify_rlc_device(d_pk4.data_ptr(), d_sig4.data_ptr(), d_midx4.data_ptr(), n4,
                                                        d_msg4.data_ptr(), d_off4.data_ptr(), len(roots4), seed,
                                                        d_st4.data_ptr(), sp)
                if rc != 0:
                    raise RuntimeError("hipbls_batch_verify_rlc_device rc=%d" % rc)
                if world > 1:
                    node4[0] = gather_node_bitmap(d_st4, 4 * V)

            rstep()
            torch.cuda.synchronize(dev)
            lib.hipbls_kernel_timing_reset()
            b_att0, b_pass0, _ = impl.rlc_batch_stats()
            tel = timed_loop(rstep, args.rlc_steps, dev, barrier, world)
            b_att1, b_pass1, _ = impl.rlc_batch_stats()
            st4 = d_st4.cpu().tolist()
            assert {i for i, x in enumerate(st4) if x != 0} == bad4, "RLC bitmap mismatch"
            if world > 1:
                got = node4[0].cpu()
                want = c4_node_bad(tag, V, len(keys4[0]), corrupt=corrupt)
                assert {i for i in range(4 * V) if not got[i]} == want, "gathered RLC node bitmap mismatch"
            w = ctypes.c_uint64()
            wf = ctypes.c_uint64()
            fb = ctypes.c_uint64()
            lib.hipbls_rlc_stats(ctypes.byref(w), ctypes.byref(wf), ctypes.byref(fb))
            per_win = RLC_FPMUL["window_1msg"] if n_roots else RLC_FPMUL["window_2msg"]
            fpmul = (RLC_FPMUL["item"] * n4 + RLC_FPMUL["hash"] * len(roots4) + per_win * w.value
                     + RLC_FPMUL["fallback"] * fb.value)
            # committee roots take the G1 MSM path (hipbls.hip launch_rlc_batch: >= 8 items per root on average,
            # roots of >= 64 items)
            g1path = n_roots > 0 and n4 >= 8 * len(roots4) and n4 // len(roots4) >= 64
            item_unit = RLCB_FPMUL["item_g1slot" if g1path else "item"]
            chunk_work = 0 if g1path else RLCB_FPMUL["chunk_1run" if n_roots else "chunk_4runs"] * ((n4 + 15) // 16)
            g1_work = (RLCB_FPMUL["g1msm_per_item_512"] * n4 + RLCB_FPMUL["g1miller_per_root"] * len(roots4)
                       if g1path else 0)
            if b_pass1 > b_pass0:  # the batch-wide check decided alone: no window pairing work
                fpmul = ((item_unit + RLCB_FPMUL["msm_per_item"]) * n4 + RLC_FPMUL["hash"] * len(roots4) + chunk_work
                         + g1_work)
            ach = fpmul * MADS_PER_FPMUL * args.rlc_steps / tel / 1e12
            rlc[variant] = {"verified_partial_sigs_per_s": round(4 * V * args.rlc_steps / tel, 1),
                            "node_items": 4 * V, "items_this_gpu": n4, "distinct_roots_this_gpu": len(roots4),
                            "fpmul_per_item": round(fpmul / max(n4, 1), 1),
                            "pipeline_roofline": {"achieved": round(ach, 3), "peak": MAD_PEAK_T, "unit": "Tmad/s",
                                                  "frac": round(ach / MAD_PEAK_T, 4),
                                                  "note": "rank 0's 4-stage pipeline over wall time (not one kernel)"},
                            "ms_per_batch": round(1000 * tel / args.rlc_steps, 3),
                            "windows": w.value, "windows_failed": wf.value, "items_fallback": fb.value,
                            "batch_checks": {"attempted": b_att1 - b_att0, "passed": b_pass1 - b_pass0},
                            "kernel_avg_ms": kernel_ms(lib, ("rlc_items", "rlc_hash", "rlc_window", "rlc_window_lg2",
                                                             "rlc_fallback", "rlc_fallback_lg2", "rlcb_items",
                                                             "rlcb_msm", "rlcb_g1plan", "rlcb_g1sort", "rlcb_g1msm",
                                                             "rlcb_g1miller", "rlcb_chunks", "rlcb_sfactor", "rlcb_product", "rlcb_final",
                                                             "rlcb_mark")),
                            "stage_frac": stage_fracs(lib, {
                                "rlc_items": RLC_FPMUL["item"] * n4, "rlc_hash": RLC_FPMUL["hash"] * len(roots4),
                                # windows and fallback do nothing once the batch-wide check has passed
                                "rlc_window": 0 if b_pass1 > b_pass0 else per_win * w.value,
                                "rlc_window_lg2": 0 if b_pass1 > b_pass0 else per_win * w.value,
                                "rlc_fallback": RLC_FPMUL["fallback"] * fb.value,
                                "rlc_fallback_lg2": RLC_FPMUL["fallback"] * fb.value,
                                "rlcb_items": item_unit * n4, "rlcb_chunks": chunk_work,
                                "rlcb_g1msm": RLCB_FPMUL["g1msm_per_item_512"] * n4 if g1path else 0,
                                "rlcb_g1miller": RLCB_FPMUL["g1miller_per_root"] * len(roots4) if g1path else 0},
                                args.rlc_steps)}
            if corrupt and variant == "i_root_per_validator":
                # the library's default policy (HIPBLS_RLC_AUTO) on the same stream: one failing batch-wide check,
                # then windows while it backs off (rlc_mode comment above)
                impl.set_rlc_mode(RLC_AUTO)
                rstep()
                torch.cuda.synchronize(dev)
                tel_auto = timed_loop(rstep, args.rlc_steps, dev, barrier, world)
                assert {i for i, x in enumerate(d_st4.cpu().tolist()) if x != 0} == bad4, "RLC bitmap mismatch (auto)"
                rlc[variant]["auto_mode_ms_per_batch"] = round(1000 * tel_auto / args.rlc_steps, 3)
                # a batch-wide check that fails (what AUTO pays once every RLC_AUTO_PERIOD calls of such a stream:
                # the check, then the windows and fallback over the same items)
                impl.set_rlc_mode(RLC_BATCH)
                rstep()
                torch.cuda.synchronize(dev)
                tel_fb = timed_loop(rstep, args.rlc_steps, dev, barrier, world)
                assert {i for i, x in enumerate(d_st4.cpu().tolist()) if x != 0} == bad4, "RLC bitmap mismatch (batch)"
                fb_ms = 1000 * tel_fb / args.rlc_steps
                rlc[variant]["failed_batch_check_ms_per_batch"] = round(fb_ms, 3)
                rlc[variant]["auto_mode_amortized_ms_per_batch"] = round(
                    ((RLC_AUTO_PERIOD - 1) * 1000 * tel / args.rlc_steps + fb_ms) / RLC_AUTO_PERIOD, 3)
                impl.set_rlc_mode(RLC_AUTO)
            if args.keys and variant in ("i_root_per_validator", "i_all_valid"):
                table4 = list(dict.fromkeys(pks4))
                pos4 = {k: j for j, k in enumerate(table4)}
                assert set(impl.load_pubshares(table4)) <= {0}
                d_k4 = torch.tensor([pos4[p] for p in pks4], dtype=torch.int32).to(dev)

                def rkstep():
                    rc = lib.hipbls_batch_verify_rlc_keys_device(d_k4.data_ptr(), d_sig4.data_ptr(), d_midx4.data_ptr(),
                                                                 n4, d_msg4.data_ptr(), d_off4.data_ptr(), len(roots4),
                                                                 seed, d_st4.data_ptr(), sp)
                    assert rc == 0

                rkstep()
                tk = timed_loop(rkstep, args.rlc_steps, dev, barrier, world)
                assert d_st4.cpu().tolist() == st4, "RLC key-table bitmap differs"
                rlc[variant]["verified_partial_sigs_per_s_pubshare_table"] = round(4 * V * args.rlc_steps / tk, 1)
                del d_k4
            if variant == "i_root_per_validator":
                c4i = (pks4, sigs4, midx4, roots4, bad4)
            del d_pk4, d_sig4, d_midx4, d_msg4, d_off4, d_st4
        impl.set_rlc_mode(RLC_AUTO)

    # ---- C5: full-slot mix on this rank's slice: RLC over the C4(i) slice + its slice of 32 validators x 4 proposer
    # partials (own roots), with the 512-key sync-committee FastAggregateVerify (hash-to-G2 of its root) overlapped on
    # rank 0
    c5 = None
    if args.c5 and c4i is not None:
        t0 = time.time()
        pks5, sigs5, midx5, roots5, bad5 = [list(x) if not isinstance(x, set) else set(x) for x in c4i]
        p_lo, p_hi = shard_range(32, rank, world)
        ppks, psigs, pmidx, proots, pbad = make_c4(impl, share_keys(impl, 128, "c5p"), "c5p", p_lo, p_hi, 32)
        off = len(roots5)
        base = len(pks5)
        pks5 += ppks
        sigs5 += psigs
        midx5 += [m + off for m in pmidx]
        roots5 += proots
        bad5 |= {base + i for i in pbad}
        n5 = len(pks5)
        sync_sks = [_scalar("c5sync", k).to_bytes(32, "big") for k in range(512)]
        sync_pks, _ = impl.secret_to_public_key_batch(sync_sks)
        sync_root = _hb("c5sync", "root")
        ssigs, _ = impl.sign_batch(sync_sks, [sync_root] * 512)
        sync_agg = impl.aggregate(ssigs)
        log("rank %d: C5 data (%d partials + 512-key sync aggregate) in %.1fs" % (rank, n5, time.time() - t0))
        d_pk5, d_sig5, d_msg5 = u8(pks5), u8(sigs5), u8(roots5)
        d_midx5 = torch.tensor(midx5, dtype=torch.int32).to(dev)
        d_off5 = torch.arange(0, 32 * (len(roots5) + 1), 32, dtype=torch.int64).to(dev)
        d_st5 = torch.full((n5,), -7, dtype=torch.int32, device=dev)
        d_spk = u8(sync_pks)
        d_skoff = torch.tensor([0, 512], dtype=torch.int64).to(dev)
        d_ssig, d_smsg = u8([sync_agg]), u8([sync_root])
        d_smoff = torch.tensor([0, 32], dtype=torch.int64).to(dev)
        d_sst = torch.full((1,), -7, dtype=torch.int32, device=dev)
        seed5 = os.urandom(32)
        node5 = [None]
        n5_node = 4 * args.rlc_node_validators + 128
        c5_rows = [4 * (shard_range(V, r, world)[1] - shard_range(V, r, world)[0])
                   + 4 * (shard_range(32, r, world)[1] - shard_range(32, r, world)[0]) for r in range(world)]
        c5_max = max(c5_rows)

        c5_fav = os.environ.get("BENCH_C5_FAV", "1") == "1"  # 0: the RLC part alone (A/B of the overlap)
        s_fav = torch.cuda.Stream(device=dev)  # a stream of its own: on the RLC's stream it would run before it
        sp_fav = ctypes.c_void_p(s_fav.cuda_stream)

        def c5step():
            if rank == 0 and c5_fav:  # on its own stream, overlapping the RLC
                rc = lib.hipbls_verify_aggregate_batch_device(d_spk.data_ptr(), 512, d_skoff.data_ptr(), 1,
                                                              d_ssig.data_ptr(), d_smsg.data_ptr(), d_smoff.data_ptr(),
                                                              d_sst.data_ptr(), sp_fav)
                assert rc == 0
            rc = lib.hipbls_batch_verify_rlc_device(d_pk5.data_ptr(), d_sig5.data_ptr(), d_midx5.data_ptr(), n5,
                                                    d_msg5.data_ptr(), d_off5.data_ptr(), len(roots5), seed5,
                                                    d_st5.data_ptr(), sp)
            assert rc == 0
            if world > 1:
                node5[0] = gather_bitmap_rows(d_st5, c5_max)

        c5step()
        torch.cuda.synchronize()
        t5 = timed_loop(c5step, args.rlc_steps, dev, barrier, world)
        torch.cuda.synchronize()
        assert {i for i, x in enumerate(d_st5.cpu().tolist()) if x != 0} == bad5, "C5 bitmap mismatch"
        if rank == 0 and c5_fav:
            assert d_sst.cpu().tolist() == [0], "sync-committee FastAggregateVerify failed"
        # the slot when AUTO retries its batch-wide check (once every RLC_AUTO_PERIOD calls of a stream with invalid
        # partials), and the average over that period
        impl.set_rlc_mode(RLC_BATCH)
        c5step()
        torch.cuda.synchronize()
        t5b = timed_loop(c5step, args.rlc_steps, dev, barrier, world)
        torch.cuda.synchronize()
        impl.set_rlc_mode(RLC_AUTO)
        assert {i for i, x in enumerate(d_st5.cpu().tolist()) if x != 0} == bad5, "C5 bitmap mismatch (batch)"
        t5k = None
        if args.keys:  # the slot as charon runs it: every partial's key from the resident pubshare table (patch 0004)
            table5 = list(dict.fromkeys(pks5))
            pos5 = {k: j for j, k in enumerate(table5)}
            assert set(impl.load_pubshares(table5)) <= {0}
            d_k5 = torch.tensor([pos5[p] for p in pks5], dtype=torch.int32).to(dev)

            def c5kstep():
                if rank == 0 and c5_fav:
                    rc = lib.hipbls_verify_aggregate_batch_device(d_spk.data_ptr(), 512, d_skoff.data_ptr(), 1,
                                                                  d_ssig.data_ptr(), d_smsg.data_ptr(),
                                                                  d_smoff.data_ptr(), d_sst.data_ptr(), sp_fav)
                    assert rc == 0
                rc = lib.hipbls_batch_verify_rlc_keys_device(d_k5.data_ptr(), d_sig5.data_ptr(), d_midx5.data_ptr(), n5,
                                                             d_msg5.data_ptr(), d_off5.data_ptr(), len(roots5), seed5,
                                                             d_st5.data_ptr(), sp)
                assert rc == 0

            impl.set_rlc_mode(RLC_WINDOWS)  # the windows regime of a stream with invalid partials, as C4 (i) is timed
            c5kstep()
            torch.cuda.synchronize()
            t5k = timed_loop(c5kstep, args.rlc_steps, dev, barrier, world)
            torch.cuda.synchronize()
            impl.set_rlc_mode(RLC_AUTO)
            assert {i for i, x in enumerate(d_st5.cpu().tolist()) if x != 0} == bad5, "C5 bitmap mismatch (table)"
            del d_k5
        if world > 1:  # node-wide failure count == construction
            rows = node5[0]
            fails = sum(int((~unpack_bitmap(rows[r], c5_rows[r])).sum()) for r in range(world))
            assert fails == len(c4_node_bad("c4i", V, 4096)) + len(c4_node_bad("c5p", 32, 128)), "C5 node bitmap"
        c5 = {"workload": "C5 (BASELINE configs[4]): RLC BatchVerify of the C4(i) node batch (%d validators x 4, one "
                          "root each) + 32 validators x 4 proposer partials (own roots), ~1%% corrupted, sliced over "
                          "the ranks by validator index, with a 512-key sync-committee FastAggregateVerify (hash-to-G2 "
                          "of its root) overlapped on rank 0" % args.rlc_node_validators,
              "node_partials": n5_node, "partials_this_gpu": n5, "ms_per_slot": round(1000 * t5 / args.rlc_steps, 3),
              "verified_partial_sigs_per_s": round(n5_node * args.rlc_steps / t5, 1),
              "sync_aggregate_verifies_per_s": round(args.rlc_steps / t5, 3),
              "failed_batch_check_ms_per_slot": round(1000 * t5b / args.rlc_steps, 3),
              "auto_mode_amortized_ms_per_slot": round(1000 * ((RLC_AUTO_PERIOD - 1) * t5 + t5b)
                                                       / (RLC_AUTO_PERIOD * args.rlc_steps), 3),
              "ms_per_slot_pubshare_table": round(1000 * t5k / args.rlc_steps, 3) if t5k else None}
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
            "data": "synthetic: seeded share keys, distinct 32-byte roots, ~1% corrupted (wrong root / swapped "
                    "share / flipped sig bit); signatures made by the engine's own sign kernel; every item a function "
                    "of (seed, global index), each rank builds its shard_range slice of the node batch",
            "config": {"workload": "C2 (BASELINE.json configs[1]): individual tbls.Verify of %d partial sigs per GPU, "
                                   "distinct messages" % args.n,
                       "items_per_gpu": args.n, "node_items": n_node,
                       "parallelism": "shard-by-validator-index x %d (RCCL all-gather of the verify bitmaps)" % world},
            "build_src_sha": build_src,
            "pairings_per_s": round(2 * value, 1),
            "drop_in_latency": latency,
            "host_path": host_path,
            "verified_partial_sigs_per_s_pubshare_table": round(keys_rate, 1) if keys_rate else None,
            "threshold_aggregates_per_s": round(tagg, 1) if tagg else None,
            "threshold_aggregates_per_s_two_streams": round(tagg2, 1) if tagg2 else None,
            "threshold_aggregate_kernel_avg_ms": tagg_kms or None,
            "threshold_aggregate_roofline": tagg_roofline,
            "threshold_aggregate_workload": "C3: %d validators per GPU x 7-of-10 Lagrange in G2 + Verify of each "
                                            "aggregate (hipbls_threshold_aggregate_verify_batch_device, sigagg in one "
                                            "call); aggregates and bitmap all-gathered" % args.tagg_groups
            if tagg else None,
        }
        if c5:
            out["full_slot_mix"] = c5
        if rlc:
            out["rlc_batch_verify"] = dict(rlc, workload="C4 (BASELINE configs[3]): the %d-validator x 4-partial node "
                                                        "batch sliced over %d GPU(s) by validator index (strong "
                                                        "scaling), items grouped by validator, ~1%% corrupted (i, ii) "
                                                        "or all valid (i_all_valid, ii_all_valid: decided by the "
                                                        "batch-wide Pippenger check of rlcb.h alone; ii with one G1 "
                                                        "MSM per committee root, g1msm.h), windows of 8 items for "
                                                        "the rest, per-item bitmap == tbls.Verify, node bitmap "
                                                        "all-gathered" % (args.rlc_node_validators, world))
        k_ms = avg_ms.value
        if k_ms > 0:
            achieved = FPMUL_PER_VERIFY * MADS_PER_FPMUL * n / (k_ms * 1e-3) / 1e12
            pmc = pmc_summary()
            out["roofline"] = {
                "bound": "valu-int (32x32->64 v_mad_u64_u32; no HBM or MFMA bound: ~190 B in per verify)",
                "kernel": "k_verify_fused",
                "achieved": round(achieved, 3),
                "peak": MAD_PEAK_T,
                "unit": "Tmad/s",
                "frac": round(achieved / MAD_PEAK_T, 4),
                "traffic": pmc.get("hbm_bytes_per_launch"),
                "traffic_ratio": pmc.get("traffic_ratio"),
                "valu_util": pmc.get("valu_util"),
                "wait_any_frac": pmc.get("wait_any_frac"),
                "pmc_source": pmc.get("source"),
                "pmc_taken_at": pmc.get("taken_at"),
                "valu_insts_per_wave": pmc.get("valu_insts_per_wave"),
                "mad_insts_per_wave": pmc.get("int64_valu_insts_per_wave"),
                "algorithmic_unit": "%d Fp-mul-equivalents x %d MADs per verify" % (FPMUL_PER_VERIFY, MADS_PER_FPMUL),
                "kernel_avg_ms": round(k_ms, 3),
                "kernel_launches": int(launches.value),
            }
            # the attainable rate of this arithmetic on this chip: the shipped product
            # routines alone on every SIMD at the kernel's occupancy, measured by charon_amd/tools/ceiling_probe.hip
            ceil = attainable_products()
            if ceil:
                got = FPMUL_PER_VERIFY * n / (k_ms * 1e-3) / 1e9
                out["roofline"]["attainable"] = {
                    "g_products_per_s": ceil["attainable_g_products_per_s_one_wave"],
                    "achieved_g_products_per_s": round(got, 2),
                    "frac": round(got / ceil["attainable_g_products_per_s_one_wave"], 4),
                    "note": "products/s of the product routines alone, one wave per SIMD (the kernel's occupancy); the "
                            "nominal peak assumes every lane issues one 32x32->64 MAD per clock at 2.4 GHz",
                    "source": ceil["source_file"]}
        if world == 1 and args.cpu_sample > 0:
            out["cpu_baseline"] = cpu_baseline(impl, (pks, roots, sigs, bad), args.cpu_sample, random.Random(SEED))
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
