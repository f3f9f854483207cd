"""n = 1 Verify with the replica race off (1) and on (8), in alternating blocks of direct batch calls: host-side p50
per block, and (under rocprofv3 --kernel-trace) the octet kernels' durations per block, in launch order.
Usage: python scripts/race_trace.py [calls_per_block] [replicas per block, e.g. 1,8,1,8,2,4] > out.json"""
import json
import statistics
import sys
import time

import bench
from charon_amd.tbls import HipBLS

K = int(sys.argv[1]) if len(sys.argv) > 1 else 100
impl = HipBLS()
pks, roots, sigs, bad = bench.make_c2(impl, bench.share_keys(impl, 64, "race"), 0, 64)
good = [i for i in range(64) if i not in bad]
for i in good[:8]:
    assert impl.batch_verify_status([pks[i]], [roots[i]], [sigs[i]]) == [0]
out = []
BLOCKS = tuple(int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "1,8,1,8,2,4").split(","))
for b, reps in enumerate(BLOCKS):
    impl.lib.hipbls_set_latency_replicas(reps)
    ts = []
    for k in range(K):
        i = good[k % len(good)]
        t0 = time.perf_counter()
        st = impl.batch_verify_status([pks[i]], [roots[i]], [sigs[i]])
        ts.append((time.perf_counter() - t0) * 1e3)
        assert st == [0]
    ts.sort()
    out.append({"block": b, "replicas": reps, "calls": K, "p50_ms": round(statistics.median(ts), 3),
                "p10_ms": round(ts[K // 10], 3), "p90_ms": round(ts[9 * K // 10], 3), "min_ms": round(ts[0], 3)})
    print(json.dumps(out[-1]), flush=True)
impl.lib.hipbls_set_latency_replicas(8)
