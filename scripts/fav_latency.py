"""Probe (round 6): latency of one sync-committee FastAggregateVerify (512 keys, one group) on an idle GPU through the
host call, p50 over 30 calls; HIPBLS_LIB selects an A/B build (scripts/gpu.sh py: step)."""
import hashlib
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from charon_amd.tbls import HipBLS  # noqa: E402

impl = HipBLS()
sks = [(int.from_bytes(hashlib.sha256(b"fav%d" % k).digest(), "big") % (1 << 250) + 1).to_bytes(32, "big")
       for k in range(512)]
pks, _ = impl.secret_to_public_key_batch(sks)
root = hashlib.sha256(b"sync root").digest()
sigs, _ = impl.sign_batch(sks, [root] * 512)
agg = impl.aggregate(sigs)
group = [(pks, agg, root)]
assert impl.batch_verify_aggregate_status(group) == [0]
ts = []
for _ in range(30):
    t0 = time.perf_counter()
    st = impl.batch_verify_aggregate_status(group)
    ts.append((time.perf_counter() - t0) * 1e3)
    assert st == [0]
print(json.dumps({"lib": os.environ.get("HIPBLS_LIB", "in-tree"), "fav_512_p50_ms": round(statistics.median(ts), 3),
                  "min_ms": round(min(ts), 3)}))
