"""Drop-in latency and small-batch Verify time per pairing layout (PAIR_QUADS vs PAIR_OCTETS, include/hipbls.h):
p50 / p90 of synchronous n = 1 calls through the submission queue (hipbls_verify, the parsigex loop shape) and of
direct n = 1 batch calls, then ms per batch call at growing n.  Prints one JSON object.  GPU only."""
import json
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from charon_amd.tbls import PAIR_AUTO, PAIR_OCTETS, PAIR_QUADS, HipBLS  # noqa: E402

R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001


def pct(xs, q):
    xs = sorted(xs)
    return round(1000 * xs[min(len(xs) - 1, int(q * len(xs)))], 3)


def main():
    impl = HipBLS()
    rng = random.Random(7)
    N = 8192
    sks = [rng.randrange(1, R_ORDER).to_bytes(32, "big") for _ in range(N)]
    pks, st = impl.secret_to_public_key_batch(sks)
    assert set(st) == {0}
    msgs = [rng.randbytes(32) for _ in range(N)]
    sigs, st = impl.sign_batch(sks, msgs)
    assert set(st) == {0}
    out = {}
    for name, mode in (("quads", PAIR_QUADS), ("octets", PAIR_OCTETS)):
        impl.set_pair_mode(mode)
        assert impl.verify_queued(pks[0], msgs[0], sigs[0]) == 0
        q = []
        for j in range(60):
            a = time.perf_counter()
            assert impl.verify_queued(pks[j], msgs[j], sigs[j]) == 0
            q.append(time.perf_counter() - a)
        d = []
        for j in range(60):
            a = time.perf_counter()
            assert impl.batch_verify_status([pks[j]], [msgs[j]], [sigs[j]]) == [0]
            d.append(time.perf_counter() - a)
        sweep = {}
        for n in (16, 256, 1024, 4096, 8192):
            impl.batch_verify_status(pks[:n], msgs[:n], sigs[:n])
            a = time.perf_counter()
            for _ in range(3):
                got = impl.batch_verify_status(pks[:n], msgs[:n], sigs[:n])
            sweep[n] = round(1000 * (time.perf_counter() - a) / 3, 3)
            assert got == [0] * n
        out[name] = {"queued_n1_p50_ms": pct(q, 0.5), "queued_n1_p90_ms": pct(q, 0.9), "queued_n1_min_ms": pct(q, 0),
                     "direct_n1_p50_ms": pct(d, 0.5), "ms_per_batch_call": sweep}
        print(name, out[name], file=sys.stderr, flush=True)
    impl.set_pair_mode(PAIR_AUTO)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
