"""Verify latency / throughput against batch size, one lane per check vs a lane pair per check.

Prints one line per (n, layout): ms per call and verifies/s, from hipbls_verify_batch_device on resident inputs
(C2-shaped: distinct 32-byte roots, 1% corrupted).  Used to place the HIPBLS_PAIR_AUTO crossover
(kLg2MaxVerify in charon_amd/csrc/hipbls.hip); the output is kept under profiles/.
"""
import ctypes
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch

    import bench
    from charon_amd.tbls import PAIR_LANES, PAIR_QUADS, PAIR_SINGLE, HipBLS, load_library
    sizes = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else
                              "1,64,1024,4096,10000,16384,24576,32768").split(",")]
    dev = torch.device("cuda", 0)
    impl = HipBLS(device=0)
    lib = load_library()
    nmax = max(sizes)
    pks, roots, sigs, bad = bench.make_c2(impl, bench.share_keys(impl, 4096, "c2"), 0, nmax)
    d_pk = torch.frombuffer(bytearray(b"".join(pks)), dtype=torch.uint8).to(dev)
    d_sig = torch.frombuffer(bytearray(b"".join(sigs)), dtype=torch.uint8).to(dev)
    d_msg = torch.frombuffer(bytearray(b"".join(roots)), dtype=torch.uint8).to(dev)
    d_off = torch.arange(0, 32 * (nmax + 1), 32, dtype=torch.int64).to(dev)
    d_st = torch.full((nmax,), -1, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)
    rows = []
    for n in sizes:
        for mode, name in ((PAIR_SINGLE, "single"), (PAIR_LANES, "lanes"), (PAIR_QUADS, "quads")):
            impl.set_pair_mode(mode)
            reps = 3 if n >= 4096 else 10

            def call():
                rc = lib.hipbls_verify_batch_device(d_pk.data_ptr(), d_msg.data_ptr(), d_off.data_ptr(),
                                                    d_sig.data_ptr(), n, d_st.data_ptr(),
                                                    ctypes.c_void_p(stream.cuda_stream))
                assert rc == 0

            call()
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for _ in range(reps):
                call()
            torch.cuda.synchronize(dev)
            dt = (time.perf_counter() - t0) / reps
            st = d_st[:n].cpu().tolist()
            assert {i for i, s in enumerate(st) if s != 0} == {i for i in bad if i < n}, (n, name)
            row = {"n": n, "layout": name, "ms_per_call": round(1000 * dt, 3), "verifies_per_s": round(n / dt, 1)}
            rows.append(row)
            print(json.dumps(row), flush=True)
    impl.set_pair_mode(0)


if __name__ == "__main__":
    main()
