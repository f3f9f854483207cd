"""Experiment (not the product): does the n = 1 octet check's duration depend on the XCD its workgroup lands on?

Run with HIPBLS_LIB=charon_amd/libhipbls_xcdprobe.so, a build with -DBLS_LQ8_XCD_PROBE=1 (charon_amd/build.py
build(out=..., extra=[...])), where k_verify_pair_lq8 runs every workgroup once per XCD (8x the grid) and each copy
records its XCC id and start / end (s_memrealtime, 100 MHz).  Prints per call the eight copies' durations by XCC, and
per XCC the mean over the calls.
"""
import ctypes
import json
import sys

import bench
from charon_amd.tbls import HipBLS, PAIR_OCTETS


def main(calls=24):
    impl = HipBLS()
    impl.set_pair_mode(PAIR_OCTETS)
    lib = impl.lib
    lib.hipbls_debug_xcd_probe.argtypes = [ctypes.POINTER(ctypes.c_uint64)]
    pks, roots, sigs, bad = bench.make_c2(impl, bench.share_keys(impl, 64, "xcdp"), 0, calls)
    per = {}
    rows = []
    buf = (ctypes.c_uint64 * 256)()
    for j in range(calls):
        st = impl.batch_verify_status([pks[j]], [roots[j]], [sigs[j]])
        assert (st[0] != 0) == (j in bad)
        assert lib.hipbls_debug_xcd_probe(buf) == 0
        rec = {}
        for b in range(8):
            x, t0, t1 = buf[4 * b], buf[4 * b + 1], buf[4 * b + 2]
            rec[int(x)] = round((t1 - t0) / 100.0 / 1000.0, 3)  # ms
            per.setdefault(int(x), []).append((t1 - t0) / 1e5)
        rows.append(rec)
        print(json.dumps({"call": j, "ms_by_xcc": rec}), flush=True)
    print(json.dumps({"mean_ms_by_xcc": {k: round(sum(v) / len(v), 3) for k, v in sorted(per.items())},
                      "min_ms_by_xcc": {k: round(min(v), 3) for k, v in sorted(per.items())},
                      "max_ms_by_xcc": {k: round(max(v), 3) for k, v in sorted(per.items())}}), flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 24)
