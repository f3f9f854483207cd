"""The C++ CPU baseline (tests/native/cpu_baseline.cpp: ops.h at -O3 with a 6 x 64-bit Montgomery product,
one thread per core) must give the oracle's statuses and bytes before bench.py times it as cpu_baseline."""
import ctypes
import json
import os

import pytest

from tests import hostlib

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def cb():
    hostlib.build_cpu_baseline()
    return hostlib.cpu_baseline_lib()


@pytest.fixture(scope="module")
def fx():
    with open(os.path.join(GOLDEN, "fixtures.json")) as f:
        return json.load(f)


def test_cpu_baseline_verify_matches_fixtures(cb, fx):
    cases = fx["verify"]
    n = len(cases)
    msgs = [bytes.fromhex(c["msg"]) for c in cases]
    offs, acc = [0], 0
    for m in msgs:
        acc += len(m)
        offs.append(acc)
    st = (ctypes.c_int32 * n)()
    cb.cb_verify_batch(b"".join(bytes.fromhex(c["pk"]) for c in cases), b"".join(msgs),
                       (ctypes.c_uint64 * (n + 1))(*offs), b"".join(bytes.fromhex(c["sig"]) for c in cases), n, st, 4)
    assert list(st) == [c["status"] for c in cases]


def test_cpu_baseline_threshold_aggregate_matches_fixtures(cb, fx):
    groups = fx["threshold_aggregate"]
    sigs, ids, offs = [], [], [0]
    for g in groups:
        for k, v in g["parts"].items():
            ids.append(int(k))
            sigs.append(bytes.fromhex(v))
        offs.append(len(ids))
    G = len(groups)
    out = ctypes.create_string_buffer(96 * G)
    st = (ctypes.c_int32 * G)()
    cb.cb_threshold_aggregate_batch(b"".join(sigs), (ctypes.c_int64 * max(len(ids), 1))(*ids),
                                    (ctypes.c_uint64 * (G + 1))(*offs), G, out, st, 2)
    for g, grp in enumerate(groups):
        if grp["err"] is None:
            assert st[g] == 0 and out.raw[96 * g:96 * g + 96].hex() == grp["out"], grp["note"]
        else:
            assert st[g] != 0, grp["note"]
