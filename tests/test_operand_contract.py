"""The device product routines' operand contract, checked on the host (round 6).

The carry-eliding Montgomery routines (charon_amd/tools/gen_fp_asm.py _comba) skip a carry capture where the column
bound proves the accumulator cannot overflow, which holds for operands below 2^382; the Fp2 square and the modular
add / sub blocks take canonical operands.  Every product operand is canonical or a lazy sum below 2p (field.h
fp_add_lazy / fp_sub_lazy), but on the host those lazy sums are normally reduced, so the host tests never see the
device's values.  The BLS_CONTRACT_CHECK build of the same per-lane code (tests/native/host_ops.cpp) keeps them
unreduced as the device does and counts every operation whose operands break its routine's contract.  Here the host
arithmetic suites (every curve, tower, pairing, hash, RLC window / fallback / batch-wide and sigagg path they drive)
run against that build in a subprocess, and the count must stay 0.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SUITES = ["tests/test_host_arith.py", "tests/test_rlc_host.py", "tests/test_rlcb_host.py", "tests/test_glv.py"]


def test_host_suites_respect_the_device_operand_contract(tmp_path):
    out = tmp_path / "contract.json"
    env = dict(os.environ, HIPBLS_HOST_CONTRACT="1", HIPBLS_HOST_CONTRACT_OUT=str(out))
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-m", "not gpu", "-p", "no:cacheprovider"]
                       + SUITES, cwd=ROOT, env=env, capture_output=True, text=True, timeout=1200)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    got = json.loads(out.read_text())
    assert got["violations"] == 0, got
    assert got["lazy_operands"] > 1000, got  # the suites do reach the products with unreduced operands


def test_contract_build_counts_a_violation(tmp_path):
    """The check is live: a product of two values at 2^382 - 1 (outside the contract) is counted."""
    env = dict(os.environ, HIPBLS_HOST_CONTRACT="1")
    code = ("import ctypes, sys; sys.path.insert(0, %r); from tests import hostlib; L = hostlib.lib(); "
            "a = ((1 << 382) - 1).to_bytes(48, 'little'); o = (ctypes.c_uint32 * 12)(); "
            "L.ht_fp_mul_raw(a, a, o); print(L.ht_contract_violations(), L.ht_contract_first().decode())") % ROOT
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    n, what = r.stdout.split(" ", 1)
    assert int(n) >= 1 and "fp_mul" in what
