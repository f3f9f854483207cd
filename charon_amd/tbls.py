"""Host-side mirror of charon's tbls.Implementation backed by the HIP engine (libhipbls.so).

charon's Go interface (/root/reference/tbls/tbls.go:28-69) has 11 methods; `HipBLS` exposes the
same methods with the same argument meaning and the same error strings as tbls.Herumi
(/root/reference/tbls/herumi.go), plus the batched entry points the north star adds
(`batch_verify`, `batch_threshold_aggregate`).  Every curve operation runs on the GPU through the
C-ABI in include/hipbls.h; there is no CPU fallback: constructing `HipBLS` without the built
library or without a GPU raises.

The Go binding a charon maintainer would add (tbls/hipbls, cgo) is in INTEGRATION.md; this module
is the same boundary seen from Python, used by the parity tests and bench.py.
"""

from __future__ import annotations

import ctypes
import os
import secrets
from typing import Dict, List, Mapping, Optional, Sequence, Tuple

R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001

OK, ERR_PUBKEY, ERR_SIGNATURE, ERR_VERIFY, ERR_SECRET, ERR_COMBINE, ERR_ZERO_SIG = 0, 1, 2, 3, 4, 5, 6
INFINITY_G2 = b"\xc0" + bytes(95)  # compressed point at infinity (the empty Aggregate, herumi.go:220-242)
ERR_ARG, ERR_DEVICE = 16, 17
PAIR_AUTO, PAIR_SINGLE, PAIR_LANES, PAIR_QUADS, PAIR_OCTETS = 0, 1, 2, 3, 4  # hipbls_set_pair_mode (hipbls.h)
RLC_AUTO, RLC_WINDOWS, RLC_BATCH = 0, 1, 2     # hipbls_rlc_set_mode: batch-wide check policy (include/hipbls.h)

# tbls/herumi.go error strings by status code
VERIFY_ERRORS = {
    ERR_PUBKEY: "cannot set compressed public key in Herumi format",
    ERR_SIGNATURE: "cannot unmarshal signature into Herumi signature",
    ERR_VERIFY: "signature not verified",
}


class TBLSError(Exception):
    """A tbls error: message is the string tbls.Herumi returns for the same input."""


class DeviceError(RuntimeError):
    """HIP runtime failure.  Never converted into a 'verified' result."""


# HIPBLS_LIB: another build of the same library (A/B measurements of compile-time variants); default in-tree
_LIB_PATH = os.environ.get("HIPBLS_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libhipbls.so")
_lib = None


def load_library(path: str = _LIB_PATH) -> ctypes.CDLL:
    """Load libhipbls.so and declare the C-ABI; raises if it is missing (no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError("hipbls native library not built: %s (run __graft_entry__.build())" % path)
    lib = ctypes.CDLL(path)
    u8p = ctypes.c_char_p
    u64 = ctypes.c_uint64
    i32p = ctypes.POINTER(ctypes.c_int32)
    u64p = ctypes.POINTER(ctypes.c_uint64)
    u32p = ctypes.POINTER(ctypes.c_uint32)
    i64p = ctypes.POINTER(ctypes.c_int64)
    vp = ctypes.c_void_p
    sig = {
        "hipbls_current_device": ([], ctypes.c_int),
        "hipbls_init_devices": ([ctypes.POINTER(ctypes.c_int32), ctypes.c_uint32], ctypes.c_int),
        "hipbls_device_slots": ([ctypes.POINTER(ctypes.c_int32), ctypes.c_uint32], ctypes.c_int),
        "hipbls_plan_ranges": ([u64, ctypes.c_uint32, u32p, u64p], ctypes.c_int),
        "hipbls_queue_keyed_batches": ([u64p], ctypes.c_int),
        "hipbls_deserialize_status": ([u8p, u64, ctypes.c_int32, i32p], ctypes.c_int),
        "hipbls_set_timing": ([ctypes.c_int], ctypes.c_int),
        "hipbls_set_pair_mode": ([ctypes.c_int], ctypes.c_int),
        "hipbls_rlc_set_mode": ([ctypes.c_int], ctypes.c_int),
        "hipbls_rlc_set_g1_msm_min": ([ctypes.c_uint32], ctypes.c_int),
        "hipbls_threshold_aggregate_verify_batch": ([u8p, i64p, u64p, u64, u8p, u8p, u64p, u8p, i32p, i32p],
                                                    ctypes.c_int),
        "hipbls_threshold_aggregate_verify_batch_device": ([vp, vp, vp, u64, u64, vp, vp, vp, vp, vp, vp, vp],
                                                           ctypes.c_int),
        "hipbls_rlc_batch_stats": ([u64p, u64p, i32p], ctypes.c_int),
        "hipbls_verify": ([u8p, u8p, u64, u8p, i32p], ctypes.c_int),
        "hipbls_verify_submit": ([u8p, u8p, u64, u8p, u64p], ctypes.c_int),
        "hipbls_verify_wait": ([u64, i32p], ctypes.c_int),
        "hipbls_queue_config": ([u64, ctypes.c_uint32], ctypes.c_int),
        "hipbls_queue_stats": ([u64p, u64p], ctypes.c_int),
        "hipbls_verify_signed_data_batch": ([u8p, u8p, u8p, u8p, u64, i32p], ctypes.c_int),
        "hipbls_aggregate_device": ([vp, u64, vp, vp, vp], ctypes.c_int),
        "hipbls_hcache_config": ([u64], ctypes.c_int),
        "hipbls_hcache_stats": ([u64p, u64p, u64p], ctypes.c_int),
        "hipbls_abi_version": ([], ctypes.c_int),
        "hipbls_init": ([ctypes.c_int], ctypes.c_int),
        "hipbls_device_count": ([], ctypes.c_int),
        "hipbls_device_streams": ([ctypes.c_int], ctypes.c_int),
        "hipbls_last_error": ([], ctypes.c_char_p),
        "hipbls_verify_batch": ([u8p, u8p, u64p, u8p, u64, i32p], ctypes.c_int),
        "hipbls_threshold_aggregate_batch": ([u8p, i64p, u64p, u64, u8p, i32p], ctypes.c_int),
        "hipbls_sign_batch": ([u8p, u8p, u64p, u64, u8p, i32p], ctypes.c_int),
        "hipbls_secret_to_public_key_batch": ([u8p, u64, u8p, i32p], ctypes.c_int),
        "hipbls_verify_aggregate": ([u8p, u64, u8p, u8p, u64, i32p], ctypes.c_int),
        "hipbls_aggregate": ([u8p, u64, u8p, i32p], ctypes.c_int),
        "hipbls_threshold_split": ([u8p, u8p, ctypes.c_uint32, ctypes.c_uint32, u8p, i32p], ctypes.c_int),
        "hipbls_recover_secret": ([u8p, i64p, ctypes.c_uint32, u8p, i32p], ctypes.c_int),
        "hipbls_verify_batch_device": ([vp, vp, vp, vp, u64, vp, vp], ctypes.c_int),
        "hipbls_threshold_aggregate_batch_device": ([vp, vp, vp, u64, u64, vp, vp, vp], ctypes.c_int),
        "hipbls_sign_batch_device": ([vp, vp, vp, u64, vp, vp, vp], ctypes.c_int),
        "hipbls_secret_to_public_key_batch_device": ([vp, u64, vp, vp, vp], ctypes.c_int),
        "hipbls_batch_verify_rlc": ([u8p, u8p, u32p, u64, u8p, u64p, u64, u8p, i32p], ctypes.c_int),
        "hipbls_batch_verify_rlc_device": ([vp, vp, vp, u64, vp, vp, u64, u8p, vp, vp], ctypes.c_int),
        "hipbls_rlc_stats": ([u64p, u64p, u64p], ctypes.c_int),
        "hipbls_pubshare_table_load": ([u8p, u64, i32p], ctypes.c_int),
        "hipbls_verify_aggregate_batch": ([u8p, u64p, u64, u8p, u8p, u64p, i32p], ctypes.c_int),
        "hipbls_verify_aggregate_batch_device": ([vp, u64, vp, u64, vp, vp, vp, vp, vp], ctypes.c_int),
        "hipbls_pubshare_table_size": ([u64p], ctypes.c_int),
        "hipbls_verify_batch_keys": ([u32p, u8p, u64p, u8p, u64, i32p], ctypes.c_int),
        "hipbls_batch_verify_rlc_keys": ([u32p, u8p, u32p, u64, u8p, u64p, u64, u8p, i32p], ctypes.c_int),
        "hipbls_verify_batch_keys_device": ([vp, vp, vp, vp, u64, vp, vp], ctypes.c_int),
        "hipbls_batch_verify_rlc_keys_device": ([vp, vp, vp, u64, vp, vp, u64, u8p, vp, vp], ctypes.c_int),
        "hipbls_kernel_timing": ([ctypes.c_char_p, ctypes.POINTER(ctypes.c_double), u64p], ctypes.c_int),
        "hipbls_kernel_timing_reset": ([], ctypes.c_int),
        "hipbls_scratch_budget": ([ctypes.c_int, u64p, u64p, u64p, ctypes.POINTER(ctypes.c_uint32)], ctypes.c_int),
        "hipbls_stream_joins": ([u64p], ctypes.c_int),
        "hipbls_kernel_names": ([], ctypes.c_char_p),
        "hipbls_queue_worker_stats": ([u64p, u64p], ctypes.c_int),
        "hipbls_set_latency_replicas": ([ctypes.c_uint32], ctypes.c_int),
        "hipbls_build_id": ([], ctypes.c_char_p),
    }
    for name, (args, res) in sig.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    _lib = lib
    return lib


def exported_symbols() -> List[str]:
    return [
        "hipbls_abi_version", "hipbls_init", "hipbls_device_count", "hipbls_last_error",
        "hipbls_verify_batch", "hipbls_threshold_aggregate_batch", "hipbls_sign_batch",
        "hipbls_secret_to_public_key_batch", "hipbls_verify_aggregate", "hipbls_aggregate",
        "hipbls_threshold_split", "hipbls_recover_secret", "hipbls_verify_batch_device",
        "hipbls_threshold_aggregate_batch_device", "hipbls_sign_batch_device",
        "hipbls_secret_to_public_key_batch_device", "hipbls_kernel_timing", "hipbls_kernel_timing_reset",
        "hipbls_batch_verify_rlc", "hipbls_batch_verify_rlc_device", "hipbls_rlc_stats",
        "hipbls_pubshare_table_load", "hipbls_pubshare_table_size", "hipbls_verify_aggregate_batch",
        "hipbls_verify_aggregate_batch_device", "hipbls_verify_batch_keys",
        "hipbls_batch_verify_rlc_keys", "hipbls_verify_batch_keys_device", "hipbls_batch_verify_rlc_keys_device",
        "hipbls_current_device", "hipbls_set_timing", "hipbls_verify", "hipbls_verify_submit", "hipbls_verify_wait",
        "hipbls_queue_config", "hipbls_queue_stats", "hipbls_verify_signed_data_batch", "hipbls_aggregate_device",
        "hipbls_hcache_config", "hipbls_hcache_stats", "hipbls_set_pair_mode",
        "hipbls_rlc_set_mode", "hipbls_rlc_batch_stats", "hipbls_threshold_aggregate_verify_batch",
        "hipbls_threshold_aggregate_verify_batch_device", "hipbls_init_devices", "hipbls_device_slots",
        "hipbls_plan_ranges", "hipbls_queue_keyed_batches", "hipbls_deserialize_status", "hipbls_device_streams",
        "hipbls_rlc_set_g1_msm_min", "hipbls_scratch_budget", "hipbls_stream_joins", "hipbls_kernel_names",
        "hipbls_queue_worker_stats", "hipbls_set_latency_replicas", "hipbls_build_id",
    ]


def build_id() -> dict:
    """The digests compiled into the loaded library (hipbls_build_id): {"src": sha256, "flags": sha256}."""
    raw = load_library().hipbls_build_id().decode()
    return dict(kv.split("=", 1) for kv in raw.split())


def plan_ranges(n: int, parts: int, run_keys: Optional[Sequence[int]] = None) -> List[int]:
    """The library's batch split (hipbls_plan_ranges; host code, no GPU): bounds of `parts` contiguous ranges of n
    items, inner bounds moved to the next change of run key (a validator's partials stay on one device)."""
    lib = load_library()
    b = (ctypes.c_uint64 * (parts + 1))()
    keys = (ctypes.c_uint32 * max(n, 1))(*run_keys) if run_keys is not None else None
    _check(lib.hipbls_plan_ranges(n, parts, keys, b), lib)
    return list(b)


def _check(rc: int, lib) -> None:
    if rc == OK:
        return
    msg = lib.hipbls_last_error()
    msg = msg.decode() if msg else ""
    if rc == ERR_DEVICE:
        raise DeviceError("hipbls device error: " + msg)
    raise ValueError("hipbls invalid argument (rc=%d) %s" % (rc, msg))


def _offsets(msgs: Sequence[bytes]):
    offs = (ctypes.c_uint64 * (len(msgs) + 1))()
    acc = 0
    for i, m in enumerate(msgs):
        offs[i] = acc
        acc += len(m)
    offs[len(msgs)] = acc
    return b"".join(msgs), offs


def _status_array(n: int):
    return (ctypes.c_int32 * max(n, 1))()


def _go_int(idx) -> int:
    """A map[int]... key of the Go API: a signed 64-bit integer (herumi.go:264-271 formats it with strconv.Itoa)."""
    v = int(idx)
    if not -(1 << 63) <= v < (1 << 63):
        raise ValueError("share index outside Go's int range")
    return v


def _check_lengths(name: str, items: Sequence[bytes], size: int) -> None:
    if any(len(x) != size for x in items):
        raise ValueError("%s must be %d bytes each" % (name, size))


class HipBLS:
    """tbls.Implementation on MI355X.  Method names follow tbls.go:28-69 (snake_case)."""

    def __init__(self, device: Optional[int] = None, devices: Optional[Sequence[int]] = None):
        """device: the one GPU of this process (default LOCAL_RANK, or 0).  devices: every GPU this process drives
        (charon's one process per node); batches are split across them (hipbls_init_devices)."""
        self.lib = load_library()
        if devices is not None:
            arr = (ctypes.c_int32 * len(devices))(*devices)
            _check(self.lib.hipbls_init_devices(arr, len(devices)), self.lib)
            return
        if device is None:
            device = int(os.environ.get("LOCAL_RANK", "0"))
        _check(self.lib.hipbls_init(device), self.lib)

    def device_slots(self) -> List[int]:
        """The device of each context the library drives (hipbls_device_slots)."""
        arr = (ctypes.c_int32 * 64)()
        n = self.lib.hipbls_device_slots(arr, 64)
        return list(arr)[:n]

    # ---------------------------------------------------------------- key tooling
    def generate_secret_key(self) -> bytes:
        """herumi.go:59-69 (SetByCSPRNG): uniform secret in [0, r)."""
        while True:
            v = int.from_bytes(secrets.token_bytes(32), "big") & ((1 << 255) - 1)
            if v < R:
                return v.to_bytes(32, "big")

    def generate_insecure_key(self, random) -> bytes:
        """herumi.go:343-360: up to 100 reads of 32 bytes until one deserializes (< r)."""
        for _ in range(100):
            b = random.read(32)
            if int.from_bytes(b, "big") < R:
                return bytes(b)
        raise TBLSError("cannot generate insecure key")

    def secret_to_public_key(self, secret: bytes) -> bytes:
        pk, st = self.secret_to_public_key_batch([secret])
        if st[0] != OK:
            v = int.from_bytes(secret, "big")
            if v >= R:
                raise TBLSError("cannot unmarshal secret into Herumi secret key")
            raise TBLSError("cannot obtain public key from secret")
        return pk[0]

    def secret_to_public_key_batch(self, secrets_: Sequence[bytes]) -> Tuple[List[bytes], List[int]]:
        n = len(secrets_)
        _check_lengths("secret keys", secrets_, 32)
        out = ctypes.create_string_buffer(48 * max(n, 1))
        st = _status_array(n)
        _check(self.lib.hipbls_secret_to_public_key_batch(b"".join(secrets_), n, out, st), self.lib)
        raw = out.raw  # one copy: .raw rebuilds the bytes object on every access
        return [raw[48 * i:48 * i + 48] for i in range(n)], list(st)[:n]

    def _split(self, secret: bytes, total: int, threshold: int, tail: Sequence[bytes]) -> Dict[int, bytes]:
        if int.from_bytes(secret, "big") >= R:
            raise TBLSError("cannot unmarshal bytes into Herumi secret key")
        out = ctypes.create_string_buffer(32 * total)
        st = _status_array(1)
        _check(self.lib.hipbls_threshold_split(secret, b"".join(tail), total, threshold, out, st), self.lib)
        if st[0] != OK:
            raise TBLSError("cannot unmarshal bytes into Herumi secret key")
        raw = out.raw
        return {i + 1: raw[32 * i:32 * i + 32] for i in range(total)}

    def threshold_split(self, secret: bytes, total: int, threshold: int) -> Dict[int, bytes]:
        """herumi.go:134-181: polynomial tail from the CSPRNG."""
        tail = [self.generate_secret_key() for _ in range(threshold - 1)]
        return self._split(secret, total, threshold, tail)

    def threshold_split_insecure(self, secret: bytes, total: int, threshold: int, random) -> Dict[int, bytes]:
        """herumi.go:84-132: polynomial tail from an insecure reader."""
        tail = [self.generate_insecure_key(random) for _ in range(threshold - 1)]
        return self._split(secret, total, threshold, tail)

    def recover_secret(self, shares: Mapping[int, bytes], total: int = 0, threshold: int = 0) -> bytes:
        """herumi.go:183-218."""
        ids = list(shares.keys())
        _check_lengths("shares", [shares[i] for i in ids], 32)
        for i in ids:
            if int.from_bytes(shares[i], "big") >= R:
                raise TBLSError("cannot unmarshal key with into Herumi secret key")
        arr = (ctypes.c_int64 * max(len(ids), 1))(*[_go_int(i) for i in ids])
        out = ctypes.create_string_buffer(32)
        st = _status_array(1)
        _check(self.lib.hipbls_recover_secret(b"".join(shares[i] for i in ids), arr, len(ids), out, st), self.lib)
        if st[0] != OK:
            raise TBLSError("cannot recover full private key from partial keys")
        return out.raw

    # ---------------------------------------------------------------- hot path
    def sign(self, private_key: bytes, data: bytes) -> bytes:
        sigs, st = self.sign_batch([private_key], [data])
        if st[0] != OK:
            raise TBLSError("cannot unmarshal secret into Herumi secret key")
        return sigs[0]

    def sign_batch(self, sks: Sequence[bytes], msgs: Sequence[bytes]) -> Tuple[List[bytes], List[int]]:
        n = len(sks)
        if len(msgs) != n:
            raise ValueError("mismatching lengths")
        _check_lengths("secret keys", sks, 32)
        blob, offs = _offsets(msgs)
        out = ctypes.create_string_buffer(96 * max(n, 1))
        st = _status_array(n)
        _check(self.lib.hipbls_sign_batch(b"".join(sks), blob, offs, n, out, st), self.lib)
        raw = out.raw
        return [raw[96 * i:96 * i + 96] for i in range(n)], list(st)[:n]

    def verify(self, compressed_public_key: bytes, data: bytes, signature: bytes) -> None:
        """herumi.go:285-301: raises TBLSError with the reference's message on failure."""
        st = self.batch_verify_status([compressed_public_key], [data], [signature])[0]
        if st != OK:
            raise TBLSError(VERIFY_ERRORS[st])

    def batch_verify_status(self, pks: Sequence[bytes], msgs: Sequence[bytes], sigs: Sequence[bytes]) -> List[int]:
        n = len(pks)
        if not (len(msgs) == n == len(sigs)):
            raise ValueError("mismatching lengths")
        if any(len(p) != 48 for p in pks) or any(len(s) != 96 for s in sigs):
            raise ValueError("bad key/signature length")
        blob, offs = _offsets(msgs)
        st = _status_array(n)
        _check(self.lib.hipbls_verify_batch(b"".join(pks), blob, offs, b"".join(sigs), n, st), self.lib)
        return list(st)[:n]

    def batch_verify(self, pks, msgs, sigs) -> List[Optional[TBLSError]]:
        """Per-item outcome of Verify: None when valid, else the TBLSError Verify would raise."""
        return [None if s == OK else TBLSError(VERIFY_ERRORS[s]) for s in self.batch_verify_status(pks, msgs, sigs)]

    def batch_verify_rlc_status(self, pks: Sequence[bytes], msgs: Sequence[bytes], sigs: Sequence[bytes],
                                seed: Optional[bytes] = None) -> List[int]:
        """Random-linear-combination BatchVerify: same per-item statuses as batch_verify_status.
        Items sharing a message (all partials of one validator) should be adjacent; the distinct
        messages are hashed once.  seed: 32 bytes of CSPRNG output (drawn here when omitted)."""
        n = len(pks)
        if not (len(msgs) == n == len(sigs)):
            raise ValueError("mismatching lengths")
        if any(len(p) != 48 for p in pks) or any(len(s) != 96 for s in sigs):
            raise ValueError("bad key/signature length")
        if seed is None:
            seed = secrets.token_bytes(32)
        if len(seed) != 32:
            raise ValueError("seed must be 32 bytes")
        pos: Dict[bytes, int] = {}
        table: List[bytes] = []
        idx = (ctypes.c_uint32 * max(n, 1))()
        for i, m in enumerate(msgs):
            m = bytes(m)
            j = pos.get(m)
            if j is None:
                j = pos[m] = len(table)
                table.append(m)
            idx[i] = j
        blob, offs = _offsets(table)
        st = _status_array(n)
        _check(self.lib.hipbls_batch_verify_rlc(b"".join(pks), b"".join(sigs), idx, n, blob, offs, len(table), seed,
                                                st), self.lib)
        return list(st)[:n]

    # ---------------------------------------------------------------- resident pubshare table (§8f.2)
    def load_pubshares(self, pks: Sequence[bytes]) -> List[int]:
        """Decode + subgroup-check every pubshare once (charon: app/app.go:343-381 at startup).
        Returns per-key status (OK / ERR_PUBKEY); keys are then named by their index."""
        n = len(pks)
        if any(len(p) != 48 for p in pks):
            raise ValueError("bad key length")
        st = _status_array(n)
        _check(self.lib.hipbls_pubshare_table_load(b"".join(pks), n, st), self.lib)
        return list(st)[:n]

    def batch_verify_keys_status(self, key_idx: Sequence[int], msgs: Sequence[bytes],
                                 sigs: Sequence[bytes]) -> List[int]:
        """batch_verify_status with pks[i] = loaded table[key_idx[i]]."""
        n = len(key_idx)
        if not (len(msgs) == n == len(sigs)):
            raise ValueError("mismatching lengths")
        _check_lengths("signatures", sigs, 96)
        blob, offs = _offsets(msgs)
        st = _status_array(n)
        idx = (ctypes.c_uint32 * max(n, 1))(*key_idx)
        _check(self.lib.hipbls_verify_batch_keys(idx, blob, offs, b"".join(sigs), n, st), self.lib)
        return list(st)[:n]

    def batch_verify_rlc_keys_status(self, key_idx: Sequence[int], msgs: Sequence[bytes], sigs: Sequence[bytes],
                                     seed: Optional[bytes] = None) -> List[int]:
        """batch_verify_rlc_status with pks[i] = loaded table[key_idx[i]]."""
        n = len(key_idx)
        if not (len(msgs) == n == len(sigs)):
            raise ValueError("mismatching lengths")
        _check_lengths("signatures", sigs, 96)
        seed = secrets.token_bytes(32) if seed is None else seed
        if len(seed) != 32:
            raise ValueError("seed must be 32 bytes")
        pos: Dict[bytes, int] = {}
        table: List[bytes] = []
        midx = (ctypes.c_uint32 * max(n, 1))()
        for i, m in enumerate(msgs):
            m = bytes(m)
            j = pos.get(m)
            if j is None:
                j = pos[m] = len(table)
                table.append(m)
            midx[i] = j
        blob, offs = _offsets(table)
        st = _status_array(n)
        kidx = (ctypes.c_uint32 * max(n, 1))(*key_idx)
        _check(self.lib.hipbls_batch_verify_rlc_keys(kidx, b"".join(sigs), midx, n, blob, offs, len(table), seed, st),
               self.lib)
        return list(st)[:n]

    def rlc_stats(self) -> Tuple[int, int, int]:
        """(windows, windows that failed the batched check, items re-verified one by one) of the last RLC call."""
        a, b, c = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        _check(self.lib.hipbls_rlc_stats(ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)), self.lib)
        return a.value, b.value, c.value

    def threshold_aggregate(self, partial_signatures_by_index: Mapping[int, bytes]) -> bytes:
        """herumi.go:244-283."""
        res = self.batch_threshold_aggregate([partial_signatures_by_index])[0]
        if isinstance(res, TBLSError):
            raise res
        return res

    def batch_threshold_aggregate(self, groups: Sequence[Mapping[int, bytes]]):
        """One ThresholdAggregate per group; returns the 96-byte signature or the TBLSError."""
        n_groups = len(groups)
        offs = (ctypes.c_uint64 * (n_groups + 1))()
        ids, sigs = [], []
        for g, grp in enumerate(groups):
            offs[g] = len(ids)
            for idx, s in grp.items():
                if len(s) != 96:
                    raise ValueError("bad signature length")
                ids.append(_go_int(idx))
                sigs.append(bytes(s))
        offs[n_groups] = len(ids)
        arr = (ctypes.c_int64 * max(len(ids), 1))(*ids)
        out = ctypes.create_string_buffer(96 * max(n_groups, 1))
        st = _status_array(n_groups)
        _check(self.lib.hipbls_threshold_aggregate_batch(b"".join(sigs), arr, offs, n_groups, out, st), self.lib)
        res = []
        raw = out.raw
        for g in range(n_groups):
            if st[g] == OK:
                res.append(raw[96 * g:96 * g + 96])
            elif st[g] == ERR_SIGNATURE:
                res.append(TBLSError("cannot unmarshal signature into Herumi signature"))
            else:
                res.append(TBLSError("cannot combine signatures"))
        return res

    def batch_threshold_aggregate_verify(self, groups: Sequence[Mapping[int, bytes]], dv_pks: Sequence[bytes],
                                         msgs: Sequence[bytes]):
        """core/sigagg in one call (sigagg.go:138-159): ThresholdAggregate of each group and Verify of the aggregate
        against the validator's root key over its message.  Returns (aggregates: bytes or TBLSError per group,
        verify statuses: OK / ERR_PUBKEY / ERR_VERIFY, or the aggregation's status when it failed)."""
        n_groups = len(groups)
        if not (len(dv_pks) == len(msgs) == n_groups):
            raise ValueError("mismatching lengths")
        _check_lengths("public keys", dv_pks, 48)
        offs = (ctypes.c_uint64 * (n_groups + 1))()
        ids, sigs = [], []
        for g, grp in enumerate(groups):
            offs[g] = len(ids)
            for idx, sg in grp.items():
                if len(sg) != 96:
                    raise ValueError("bad signature length")
                ids.append(_go_int(idx))
                sigs.append(bytes(sg))
        offs[n_groups] = len(ids)
        arr = (ctypes.c_int64 * max(len(ids), 1))(*ids)
        blob, moffs = _offsets([bytes(m) for m in msgs])
        out = ctypes.create_string_buffer(96 * max(n_groups, 1))
        ast = _status_array(n_groups)
        vst = _status_array(n_groups)
        _check(self.lib.hipbls_threshold_aggregate_verify_batch(b"".join(sigs), arr, offs, n_groups, b"".join(dv_pks),
                                                                blob, moffs, out, ast, vst), self.lib)
        res = []
        raw = out.raw
        for g in range(n_groups):
            if ast[g] == OK:
                res.append(raw[96 * g:96 * g + 96])
            elif ast[g] == ERR_SIGNATURE:
                res.append(TBLSError("cannot unmarshal signature into Herumi signature"))
            else:
                res.append(TBLSError("cannot combine signatures"))
        return res, list(vst)[:n_groups]

    def verify_aggregate(self, shares: Sequence[bytes], signature: bytes, data: bytes) -> None:
        """herumi.go:315-339 (FastAggregateVerify)."""
        _check_lengths("public keys", shares, 48)
        _check_lengths("signature", [signature], 96)
        st = _status_array(1)
        _check(self.lib.hipbls_verify_aggregate(b"".join(shares), len(shares), signature, data, len(data), st),
               self.lib)
        if st[0] == ERR_SIGNATURE:
            raise TBLSError("cannot unmarshal signature into Herumi signature")
        if st[0] == ERR_PUBKEY:
            raise TBLSError("cannot set compressed public key in Herumi format")
        if st[0] != OK:
            raise TBLSError("signature verification failed")

    def batch_verify_aggregate_status(self, groups: Sequence[Tuple[Sequence[bytes], bytes, bytes]]) -> List[int]:
        """One FastAggregateVerify per (shares, signature, data) group in one launch; per-group status
        (OK / ERR_SIGNATURE / ERR_PUBKEY / ERR_VERIFY, as verify_aggregate raises)."""
        g = len(groups)
        for shares, sig, _ in groups:
            _check_lengths("public keys", shares, 48)
            _check_lengths("signature", [sig], 96)
        koffs = (ctypes.c_uint64 * (g + 1))()
        keys: List[bytes] = []
        for j, (shares, _, _) in enumerate(groups):
            koffs[j] = len(keys)
            keys.extend(bytes(s) for s in shares)
        koffs[g] = len(keys)
        blob, moffs = _offsets([bytes(d) for _, _, d in groups])
        st = _status_array(g)
        _check(self.lib.hipbls_verify_aggregate_batch(b"".join(keys), koffs, g, b"".join(bytes(s) for _, s, _ in groups),
                                                      blob, moffs, st), self.lib)
        return list(st)[:g]

    def aggregate(self, signs: Sequence[bytes]) -> bytes:
        """herumi.go:220-242: the G2 sum; the only error is a signature that does not deserialize.  An empty
        list is not an error: the result is the point at infinity (INFINITY_G2)."""
        _check_lengths("signatures", signs, 96)
        out = ctypes.create_string_buffer(96)
        st = _status_array(1)
        _check(self.lib.hipbls_aggregate(b"".join(signs), len(signs), out, st), self.lib)
        if st[0] == ERR_SIGNATURE:
            raise TBLSError("cannot unmarshal signature into Herumi signature")
        if st[0] != OK:
            raise DeviceError("unexpected aggregate status %d" % st[0])
        return out.raw

    def deserialize_status(self, points: Sequence[bytes], kind: int) -> List[int]:
        """herumi Deserialize per point: kind 1 = public keys (OK / ERR_PUBKEY), 2 = signatures (OK / ERR_SIGNATURE)."""
        size = 48 if kind == 1 else 96
        _check_lengths("points", points, size)
        st = _status_array(len(points))
        _check(self.lib.hipbls_deserialize_status(b"".join(points), len(points), kind, st), self.lib)
        return list(st)[:len(points)]

    # ---------------------------------------------------------------- submission queue (coalesced Verify)
    def verify_queued(self, compressed_public_key: bytes, data: bytes, signature: bytes) -> int:
        """One tbls.Verify through the library's submission queue (hipbls_verify): concurrent callers are
        coalesced into batched launches.  Returns the status code (OK / ERR_*)."""
        _check_lengths("public key", [compressed_public_key], 48)
        _check_lengths("signature", [signature], 96)
        st = ctypes.c_int32(-1)
        _check(self.lib.hipbls_verify(compressed_public_key, data, len(data), signature, ctypes.byref(st)), self.lib)
        return st.value

    def verify_submit(self, compressed_public_key: bytes, data: bytes, signature: bytes) -> int:
        _check_lengths("public key", [compressed_public_key], 48)
        _check_lengths("signature", [signature], 96)
        t = ctypes.c_uint64()
        _check(self.lib.hipbls_verify_submit(compressed_public_key, data, len(data), signature, ctypes.byref(t)),
               self.lib)
        return t.value

    def verify_wait(self, ticket: int) -> int:
        st = ctypes.c_int32(-1)
        _check(self.lib.hipbls_verify_wait(ticket, ctypes.byref(st)), self.lib)
        return st.value

    def queue_config(self, max_batch: int = 65536, gather_us: int = 200) -> None:
        _check(self.lib.hipbls_queue_config(max_batch, gather_us), self.lib)

    def queue_keyed_batches(self) -> int:
        """Queue batches that ran keyed (resident pubshare table + distinct messages through the H(m) cache)."""
        b = ctypes.c_uint64()
        _check(self.lib.hipbls_queue_keyed_batches(ctypes.byref(b)), self.lib)
        return b.value

    def queue_stats(self) -> Tuple[int, int]:
        b, i = ctypes.c_uint64(), ctypes.c_uint64()
        _check(self.lib.hipbls_queue_stats(ctypes.byref(b), ctypes.byref(i)), self.lib)
        return b.value, i.value

    # ---------------------------------------------------------------- eth2util/signing.Verify (§8f.3)
    def verify_signed_data_status(self, pks: Sequence[bytes], object_roots: Sequence[bytes],
                                  domains: Sequence[bytes], sigs: Sequence[bytes]) -> List[int]:
        """eth2util/signing/signing.go:88-107 per item: signing root SHA-256(object_root || domain) on the GPU,
        ERR_ZERO_SIG for an all-zero signature, else the Verify status."""
        n = len(pks)
        if not (len(object_roots) == len(domains) == len(sigs) == n):
            raise ValueError("mismatching lengths")
        _check_lengths("public keys", pks, 48)
        _check_lengths("object roots", object_roots, 32)
        _check_lengths("domains", domains, 32)
        _check_lengths("signatures", sigs, 96)
        st = _status_array(n)
        _check(self.lib.hipbls_verify_signed_data_batch(b"".join(pks), b"".join(object_roots), b"".join(domains),
                                                        b"".join(sigs), n, st), self.lib)
        return list(st)[:n]

    # ---------------------------------------------------------------- resident H(m) cache (§8f.2)
    def hcache_config(self, capacity: int) -> None:
        _check(self.lib.hipbls_hcache_config(capacity), self.lib)

    def hcache_stats(self) -> Tuple[int, int, int]:
        a, b, c = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        _check(self.lib.hipbls_hcache_stats(ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)), self.lib)
        return a.value, b.value, c.value

    # ---------------------------------------------------------------- pairing-check layout
    def set_pair_mode(self, mode: int) -> int:
        """PAIR_AUTO / PAIR_SINGLE (one lane per check) / PAIR_LANES (a lane pair per check) / PAIR_QUADS (four
        lanes per Verify-shaped check, each Miller loop split across a pair) / PAIR_OCTETS (eight lanes per Verify:
        quads with every Fp2 product split across twin lanes, the n = 1 latency path); returns the previous mode.  Results are identical in every mode; only latency and lane use differ."""
        rc = self.lib.hipbls_set_pair_mode(mode)
        if rc not in (PAIR_AUTO, PAIR_SINGLE, PAIR_LANES, PAIR_QUADS, PAIR_OCTETS):
            _check(rc, self.lib)
        return rc

    # ---------------------------------------------------------------- batch-wide RLC check (rlcb.h)
    def set_rlc_mode(self, mode: int) -> int:
        """RLC_AUTO / RLC_WINDOWS / RLC_BATCH; returns the previous mode.  Statuses never depend on it."""
        rc = self.lib.hipbls_rlc_set_mode(mode)
        if rc not in (RLC_AUTO, RLC_WINDOWS, RLC_BATCH):
            _check(rc, self.lib)
        return rc

    def set_rlc_g1_msm_min(self, min_items: int) -> int:
        """Items per message from which the batch-wide check sums [r_i] pk_i by one Pippenger MSM per message
        (g1msm.h; batches averaging >= 8 items per message); 0 = off.  Returns the previous value.  Statuses never
        depend on it."""
        if not 0 <= min_items < 1 << 31:
            raise ValueError("min_items out of range")
        return self.lib.hipbls_rlc_set_g1_msm_min(min_items)

    def rlc_batch_stats(self) -> Tuple[int, int, int]:
        """(batch-wide checks launched, passed, last verdict: -1 none / 0 failed / 1 passed)."""
        a, b, c = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_int32()
        _check(self.lib.hipbls_rlc_batch_stats(ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)), self.lib)
        return a.value, b.value, c.value
