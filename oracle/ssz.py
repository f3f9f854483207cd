"""CPU oracle: the SSZ signing-root helpers charon computes before tbls.Verify/Sign.

TEST INFRASTRUCTURE ONLY (see oracle/bls12381.py header).  Restates:
  eth2util/signing/signing.go:57-69      GetDataRoot = SigningData{ObjectRoot, Domain}.HashTreeRoot
  eth2util/deposit/deposit.go:113-157    deposit domain = 0x03000000 || ForkData{version, 0}.root[:28]
  eth2util/registration/registration.go:60-101  builder domain = 0x00000001 || ForkData{genesis_version, 0}.root[:28]
SSZ merkleization per the consensus-specs (SHA-256, 32-byte chunks, little-endian uints).
"""
import hashlib


def _h(a: bytes, b: bytes) -> bytes:
    return hashlib.sha256(a + b).digest()


def merkleize(chunks):
    n = 1
    while n < len(chunks):
        n *= 2
    layer = list(chunks) + [bytes(32)] * (n - len(chunks))
    while len(layer) > 1:
        layer = [_h(layer[i], layer[i + 1]) for i in range(0, len(layer), 2)]
    return layer[0]


def pack_bytes(b: bytes):
    """Fixed-size byte vector -> root (chunks padded to 32)."""
    chunks = [b[i:i + 32].ljust(32, b"\x00") for i in range(0, len(b), 32)] or [bytes(32)]
    return merkleize(chunks)


def uint64(v: int) -> bytes:
    return v.to_bytes(8, "little").ljust(32, b"\x00")


def signing_data_root(object_root: bytes, domain: bytes) -> bytes:
    return merkleize([object_root, domain])


def fork_data_root(version: bytes, genesis_validators_root: bytes = bytes(32)) -> bytes:
    return merkleize([version.ljust(32, b"\x00"), genesis_validators_root])


def compute_domain(domain_type: bytes, fork_version: bytes, genesis_validators_root: bytes = bytes(32)) -> bytes:
    return domain_type + fork_data_root(fork_version, genesis_validators_root)[:28]


def validator_registration_root(fee_recipient: bytes, gas_limit: int, timestamp: int, pubkey: bytes) -> bytes:
    return merkleize([fee_recipient.ljust(32, b"\x00"), uint64(gas_limit), uint64(timestamp), pack_bytes(pubkey)])


def deposit_message_root(pubkey: bytes, withdrawal_credentials: bytes, amount: int) -> bytes:
    return merkleize([pack_bytes(pubkey), withdrawal_credentials, uint64(amount)])


DOMAIN_DEPOSIT = bytes.fromhex("03000000")
DOMAIN_APPLICATION_BUILDER = bytes.fromhex("00000001")
