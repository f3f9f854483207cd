"""Collect the herumi-produced known-answer vectors that charon's own tests hold.

Run in the build container (needs /root/reference); writes tests/golden/kat_reference.json, a pure
data fixture (hex strings).  Nothing here is reference source: each entry is an input/output vector
and cites the reference file:line it was taken from.

  prysm      core/validatorapi/validatorapi_test.go:228-291   sk=0x01||00*31, signing root -> sig
  teku       eth2util/signing/signing_test.go:22-69, :99-104  registration -> root -> sig, domain
  deposit    eth2util/deposit/deposit_test.go:21-63 + testdata/TestMarshalDepositData.golden
  locks      cluster/examples/cluster-lock-00{0,1,2,3}.json via cluster/cluster_test.go:214-230
             (cluster/lock.go:144-189 FastAggregateVerify over all pubshares on lock_hash;
              cluster/lock.go:228-274 builder registrations = ThresholdAggregate outputs, Verify
              against the DV root key)
  manifest   cluster/manifest/testdata/lock2.json, lock.json via cluster/manifest/load_test.go:31,77
             (lock2: FastAggregateVerify of signature_aggregate over its 12 pubshares on lock_hash;
              lock: the deposit_data signatures, threshold-aggregated by the DKG (dkg/dkg.go aggDepositData),
              verified under each DV key with the deposit domain of the definition's fork version.  lock.json's own
              aggregate and registrations do not verify and no reference test says they should: not vectors)
"""
import base64
import json
import os
import re

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "kat_reference.json")


def _b(s: str) -> str:
    """Lock JSON bytes: v1.1 base64, v1.2+ 0x-hex -> plain hex."""
    if s.startswith("0x"):
        return s[2:]
    return base64.b64decode(s).hex()


def main():
    kat = {"source": "herumi/bls-eth-go-binary v1.32.1 outputs held by charon's tests"}

    # 1. prysm attestation
    src = open(os.path.join(REF, "core/validatorapi/validatorapi_test.go")).read()
    root = re.search(r'"(0x02bbdb88[0-9a-f]+)"', src).group(1)[2:]
    sig = re.search(r'"(0xb6a60f84[0-9a-f]+)"', src).group(1)[2:]
    kat["prysm"] = {"cite": "core/validatorapi/validatorapi_test.go:228-291",
                    "sk": "01" + "00" * 31, "signing_root": root, "sig": sig}

    # 2. teku registration
    src = open(os.path.join(REF, "eth2util/signing/signing_test.go")).read()
    sk = re.search(r'DecodeString\("([0-9a-f]{64})"\)', src).group(1)
    reg = json.loads(re.search(r"registrationJSON := `(.*?)`", src, re.S).group(1))
    dom = re.search(r"expect := eth2p0.Domain\{(.*?)\}", src, re.S).group(1)
    dom_hex = "".join("%02x" % int(x, 16) for x in re.findall(r"0x([0-9a-f]{2})", dom))
    m = reg["message"]
    kat["teku"] = {"cite": "eth2util/signing/signing_test.go:22-69,99-104",
                   "sk": sk, "fee_recipient": m["fee_recipient"][2:], "gas_limit": int(m["gas_limit"]),
                   "timestamp": int(m["timestamp"]), "pubkey": m["pubkey"][2:],
                   "domain": dom_hex, "sig": reg["signature"][2:]}

    # 3. deposit golden
    src = open(os.path.join(REF, "eth2util/deposit/deposit_test.go")).read()
    sks = re.findall(r'"([0-9a-f]{64})"', src)
    golden = json.load(open(os.path.join(REF, "eth2util/deposit/testdata/TestMarshalDepositData.golden")))
    kat["deposit"] = {"cite": "eth2util/deposit/deposit_test.go:21-63, testdata/TestMarshalDepositData.golden",
                      "sks": sks, "entries": golden}

    # 4. cluster lock examples
    locks = []
    for i in range(4):
        path = "cluster/examples/cluster-lock-%03d.json" % i
        d = json.load(open(os.path.join(REF, path)))
        vals = []
        for v in d["distributed_validators"]:
            ent = {"distributed_public_key": _b(v["distributed_public_key"]),
                   "public_shares": [_b(s) for s in v["public_shares"]]}
            br = v.get("builder_registration")
            if br and br.get("signature"):
                msg = br["message"]
                ent["builder_registration"] = {
                    "fee_recipient": _b(msg["fee_recipient"]), "gas_limit": int(msg["gas_limit"]),
                    "timestamp": int(msg["timestamp"]), "pubkey": _b(msg["pubkey"]),
                    "signature": _b(br["signature"])}
            vals.append(ent)
        locks.append({"cite": path, "version": d["cluster_definition"]["version"],
                      "fork_version": d["cluster_definition"]["fork_version"][2:],
                      "lock_hash": _b(d["lock_hash"]), "signature_aggregate": _b(d["signature_aggregate"]),
                      "validators": vals})
    kat["locks"] = locks

    # 5. cluster/manifest testdata (round 6)
    path = "cluster/manifest/testdata/lock2.json"
    d = json.load(open(os.path.join(REF, path)))
    man = {"lock2": {"cite": path + " (cluster/manifest/load_test.go:77)",
                     "lock_hash": _b(d["lock_hash"]), "signature_aggregate": _b(d["signature_aggregate"]),
                     "public_shares": [_b(s) for v in d["distributed_validators"] for s in v["public_shares"]]}}
    path = "cluster/manifest/testdata/lock.json"
    d = json.load(open(os.path.join(REF, path)))
    man["lock_deposits"] = {"cite": path + " (cluster/manifest/load_test.go:31)",
                            "fork_version": d["cluster_definition"]["fork_version"][2:],
                            "deposit_data": [{"pubkey": _b(v["deposit_data"]["pubkey"]),
                                              "withdrawal_credentials": _b(v["deposit_data"]["withdrawal_credentials"]),
                                              "amount": int(v["deposit_data"]["amount"]),
                                              "signature": _b(v["deposit_data"]["signature"])}
                                             for v in d["distributed_validators"]]}
    kat["manifest"] = man

    with open(OUT, "w") as f:
        json.dump(kat, f, indent=1)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
