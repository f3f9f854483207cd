//go:build hipbls

// Package hipbls implements tbls.Implementation on AMD MI355X (gfx950) GPUs through libhipbls, the C-ABI in
// include/hipbls.h (ABI 12).  It replaces tbls.Herumi (tbls/herumi.go) method for method: same argument meaning,
// same error strings and wrapping, bit-identical keys, signatures and verdicts.  Every curve operation runs in the
// library's HIP kernels; Go only range-checks 32-byte scalars (as herumi's SecretKey.Deserialize does) and moves
// bytes.
//
// Build: copy charon_amd/libhipbls.so to ./lib and include/hipbls.h to ./include (or point CGO_CFLAGS /
// CGO_LDFLAGS at them) and build charon with -tags hipbls.  Without the tag this package is not compiled and charon
// builds exactly as before.
package hipbls

/*
#cgo CFLAGS: -I${SRCDIR}/include
#cgo LDFLAGS: -L${SRCDIR}/lib -lhipbls -Wl,-rpath,${SRCDIR}/lib
#include <stdlib.h>
#include "hipbls.h"
*/
import "C"

import (
	"crypto/rand"
	"fmt"
	"io"
	"math/big"
	"sync"
	"testing"
	"unsafe"

	"github.com/stretchr/testify/require"

	"github.com/obolnetwork/charon/app/errors"
	"github.com/obolnetwork/charon/app/z"
	"github.com/obolnetwork/charon/tbls"
)

// abiVersion is the include/hipbls.h ABI this file is written against.
const abiVersion = 12

// BLS12-381 group order r: a 32-byte big-endian scalar deserializes iff it is < r (herumi SecretKey.Deserialize).
var order, _ = new(big.Int).SetString("73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001", 16)

// HipBLS holds no state of its own: libhipbls holds one context per GPU (device, streams, workspaces, the resident
// pubshare table and H(m) cache, a Verify submission queue), and the Go side keeps only the table's key -> index map
// (pubShareIndex, process-wide like the library).  Every method is safe for concurrent use.
type HipBLS struct{}

var (
	_ tbls.Implementation = HipBLS{} // all 11 methods
	_ tbls.BatchVerifier  = HipBLS{} // the batch extension (patches/0001)
	_ tbls.PubShareLoader = HipBLS{} // the resident pubshare table (patches/0001, loaded by app/app.go)
)

// pubShareIndex maps every pubshare loaded into the library's resident table (LoadPubShares) to its table index.
var pubShareIndex struct {
	sync.RWMutex
	idx map[tbls.PublicKey]uint32
}

// New binds the charon process to the given GPUs (all of the node's, normally: charon is one process per node,
// app/app.go:127).  Every batch is split into contiguous validator ranges across them and the results land in the
// caller's slices; single Verify calls go to the GPU their signing root hashes to (hipbls_init_devices).  New() with
// no ids uses every visible GPU.
func New(devices ...int) (HipBLS, error) {
	if v := int(C.hipbls_abi_version()); v != abiVersion {
		return HipBLS{}, errors.New("hipbls: library ABI mismatch", z.Int("want", abiVersion), z.Int("got", v))
	}
	if len(devices) == 0 {
		for d := 0; d < int(C.hipbls_device_count()); d++ {
			devices = append(devices, d)
		}
	}
	if len(devices) == 0 {
		return HipBLS{}, errors.New("hipbls: no GPU")
	}
	ids := make([]C.int32_t, len(devices))
	for i, d := range devices {
		ids[i] = C.int32_t(d)
	}
	if rc := C.hipbls_init_devices(&ids[0], C.uint32_t(len(ids))); rc != C.HIPBLS_OK {
		return HipBLS{}, devErr(rc) // includes a device whose scratch region cannot hold the library's queues
	}
	for _, d := range devices {
		if _, err := ScratchBudget(d); err != nil {
			return HipBLS{}, err
		}
	}

	return HipBLS{}, nil
}

// Scratch is a device's scratch budget (hipbls_scratch_budget, DESIGN.md 5.1.1): every hardware queue that runs the
// library's kernels holds PerQueue bytes of the device's Limit-byte scratch region; the library holds four queues
// (reserved at New) and never puts its kernels on a caller's priority or CU-masked stream, so Headroom is what the
// rest of the process (another GPU library, a priority stream) may still hold on the device.
type Scratch struct {
	PerLane, PerQueue, Limit uint64
	Queues                   uint32
}

// Headroom is the scratch the library's four queues leave on the device (0 when the runtime reports no limit).
func (s Scratch) Headroom() uint64 {
	if s.Limit < 4*s.PerQueue {
		return 0
	}

	return s.Limit - 4*s.PerQueue
}

// ScratchBudget returns device d's scratch budget as the library computed it when New bound the device.
func ScratchBudget(d int) (Scratch, error) {
	var pl, pq, lim C.uint64_t
	var q C.uint32_t
	if rc := C.hipbls_scratch_budget(C.int(d), &pl, &pq, &lim, &q); rc != C.HIPBLS_OK {
		return Scratch{}, devErr(rc)
	}

	return Scratch{PerLane: uint64(pl), PerQueue: uint64(pq), Limit: uint64(lim), Queues: uint32(q)}, nil
}

// LoadPubShares decodes and subgroup-checks the cluster's pubshares once into every GPU's resident table
// (hipbls_pubshare_table_load; SURVEY.md §8f.2: the lock's keys, app/app.go:344-381).  Afterwards BatchVerify and
// BatchVerifyRLC name keys by table index when every key of a call is in the table (no per-call decode or subgroup
// test; herumi does both on every Verify, tbls/herumi.go:286-289), and the submission queue behind Verify turns
// batches of table keys into random-linear-combination checks.  Results are unchanged.  A key that does not decode
// stays out of the index, so calls naming it take the wire-format path and get herumi's error for it.  Loading again
// replaces the table.
func (HipBLS) LoadPubShares(pubshares []tbls.PublicKey) error {
	pubShareIndex.Lock()
	defer pubShareIndex.Unlock()
	idx := make(map[tbls.PublicKey]uint32, len(pubshares))
	if len(pubshares) > 0 {
		flat := make([]byte, 0, 48*len(pubshares))
		for _, k := range pubshares {
			flat = append(flat, k[:]...)
		}
		status := make([]int32, len(pubshares))
		if rc := C.hipbls_pubshare_table_load(u8(flat), C.uint64_t(len(pubshares)), i32(status)); rc != C.HIPBLS_OK {
			pubShareIndex.idx = nil
			return devErr(rc)
		}
		for i, k := range pubshares {
			if _, dup := idx[k]; !dup && status[i] == C.HIPBLS_OK {
				idx[k] = uint32(i)
			}
		}
	}
	pubShareIndex.idx = idx

	return nil
}

// lockTable returns every key's index in the resident pubshare table (ok false when one is not in it) and holds the
// table's read lock until release is called.  The keyed C call must run before release: a concurrent LoadPubShares
// replaces the device table, and an index resolved against the old table would then name another key (ADVICE r05).
// Readers share the lock, so batch calls still run side by side; only a reload waits for them.
func lockTable(pks []tbls.PublicKey) (kidx []uint32, ok bool, release func()) {
	pubShareIndex.RLock()
	if len(pubShareIndex.idx) == 0 {
		return nil, false, pubShareIndex.RUnlock
	}
	out := make([]uint32, len(pks))
	for i, k := range pks {
		j, found := pubShareIndex.idx[k]
		if !found {
			return nil, false, pubShareIndex.RUnlock
		}
		out[i] = j
	}

	return out, true, pubShareIndex.RUnlock
}

func devErr(rc C.int) error {
	return errors.New("hipbls device error", z.Int("rc", int(rc)), z.Str("err", C.GoString(C.hipbls_last_error())))
}

// herumiCause is the error herumi's Deserialize returns underneath charon's wrap (INTEGRATION.md "Errors": the text
// lives in bls-eth-go-binary v1.32.1, not vendored; callers only test err != nil).
func herumiCause(kind string, buf []byte) error {
	return fmt.Errorf("err bls%sDeserialize %x", kind, buf) //nolint:forbidigo // herumi's own text
}

// deserErr: what herumi returns for a key or signature that does not deserialize (tbls/herumi.go:287-294).
func deserErr(status C.int32_t, pk, sig []byte) error {
	if status == C.HIPBLS_ERR_PUBKEY {
		return errors.Wrap(herumiCause("PublicKey", pk), "cannot set compressed public key in Herumi format")
	}

	return errors.Wrap(herumiCause("Signature", sig), "cannot unmarshal signature into Herumi signature")
}

// verifyErr maps one Verify status onto herumi's error for that item (tbls/herumi.go:285-301).
func verifyErr(s int32, pk, sig []byte) error {
	switch C.int32_t(s) {
	case C.HIPBLS_OK:
		return nil
	case C.HIPBLS_ERR_VERIFY:
		return errors.New("signature not verified")
	default:
		return deserErr(C.int32_t(s), pk, sig)
	}
}

// firstBad: the index of the first point of kind (1 = 48-byte G1, 2 = 96-byte G2) that does not deserialize
// (hipbls_deserialize_status), for the signature_number field of herumi.go:228-233 / 254-259; -1 when none.
func firstBad(flat []byte, n int, kind int32) int {
	if n == 0 {
		return -1
	}
	st := make([]int32, n)
	if C.hipbls_deserialize_status(u8(flat), C.uint64_t(n), C.int32_t(kind), i32(st)) != C.HIPBLS_OK {
		return -1
	}
	for i, s := range st {
		if s != C.HIPBLS_OK {
			return i
		}
	}

	return -1
}

func u8(b []byte) *C.uint8_t {
	if len(b) == 0 {
		return nil
	}

	return (*C.uint8_t)(unsafe.Pointer(&b[0]))
}

func i32(s []int32) *C.int32_t   { return (*C.int32_t)(unsafe.Pointer(&s[0])) }
func u64(s []uint64) *C.uint64_t { return (*C.uint64_t)(unsafe.Pointer(&s[0])) }

func i64(s []int64) *C.int64_t {
	if len(s) == 0 {
		return nil
	}

	return (*C.int64_t)(unsafe.Pointer(&s[0]))
}

func validScalar(b [32]byte) bool { return new(big.Int).SetBytes(b[:]).Cmp(order) < 0 }

// flatten concatenates messages and returns the blob + n+1 offsets (hipbls_verify_batch layout).
func flatten(msgs [][]byte) ([]byte, []uint64) {
	offs := make([]uint64, len(msgs)+1)
	var flat []byte
	for i, m := range msgs {
		flat = append(flat, m...)
		offs[i+1] = uint64(len(flat))
	}

	return flat, offs
}

// ---------------------------------------------------------------- key tooling (tbls/herumi.go:44-218)

// GenerateSecretKey: uniform in [0, r) from crypto/rand (herumi SetByCSPRNG).
func (HipBLS) GenerateSecretKey() (tbls.PrivateKey, error) {
	for {
		var k tbls.PrivateKey
		if _, err := rand.Read(k[:]); err != nil {
			return tbls.PrivateKey{}, errors.Wrap(err, "read random")
		}
		k[0] &= 0x7f // r < 2^255: rejection sampling on 255 bits
		if validScalar(k) {
			return k, nil
		}
	}
}

// GenerateInsecureKey: up to 100 reads of 32 bytes until one deserializes (tbls/herumi.go:343-360).
func (HipBLS) GenerateInsecureKey(t *testing.T, random io.Reader) (tbls.PrivateKey, error) {
	t.Helper()
	for i := 0; i < 100; i++ {
		var k tbls.PrivateKey
		_, err := random.Read(k[:])
		require.NoError(t, err)
		if validScalar(k) {
			return k, nil
		}
	}

	return tbls.PrivateKey{}, errors.New("cannot generate insecure key")
}

// SecretToPublicKey (tbls/herumi.go:67-80).
func (HipBLS) SecretToPublicKey(secret tbls.PrivateKey) (tbls.PublicKey, error) {
	if !validScalar(secret) {
		return tbls.PublicKey{}, errors.New("cannot unmarshal secret into Herumi secret key")
	}
	var pk tbls.PublicKey
	status := make([]int32, 1)
	if rc := C.hipbls_secret_to_public_key_batch(u8(secret[:]), 1, u8(pk[:]), i32(status)); rc != C.HIPBLS_OK {
		return tbls.PublicKey{}, devErr(rc)
	}
	if status[0] != C.HIPBLS_OK { // zero secret: GetSafePublicKey fails (herumi.go:74)
		return tbls.PublicKey{}, errors.New("cannot obtain public key from secret")
	}

	return pk, nil
}

func (h HipBLS) split(secret tbls.PrivateKey, total, threshold uint, tail func() (tbls.PrivateKey, error)) (map[int]tbls.PrivateKey, error) {
	if !validScalar(secret) {
		return nil, errors.New("cannot unmarshal bytes into Herumi secret key")
	}
	poly := make([]byte, 0, 32*int(threshold))
	for i := 1; i < int(threshold); i++ {
		k, err := tail()
		if err != nil {
			return nil, err
		}
		poly = append(poly, k[:]...)
	}
	out := make([]byte, 32*int(total))
	status := make([]int32, 1)
	if rc := C.hipbls_threshold_split(u8(secret[:]), u8(poly), C.uint32_t(total), C.uint32_t(threshold), u8(out),
		i32(status)); rc != C.HIPBLS_OK {
		return nil, devErr(rc)
	}
	if status[0] != C.HIPBLS_OK {
		return nil, errors.New("cannot unmarshal bytes into Herumi secret key")
	}
	ret := make(map[int]tbls.PrivateKey, total)
	for i := 1; i <= int(total); i++ {
		var k tbls.PrivateKey
		copy(k[:], out[32*(i-1):32*i]) // share i = f(i), ids 1..total (herumi.go:110-129)
		ret[i] = k
	}

	return ret, nil
}

// ThresholdSplit: polynomial tail from crypto/rand (tbls/herumi.go:134-181).
func (h HipBLS) ThresholdSplit(secret tbls.PrivateKey, total, threshold uint) (map[int]tbls.PrivateKey, error) {
	return h.split(secret, total, threshold, h.GenerateSecretKey)
}

// ThresholdSplitInsecure: polynomial tail from the caller's reader (tbls/herumi.go:84-132).
func (h HipBLS) ThresholdSplitInsecure(t *testing.T, secret tbls.PrivateKey, total, threshold uint, random io.Reader) (map[int]tbls.PrivateKey, error) {
	t.Helper()

	return h.split(secret, total, threshold, func() (tbls.PrivateKey, error) { return h.GenerateInsecureKey(t, random) })
}

// RecoverSecret: Lagrange at 0 over Fr with ids as Fr elements (strconv.Itoa(idx) -> SetDecString: int64 mod r,
// tbls/herumi.go:183-218).
func (HipBLS) RecoverSecret(shares map[int]tbls.PrivateKey, _, _ uint) (tbls.PrivateKey, error) {
	var flat []byte
	var ids []int64
	for idx, k := range shares {
		if !validScalar(k) {
			return tbls.PrivateKey{}, errors.New("cannot unmarshal key with into Herumi secret key", z.Int("key_number", idx))
		}
		flat = append(flat, k[:]...)
		ids = append(ids, int64(idx))
	}
	var out tbls.PrivateKey
	status := make([]int32, 1)
	if rc := C.hipbls_recover_secret(u8(flat), i64(ids), C.uint32_t(len(ids)), u8(out[:]), i32(status)); rc != C.HIPBLS_OK {
		return tbls.PrivateKey{}, devErr(rc)
	}
	if status[0] != C.HIPBLS_OK {
		return tbls.PrivateKey{}, errors.New("cannot recover full private key from partial keys")
	}

	return out, nil
}

// ---------------------------------------------------------------- hot path

// Sign (tbls/herumi.go:303-313).
func (HipBLS) Sign(privateKey tbls.PrivateKey, data []byte) (tbls.Signature, error) {
	if !validScalar(privateKey) {
		return tbls.Signature{}, errors.New("cannot unmarshal secret into Herumi secret key")
	}
	var sig tbls.Signature
	flat, offs := flatten([][]byte{data})
	status := make([]int32, 1)
	if rc := C.hipbls_sign_batch(u8(privateKey[:]), u8(flat), u64(offs), 1, u8(sig[:]), i32(status)); rc != C.HIPBLS_OK {
		return tbls.Signature{}, devErr(rc)
	}
	if status[0] != C.HIPBLS_OK {
		return tbls.Signature{}, errors.New("cannot unmarshal secret into Herumi secret key")
	}

	return sig, nil
}

// Verify (tbls/herumi.go:285-301) goes through the library's submission queue: concurrent goroutines (parsigex,
// validatorapi, sigagg) are coalesced into one GPU launch per batch, no lock is held while the GPU runs, and each
// caller blocks only on its own item (hipbls_verify).  Callers with many items use BatchVerify (batch.go).
func (HipBLS) Verify(pk tbls.PublicKey, data []byte, sig tbls.Signature) error {
	var status C.int32_t
	if rc := C.hipbls_verify(u8(pk[:]), u8(data), C.uint64_t(len(data)), u8(sig[:]), &status); rc != C.HIPBLS_OK {
		return observeFailure("verify", 1, devErr(rc))
	}
	err := verifyErr(int32(status), pk[:], sig[:])
	observeOne("verify", err)

	return err
}

// ThresholdAggregate (tbls/herumi.go:244-283): ids are the map keys as Fr elements (int64 mod r); one group of the
// batched kernel.  A partial that does not deserialize is named by its map key (signature_number).
func (h HipBLS) ThresholdAggregate(parts map[int]tbls.Signature) (tbls.Signature, error) {
	out, errs, err := h.BatchThresholdAggregate([]map[int]tbls.Signature{parts})
	if err != nil {
		return tbls.Signature{}, err
	}
	if errs[0] != nil && errs[0].Error() == "cannot unmarshal signature into Herumi signature" {
		for idx, s := range parts {
			if firstBad(s[:], 1, 2) == 0 {
				return tbls.Signature{}, errors.Wrap(herumiCause("Signature", s[:]),
					"cannot unmarshal signature into Herumi signature", z.Int("signature_number", idx))
			}
		}
	}

	return out[0], errs[0]
}

// VerifyAggregate: FastAggregateVerify (tbls/herumi.go:315-339); an empty key list is "signature verification
// failed".
func (HipBLS) VerifyAggregate(shares []tbls.PublicKey, sig tbls.Signature, data []byte) error {
	keys := make([]byte, 0, 48*len(shares))
	for _, s := range shares {
		keys = append(keys, s[:]...)
	}
	status := make([]int32, 1)
	if rc := C.hipbls_verify_aggregate(u8(keys), C.uint64_t(len(shares)), u8(sig[:]), u8(data), C.uint64_t(len(data)),
		i32(status)); rc != C.HIPBLS_OK {
		return observeFailure("verify_aggregate", 1, devErr(rc))
	}
	observeStatus("verify_aggregate", 1, status[0] != C.HIPBLS_OK)
	switch C.int32_t(status[0]) {
	case C.HIPBLS_OK:
		return nil
	case C.HIPBLS_ERR_SIGNATURE:
		return deserErr(C.HIPBLS_ERR_SIGNATURE, nil, sig[:])
	case C.HIPBLS_ERR_PUBKEY: // the first share that does not deserialize (herumi.go:325-330)
		if i := firstBad(keys, len(shares), 1); i >= 0 {
			return deserErr(C.HIPBLS_ERR_PUBKEY, shares[i][:], nil)
		}

		return errors.New("cannot set compressed public key in Herumi format")
	default:
		return errors.New("signature verification failed")
	}
}

// Aggregate (tbls/herumi.go:220-242): the G2 sum; the only error is a signature that does not deserialize.  An
// empty slice is not an error: the zero point's encoding 0xc0 || 0^95.
func (HipBLS) Aggregate(signs []tbls.Signature) (tbls.Signature, error) {
	flat := make([]byte, 0, 96*len(signs))
	for _, s := range signs {
		flat = append(flat, s[:]...)
	}
	var out tbls.Signature
	status := make([]int32, 1)
	if rc := C.hipbls_aggregate(u8(flat), C.uint64_t(len(signs)), u8(out[:]), i32(status)); rc != C.HIPBLS_OK {
		return tbls.Signature{}, observeFailure("aggregate", len(signs), devErr(rc))
	}
	observeStatus("aggregate", len(signs), status[0] != C.HIPBLS_OK)
	if status[0] != C.HIPBLS_OK {
		i := firstBad(flat, len(signs), 2)
		if i < 0 {
			i = 0
		}

		return tbls.Signature{}, errors.Wrap(herumiCause("Signature", signs[i][:]),
			"cannot unmarshal signature into Herumi signature", z.Int("signature_number", i))
	}

	return out, nil
}
