//go:build hipbls

package hipbls

/*
#include "hipbls.h"
*/
import "C"

import (
	"crypto/rand"
	"unsafe"

	"github.com/obolnetwork/charon/app/errors"
	"github.com/obolnetwork/charon/tbls"
)

// The batch extension (tbls.BatchVerifier, patches/0001-tbls-batch-extension.patch): one GPU launch sequence for
// what charon's callers do in loops (core/parsigex/parsigex.go:86-91, core/validatorapi/validatorapi.go:246-283,
// core/sigagg/sigagg.go:138-159).  Every result equals the serial call's for that item: errs[i] is exactly what
// Verify / ThresholdAggregate / VerifyAggregate would return.  A device failure fails the whole call (the error
// return) and is never turned into per-item results.

// BatchVerify verifies n (pk, msg, sig) items in one launch; errs[i] is what Verify returns for item i.
func (HipBLS) BatchVerify(pks []tbls.PublicKey, msgs [][]byte, sigs []tbls.Signature) ([]error, error) {
	n := len(pks)
	if n == 0 {
		return nil, nil
	}
	if len(msgs) != n || len(sigs) != n {
		return nil, errors.New("mismatching lengths")
	}
	flat, offs := flatten(msgs)
	status := make([]int32, n)
	var rc C.int
	path := "batch_verify"
	kidx, keyed, release := lockTable(pks) // held across the call: a reload cannot swap the table under the indices
	if keyed { // keys by resident table index: no per-call decode or subgroup test
		path = "batch_verify_keys"
		rc = C.hipbls_verify_batch_keys((*C.uint32_t)(unsafe.Pointer(&kidx[0])), u8(flat), u64(offs),
			(*C.uint8_t)(unsafe.Pointer(&sigs[0][0])), C.uint64_t(n), i32(status))
	} else {
		rc = C.hipbls_verify_batch((*C.uint8_t)(unsafe.Pointer(&pks[0][0])), u8(flat), u64(offs),
			(*C.uint8_t)(unsafe.Pointer(&sigs[0][0])), C.uint64_t(n), i32(status))
	}
	release()
	if rc != C.HIPBLS_OK {
		return nil, observeFailure(path, n, devErr(rc))
	}
	errs := make([]error, n)
	for i, s := range status {
		errs[i] = verifyErr(s, pks[i][:], sigs[i][:])
	}
	observe(path, errs)

	return errs, nil
}

// BatchVerifyRLC: the same per-item results as BatchVerify, decided by random-linear-combination checks (one
// batch-wide Pippenger check for all-valid batches, windows of 8 otherwise; DESIGN.md 4.6).  msgs are DISTINCT roots,
// msgIdx[i] < len(msgs) names item i's root, and a validator's items should be adjacent.  The seed is fresh from
// crypto/rand on every call: the check is only sound if the signers cannot predict it.
func (HipBLS) BatchVerifyRLC(pks []tbls.PublicKey, sigs []tbls.Signature, msgIdx []uint32, msgs [][]byte) ([]error, error) {
	n := len(pks)
	if n == 0 {
		return nil, nil
	}
	if len(sigs) != n || len(msgIdx) != n {
		return nil, errors.New("mismatching lengths")
	}
	flat, offs := flatten(msgs)
	var seed [32]byte
	if _, err := rand.Read(seed[:]); err != nil {
		return nil, errors.Wrap(err, "rlc seed")
	}
	status := make([]int32, n)
	var rc C.int
	path := "batch_verify_rlc"
	kidx, keyed, release := lockTable(pks) // held across the call, as in BatchVerify
	if keyed { // keys by resident table index
		path = "batch_verify_rlc_keys"
		rc = C.hipbls_batch_verify_rlc_keys((*C.uint32_t)(unsafe.Pointer(&kidx[0])),
			(*C.uint8_t)(unsafe.Pointer(&sigs[0][0])), (*C.uint32_t)(unsafe.Pointer(&msgIdx[0])), C.uint64_t(n), u8(flat),
			u64(offs), C.uint64_t(len(msgs)), u8(seed[:]), i32(status))
	} else {
		rc = C.hipbls_batch_verify_rlc((*C.uint8_t)(unsafe.Pointer(&pks[0][0])),
			(*C.uint8_t)(unsafe.Pointer(&sigs[0][0])), (*C.uint32_t)(unsafe.Pointer(&msgIdx[0])), C.uint64_t(n), u8(flat),
			u64(offs), C.uint64_t(len(msgs)), u8(seed[:]), i32(status))
	}
	release()
	if rc != C.HIPBLS_OK {
		return nil, observeFailure(path, n, devErr(rc))
	}
	errs := make([]error, n)
	for i, s := range status {
		errs[i] = verifyErr(s, pks[i][:], sigs[i][:])
	}
	observe(path, errs)
	observeRLC()

	return errs, nil
}

// groupsFlat lays out ThresholdAggregate groups for the C-ABI: signatures, int64 ids (map keys, no truncation) and
// group offsets.  Map iteration order is irrelevant to the result (Lagrange at 0 is symmetric).
func groupsFlat(groups []map[int]tbls.Signature) ([]byte, []int64, []uint64) {
	var sigs []byte
	var ids []int64
	offs := []uint64{0}
	for _, g := range groups {
		for idx, s := range g {
			sigs = append(sigs, s[:]...)
			ids = append(ids, int64(idx))
		}
		offs = append(offs, uint64(len(ids)))
	}

	return sigs, ids, offs
}

// aggErr maps an aggregation status onto herumi's error text (tbls/herumi.go:244-283).
func aggErr(s int32) error {
	switch C.int32_t(s) {
	case C.HIPBLS_OK:
		return nil
	case C.HIPBLS_ERR_SIGNATURE:
		return errors.New("cannot unmarshal signature into Herumi signature")
	default: // empty group, id 0 (mod r), duplicate id
		return errors.New("cannot combine signatures")
	}
}

// BatchThresholdAggregate: one output signature (or error) per group.
func (HipBLS) BatchThresholdAggregate(groups []map[int]tbls.Signature) ([]tbls.Signature, []error, error) {
	if len(groups) == 0 {
		return nil, nil, nil
	}
	sigs, ids, offs := groupsFlat(groups)
	out := make([]tbls.Signature, len(groups))
	status := make([]int32, len(groups))
	rc := C.hipbls_threshold_aggregate_batch(u8(sigs), i64(ids), u64(offs), C.uint64_t(len(groups)),
		(*C.uint8_t)(unsafe.Pointer(&out[0][0])), i32(status))
	if rc != C.HIPBLS_OK {
		return nil, nil, observeFailure("threshold_aggregate", len(groups), devErr(rc))
	}
	errs := make([]error, len(groups))
	for g, s := range status {
		errs[g] = aggErr(s)
	}
	observe("threshold_aggregate", errs)

	return out, errs, nil
}

// BatchVerifyAggregate: one FastAggregateVerify per (keys, sig, msg) group in one launch (cluster.Lock
// VerifySignatures over every lock and registration, cluster/lock.go:144-274).
func (h HipBLS) BatchVerifyAggregate(keys [][]tbls.PublicKey, sigs []tbls.Signature, msgs [][]byte) ([]error, error) {
	g := len(keys)
	if g == 0 {
		return nil, nil
	}
	if len(sigs) != g || len(msgs) != g {
		return nil, errors.New("mismatching lengths")
	}
	var flatKeys []byte
	koffs := make([]uint64, g+1)
	for i, ks := range keys {
		for _, k := range ks {
			flatKeys = append(flatKeys, k[:]...)
		}
		koffs[i+1] = uint64(len(flatKeys) / 48)
	}
	flat, moffs := flatten(msgs)
	status := make([]int32, g)
	rc := C.hipbls_verify_aggregate_batch(u8(flatKeys), u64(koffs), C.uint64_t(g),
		(*C.uint8_t)(unsafe.Pointer(&sigs[0][0])), u8(flat), u64(moffs), i32(status))
	if rc != C.HIPBLS_OK {
		return nil, observeFailure("batch_verify_aggregate", g, devErr(rc))
	}
	errs := make([]error, g)
	for i, s := range status {
		switch C.int32_t(s) {
		case C.HIPBLS_OK:
		case C.HIPBLS_ERR_SIGNATURE:
			errs[i] = deserErr(C.HIPBLS_ERR_SIGNATURE, nil, sigs[i][:])
		case C.HIPBLS_ERR_PUBKEY: // name the key as VerifyAggregate does
			errs[i] = h.VerifyAggregate(keys[i], sigs[i], msgs[i])
		default:
			errs[i] = errors.New("signature verification failed")
		}
	}
	observe("batch_verify_aggregate", errs)

	return errs, nil
}

// BatchThresholdAggregateVerify: core/sigagg in one call (sigagg.go:138-159).  For each validator g: the aggregate
// of its partials (or the aggregation error) and the error Verify(dvPks[g], msgs[g], aggregate) would return (the
// aggregation's error when it failed).  Same results as BatchThresholdAggregate + BatchVerify; the root key decode
// and H(m) run beside the aggregation and the aggregate is not decompressed again (DESIGN.md 4.9).
func (HipBLS) BatchThresholdAggregateVerify(groups []map[int]tbls.Signature, dvPks []tbls.PublicKey,
	msgs [][]byte,
) ([]tbls.Signature, []error, []error, error) {
	n := len(groups)
	if n == 0 {
		return nil, nil, nil, nil
	}
	if len(dvPks) != n || len(msgs) != n {
		return nil, nil, nil, errors.New("mismatching lengths")
	}
	sigs, ids, offs := groupsFlat(groups)
	flat, moffs := flatten(msgs)
	out := make([]tbls.Signature, n)
	ast := make([]int32, n)
	vst := make([]int32, n)
	rc := C.hipbls_threshold_aggregate_verify_batch(u8(sigs), i64(ids), u64(offs), C.uint64_t(n),
		(*C.uint8_t)(unsafe.Pointer(&dvPks[0][0])), u8(flat), u64(moffs), (*C.uint8_t)(unsafe.Pointer(&out[0][0])),
		i32(ast), i32(vst))
	if rc != C.HIPBLS_OK {
		return nil, nil, nil, observeFailure("fused_sigagg", n, devErr(rc))
	}
	aggErrs := make([]error, n)
	verErrs := make([]error, n)
	for g := range groups {
		aggErrs[g] = aggErr(ast[g])
		if aggErrs[g] != nil {
			verErrs[g] = aggErrs[g]
		} else {
			verErrs[g] = verifyErr(vst[g], dvPks[g][:], out[g][:])
		}
	}
	observe("fused_sigagg", verErrs)

	return out, aggErrs, verErrs, nil
}
