// Copyright © 2022-2023 Obol Labs Inc. Licensed under the terms of a Business Source License 1.1

package dkg

import (
	"github.com/obolnetwork/charon/tbls"
)

// verifyStep is one step of a DKG aggregation loop, in the serial loop's order: an error the loop returns at that
// point (err), or one tbls.Verify(pubkey, msg, sig) whose failure the loop returns as fail(verifyErr).
type verifyStep struct {
	err    error
	pubkey tbls.PublicKey
	msg    []byte
	sig    tbls.Signature
	fail   func(error) error
}

// stepErrors returns, for every step before the first err step, the error that step's Verify makes the serial loop
// return (nil when it verifies).  Every Verify runs in ONE tbls.BatchVerifyRLC call over the distinct messages: the
// lock hash is one message for every partial of the ceremony, a deposit or registration root one per DV, so the
// random-linear-combination check shares each root's hash-to-G2 and pairing (one GPU launch sequence with tbls/hipbls,
// the serial calls with any other implementation).  The error return is a failure of the whole call.
func stepErrors(steps []verifyStep) ([]error, error) {
	var (
		pks    []tbls.PublicKey
		sigs   []tbls.Signature
		msgIdx []uint32
		msgs   [][]byte
	)
	index := make(map[string]uint32)
	for _, s := range steps {
		if s.err != nil {
			break // the serial loop returns here: later steps are never reached
		}
		k, ok := index[string(s.msg)]
		if !ok {
			k = uint32(len(msgs))
			index[string(s.msg)] = k
			msgs = append(msgs, s.msg)
		}
		pks = append(pks, s.pubkey)
		sigs = append(sigs, s.sig)
		msgIdx = append(msgIdx, k)
	}

	res, err := tbls.BatchVerifyRLC(pks, sigs, msgIdx, msgs)
	if err != nil {
		return nil, err
	}

	errs := make([]error, len(steps))
	for i, s := range steps {
		switch {
		case s.err != nil:
			errs[i] = s.err
			return errs, nil
		case res[i] != nil:
			errs[i] = s.fail(res[i])
		}
	}

	return errs, nil
}

// firstFailure returns what the serial loop over steps returns: the first step whose err is set or whose Verify fails
// (nil when none does), with every Verify in one batch call (stepErrors).
func firstFailure(steps []verifyStep) error {
	errs, err := stepErrors(steps)
	if err != nil {
		return err
	}
	for _, err := range errs {
		if err != nil {
			return err
		}
	}

	return nil
}

// dvAggregation is one DV of aggDepositData / aggValidatorRegistrations after its partial-signature steps: the
// steps [first, end) of the ceremony's step list, the partials to threshold-aggregate, and what the aggregate is
// verified against.  A DV whose lookups failed is the last one and is not complete: steps[end] is that failure.
type dvAggregation struct {
	first, end int
	complete   bool // every lookup succeeded: the serial loop reaches this DV's aggregation
	psigs      map[int]tbls.Signature
	pubkey     tbls.PublicKey
	pubkeyErr  error
	root       []byte
}

// aggregateVerified runs what the serial DKG aggregation loops run per DV -- every partial Verify, then
// ThresholdAggregate and Verify of the aggregate under the DV key -- as two batch calls: one tbls.BatchVerifyRLC over
// every partial (stepErrors) and one tbls.BatchThresholdAggregateVerify over every DV whose partials all verified.
// Results are replayed DV by DV in the loop's order: a DV's first failing step, then its aggregation error, its key
// error, then its aggregate's Verify wrapped by aggFail.  It returns the aggregates of every DV, or the first failure.
func aggregateVerified(steps []verifyStep, dvs []dvAggregation, aggFail func(error) error) ([]tbls.Signature, error) {
	errs, err := stepErrors(steps)
	if err != nil {
		return nil, err
	}

	var (
		groups []map[int]tbls.Signature
		dvPks  []tbls.PublicKey
		msgs   [][]byte
	)
	gi := make([]int, len(dvs))
	for d, dv := range dvs {
		gi[d] = -1
		if !dv.complete {
			break
		}
		ok := true
		for i := dv.first; i < dv.end; i++ {
			ok = ok && errs[i] == nil
		}
		if !ok {
			break // the serial loop stops at this DV's failing partial
		}
		gi[d] = len(groups)
		groups = append(groups, dv.psigs)
		dvPks = append(dvPks, dv.pubkey)
		msgs = append(msgs, dv.root)
	}

	var (
		aggs             []tbls.Signature
		aggErrs, verErrs []error
	)
	if len(groups) > 0 {
		aggs, aggErrs, verErrs, err = tbls.BatchThresholdAggregateVerify(groups, dvPks, msgs)
		if err != nil {
			return nil, err
		}
	}

	out := make([]tbls.Signature, 0, len(dvs))
	for d, dv := range dvs {
		for i := dv.first; i < dv.end; i++ {
			if errs[i] != nil {
				return nil, errs[i]
			}
		}
		if !dv.complete {
			return nil, errs[dv.end] // the lookup that stopped the serial loop inside this DV
		}
		g := gi[d]
		if aggErrs[g] != nil {
			return nil, aggErrs[g]
		}
		if dv.pubkeyErr != nil {
			return nil, dv.pubkeyErr
		}
		if verErrs[g] != nil {
			return nil, aggFail(verErrs[g])
		}
		out = append(out, aggs[g])
	}

	return out, nil
}
