// Copyright © 2022-2023 Obol Labs Inc. Licensed under the terms of a Business Source License 1.1

package cluster_test

import (
	"encoding/json"
	"os"
	"path/filepath"
	"testing"

	"github.com/stretchr/testify/require"

	"github.com/obolnetwork/charon/cluster"
)

// withValidators returns lock with its own copy of the validators, so a mutation does not reach the original.
func withValidators(lock cluster.Lock) cluster.Lock {
	vals := make([]cluster.DistValidator, len(lock.Validators))
	copy(vals, lock.Validators)
	lock.Validators = vals

	return lock
}

// TestVerifyLocksSignaturesEqualsSerial checks the bulk lock verification against the serial one: for the example
// locks (cluster_test.go TestExamples) and mutations of them -- another lock's aggregate, no aggregate (accepted by
// v1.0/v1.1 only), a registration signed by the wrong validator, a missing registration, and both in one lock --
// VerifyLocksSignatures(locks)[i] is locks[i].VerifySignatures(), error text included, with every lock in one call.
func TestVerifyLocksSignaturesEqualsSerial(t *testing.T) {
	files, err := filepath.Glob("examples/*lock*")
	require.NoError(t, err)

	var locks []cluster.Lock
	for _, file := range files {
		b, err := os.ReadFile(file)
		require.NoError(t, err)

		var lock cluster.Lock
		require.NoError(t, json.Unmarshal(b, &lock))
		locks = append(locks, lock)
	}
	require.Len(t, locks, 4)

	var cases []cluster.Lock
	for i, lock := range locks {
		cases = append(cases, lock)

		other := lock
		other.SignatureAggregate = locks[(i+1)%len(locks)].SignatureAggregate
		cases = append(cases, other)

		empty := lock
		empty.SignatureAggregate = nil
		cases = append(cases, empty)

		if len(lock.Validators) < 2 || len(lock.Validators[0].BuilderRegistration.Signature) == 0 {
			continue
		}

		swapped := withValidators(lock)
		swapped.Validators[0].BuilderRegistration.Signature = lock.Validators[1].BuilderRegistration.Signature
		cases = append(cases, swapped)

		missing := withValidators(lock)
		missing.Validators[1].BuilderRegistration = cluster.BuilderRegistration{}
		cases = append(cases, missing)

		both := withValidators(swapped)
		both.Validators[1].BuilderRegistration = cluster.BuilderRegistration{}
		cases = append(cases, both)
	}

	errs := cluster.VerifyLocksSignatures(cases)
	require.Len(t, errs, len(cases))

	var failed int
	for i, lock := range cases {
		want := lock.VerifySignatures()
		if want == nil {
			require.NoError(t, errs[i], "case %d", i)
			continue
		}
		failed++
		require.EqualError(t, errs[i], want.Error(), "case %d", i)
	}
	require.Positive(t, failed)

	for i := range locks {
		require.NoError(t, cluster.VerifyLocksSignatures(locks)[i])
	}
}
