//go:build hipbls

package hipbls_test

import (
	"crypto/rand"
	"testing"

	"github.com/stretchr/testify/require"

	"github.com/obolnetwork/charon/tbls"
	"github.com/obolnetwork/charon/tbls/hipbls"
)

// Bit-exactness against herumi (tbls.Herumi, the reference implementation in this tree) on the same inputs:
// identical keys, signatures and aggregates, identical error presence per item; and every batch call equal to the
// serial calls it replaces.  The Python twin of these checks is tests/test_gpu_r03.py / test_gpu_r04.py in the
// hipbls repository.

func gpu(t *testing.T) hipbls.HipBLS {
	t.Helper()
	h, err := hipbls.New()
	require.NoError(t, err)

	return h
}

func TestBytesEqualHerumi(t *testing.T) {
	h, ref := gpu(t), tbls.Herumi{}
	for i := 0; i < 16; i++ {
		secret, err := ref.GenerateSecretKey()
		require.NoError(t, err)
		msg := make([]byte, 32)
		_, _ = rand.Read(msg)

		pkG, err := h.SecretToPublicKey(secret)
		require.NoError(t, err)
		pkR, err := ref.SecretToPublicKey(secret)
		require.NoError(t, err)
		require.Equal(t, pkR, pkG)

		sigG, err := h.Sign(secret, msg)
		require.NoError(t, err)
		sigR, err := ref.Sign(secret, msg)
		require.NoError(t, err)
		require.Equal(t, sigR, sigG)

		require.NoError(t, h.Verify(pkR, msg, sigR))
		msg[0] ^= 1
		require.Error(t, h.Verify(pkR, msg, sigR))
		require.Error(t, ref.Verify(pkR, msg, sigR))

		// 3-of-5 shares from herumi, aggregated by both
		shares, err := ref.ThresholdSplit(secret, 5, 3)
		require.NoError(t, err)
		parts := make(map[int]tbls.Signature)
		for _, idx := range []int{1, 3, 5} {
			parts[idx], err = ref.Sign(shares[idx], msg)
			require.NoError(t, err)
		}
		aggG, err := h.ThresholdAggregate(parts)
		require.NoError(t, err)
		aggR, err := ref.ThresholdAggregate(parts)
		require.NoError(t, err)
		require.Equal(t, aggR, aggG)

		recG, err := h.RecoverSecret(shares, 5, 3)
		require.NoError(t, err)
		require.Equal(t, secret, recG)
	}
}

func TestBatchEqualsSerial(t *testing.T) {
	h, ref := gpu(t), tbls.Herumi{}
	const n = 64
	pks := make([]tbls.PublicKey, n)
	sigs := make([]tbls.Signature, n)
	msgs := make([][]byte, n)
	for i := 0; i < n; i++ {
		secret, err := ref.GenerateSecretKey()
		require.NoError(t, err)
		pks[i], err = ref.SecretToPublicKey(secret)
		require.NoError(t, err)
		msgs[i] = make([]byte, 32)
		_, _ = rand.Read(msgs[i])
		sigs[i], err = ref.Sign(secret, msgs[i])
		require.NoError(t, err)
	}
	msgs[3] = []byte("other root") // signature not verified
	sigs[7][0] &= 0x7f            // does not deserialize
	pks[9] = pks[10]              // wrong key
	errs, err := h.BatchVerify(pks, msgs, sigs)
	require.NoError(t, err)
	for i := range pks {
		serial := ref.Verify(pks[i], msgs[i], sigs[i])
		require.Equal(t, serial == nil, errs[i] == nil, i)
		switch {
		case i == 7:
			require.ErrorContains(t, errs[i], "cannot unmarshal signature into Herumi signature")
		case serial != nil:
			require.EqualError(t, errs[i], "signature not verified")
		}
	}
	// the same items as an RLC batch over a distinct-root table
	idx := make([]uint32, n)
	for i := range idx {
		idx[i] = uint32(i)
	}
	rlc, err := h.BatchVerifyRLC(pks, sigs, idx, msgs)
	require.NoError(t, err)
	for i := range errs {
		require.Equal(t, errs[i] == nil, rlc[i] == nil, i)
	}
}

func TestPubShareTableSameResults(t *testing.T) {
	h, ref := gpu(t), tbls.Herumi{}
	const n = 48
	pks := make([]tbls.PublicKey, n)
	sigs := make([]tbls.Signature, n)
	msgs := make([][]byte, n)
	root := make([]byte, 32)
	_, _ = rand.Read(root)
	for i := 0; i < n; i++ {
		secret, err := ref.GenerateSecretKey()
		require.NoError(t, err)
		pks[i], err = ref.SecretToPublicKey(secret)
		require.NoError(t, err)
		msgs[i] = root // one committee root: the RLC path over one message
		sigs[i], err = ref.Sign(secret, msgs[i])
		require.NoError(t, err)
	}
	sigs[5], sigs[6] = sigs[6], sigs[5] // two wrong signatures
	before, err := h.BatchVerify(pks, msgs, sigs)
	require.NoError(t, err)
	require.NoError(t, h.LoadPubShares(pks))
	after, err := h.BatchVerify(pks, msgs, sigs)
	require.NoError(t, err)
	rlc, err := h.BatchVerifyRLC(pks, sigs, make([]uint32, n), [][]byte{root})
	require.NoError(t, err)
	for i := range pks {
		require.Equal(t, before[i] == nil, after[i] == nil, i)
		require.Equal(t, before[i] == nil, rlc[i] == nil, i)
		require.Equal(t, ref.Verify(pks[i], msgs[i], sigs[i]) == nil, after[i] == nil, i)
	}
	require.NoError(t, h.LoadPubShares(nil)) // empty table: the wire-format path again (internal_test.go)
}
