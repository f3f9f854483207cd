//go:build hipbls

package hipbls

import (
	"crypto/rand"
	"sync"
	"testing"

	promtest "github.com/prometheus/client_golang/prometheus/testutil"
	"github.com/stretchr/testify/require"

	"github.com/obolnetwork/charon/tbls"
)

// keys returns n (pk, sig over root) pairs made by tbls.Herumi, with sigs[1] and sigs[2] swapped (two failures).
func keys(t *testing.T, n int, root []byte) ([]tbls.PublicKey, []tbls.Signature, []map[int]tbls.Signature) {
	t.Helper()
	ref := tbls.Herumi{}
	pks := make([]tbls.PublicKey, n)
	sigs := make([]tbls.Signature, n)
	for i := 0; i < n; i++ {
		secret, err := ref.GenerateSecretKey()
		require.NoError(t, err)
		pks[i], err = ref.SecretToPublicKey(secret)
		require.NoError(t, err)
		sigs[i], err = ref.Sign(secret, root)
		require.NoError(t, err)
	}
	groups := []map[int]tbls.Signature{{1: sigs[0]}, {1: sigs[3], 2: sigs[4]}}
	sigs[1], sigs[2] = sigs[2], sigs[1]

	return pks, sigs, groups
}

// TestMetricsCountEveryEntryPoint: every entry point records its batch size, items and failed items under its path
// label, and the RLC window counters advance (metrics.go; SURVEY.md §5, VERDICT r05 next 6).
func TestMetricsCountEveryEntryPoint(t *testing.T) {
	h, err := New()
	require.NoError(t, err)
	const n = 8
	root := make([]byte, 32)
	_, _ = rand.Read(root)
	pks, sigs, groups := keys(t, n, root)
	msgs := make([][]byte, n)
	for i := range msgs {
		msgs[i] = root
	}

	items := func(path string) float64 { return promtest.ToFloat64(itemsCounter.WithLabelValues(path)) }
	failed := func(path string) float64 { return promtest.ToFloat64(failedCounter.WithLabelValues(path)) }

	i0, f0 := items("batch_verify"), failed("batch_verify")
	_, err = h.BatchVerify(pks, msgs, sigs)
	require.NoError(t, err)
	require.InDelta(t, n, items("batch_verify")-i0, 0)
	require.InDelta(t, 2, failed("batch_verify")-f0, 0)

	i0, w0 := items("batch_verify_rlc"), promtest.ToFloat64(rlcWindows)
	_, err = h.BatchVerifyRLC(pks, sigs, make([]uint32, n), [][]byte{root})
	require.NoError(t, err)
	require.InDelta(t, n, items("batch_verify_rlc")-i0, 0)
	require.Greater(t, promtest.ToFloat64(rlcWindows), w0)

	i0 = items("verify")
	require.Error(t, h.Verify(pks[1], root, sigs[1]))
	require.InDelta(t, 1, items("verify")-i0, 0)

	i0 = items("threshold_aggregate")
	_, _, err = h.BatchThresholdAggregate(groups)
	require.NoError(t, err)
	require.InDelta(t, len(groups), items("threshold_aggregate")-i0, 0)

	i0 = items("fused_sigagg")
	_, _, _, err = h.BatchThresholdAggregateVerify(groups, pks[:2], [][]byte{root, root})
	require.NoError(t, err)
	require.InDelta(t, len(groups), items("fused_sigagg")-i0, 0)

	i0 = items("batch_verify_aggregate")
	_, err = h.BatchVerifyAggregate([][]tbls.PublicKey{pks[:1], pks[3:5]}, []tbls.Signature{sigs[0], sigs[3]},
		[][]byte{root, root})
	require.NoError(t, err)
	require.InDelta(t, 2, items("batch_verify_aggregate")-i0, 0)

	require.NoError(t, h.LoadPubShares(pks))
	i0 = items("batch_verify_keys")
	_, err = h.BatchVerify(pks, msgs, sigs)
	require.NoError(t, err)
	require.InDelta(t, n, items("batch_verify_keys")-i0, 0)
	require.NoError(t, h.LoadPubShares(nil))
}

// TestReloadWaitsForKeyedCalls: the table's read lock is held across a keyed call (lockTable), so a LoadPubShares
// racing batch calls never leaves a call verifying against indices of another table (ADVICE r05): every keyed
// result equals the wire-format result for the same items.
func TestReloadWaitsForKeyedCalls(t *testing.T) {
	h, err := New()
	require.NoError(t, err)
	const n = 16
	root := make([]byte, 32)
	_, _ = rand.Read(root)
	pks, sigs, _ := keys(t, n, root)
	other, _, _ := keys(t, n, root) // a table of other keys: a stale index would name one of these
	msgs := make([][]byte, n)
	for i := range msgs {
		msgs[i] = root
	}
	want, err := h.BatchVerify(pks, msgs, sigs)
	require.NoError(t, err)

	var (
		wg      sync.WaitGroup
		loadErr error
	)
	wg.Add(1)
	go func() {
		defer wg.Done()
		for k := 0; k < 20 && loadErr == nil; k++ {
			if loadErr = h.LoadPubShares(pks); loadErr == nil {
				loadErr = h.LoadPubShares(other)
			}
		}
	}()
	for k := 0; k < 20; k++ {
		got, err := h.BatchVerify(pks, msgs, sigs)
		require.NoError(t, err)
		for i := range want {
			require.Equal(t, want[i] == nil, got[i] == nil, i)
		}
	}
	wg.Wait()
	require.NoError(t, loadErr)

	require.NoError(t, h.LoadPubShares(nil))
	_, ok, release := lockTable(pks)
	release()
	require.False(t, ok)
}
