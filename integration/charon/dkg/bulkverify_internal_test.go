// Copyright © 2022-2023 Obol Labs Inc. Licensed under the terms of a Business Source License 1.1

package dkg

import (
	"testing"

	eth2p0 "github.com/attestantio/go-eth2-client/spec/phase0"
	"github.com/stretchr/testify/require"

	"github.com/obolnetwork/charon/core"
	"github.com/obolnetwork/charon/eth2util"
	"github.com/obolnetwork/charon/eth2util/deposit"
	"github.com/obolnetwork/charon/tbls"
	"github.com/obolnetwork/charon/tbls/tblsconv"
	"github.com/obolnetwork/charon/testutil"
)

// TestBulkAggregation runs the batched DKG aggregation over several DVs (dkg_internal_test.go covers one DV per
// call): every DV's deposit data aggregates to Sign(secret), and a bad partial of any one DV fails the whole call
// with the serial loop's error text; the lock hash partials of every DV go through one batch check.
func TestBulkAggregation(t *testing.T) {
	const (
		n   = 4
		th  = 3
		dvs = 5
	)
	network := eth2util.Goerli.Name

	var (
		shares  []share
		secrets []tbls.PrivateKey
		splits  []map[int]tbls.PrivateKey
		corePks []core.PubKey
	)
	msgs := make(map[core.PubKey]eth2p0.DepositMessage)
	byPubkey := make(map[core.PubKey]share)
	for d := 0; d < dvs; d++ {
		secret, err := tbls.GenerateSecretKey()
		require.NoError(t, err)
		pubkey, err := tbls.SecretToPublicKey(secret)
		require.NoError(t, err)
		split, err := tbls.ThresholdSplit(secret, n, th)
		require.NoError(t, err)

		pubshares := make(map[int]tbls.PublicKey)
		for idx, sk := range split {
			pubshares[idx], err = tbls.SecretToPublicKey(sk)
			require.NoError(t, err)
		}
		sh := share{PubKey: pubkey, SecretShare: split[1], PublicShares: pubshares}
		shares = append(shares, sh)
		secrets = append(secrets, secret)
		splits = append(splits, split)

		corePk, err := core.PubKeyFromBytes(pubkey[:])
		require.NoError(t, err)
		eth2Pk, err := corePk.ToETH2()
		require.NoError(t, err)
		msgs[corePk], err = deposit.NewMessage(eth2Pk, testutil.RandomETHAddress())
		require.NoError(t, err)
		corePks = append(corePks, corePk)
		byPubkey[corePk] = sh
	}

	partials := func(bad int, msgOf func(d int) []byte) map[core.PubKey][]core.ParSignedData {
		data := make(map[core.PubKey][]core.ParSignedData)
		for d, pk := range corePks {
			for idx := 1; idx <= th; idx++ {
				msg := msgOf(d)
				if d == bad && idx == th {
					msg = []byte("invalid msg")
				}
				sig, err := tbls.Sign(splits[d][idx], msg)
				require.NoError(t, err)
				data[pk] = append(data[pk], core.NewPartialSignature(tblsconv.SigToCore(sig), idx))
			}
		}

		return data
	}
	depositRoot := func(d int) []byte {
		root, err := deposit.GetMessageSigningRoot(msgs[corePks[d]], network)
		require.NoError(t, err)

		return root[:]
	}

	datas, err := aggDepositData(partials(-1, depositRoot), shares, msgs, network)
	require.NoError(t, err)
	require.Len(t, datas, dvs)
	for _, dd := range datas {
		for d, pk := range corePks {
			eth2Pk, err := pk.ToETH2()
			require.NoError(t, err)
			if eth2Pk != dd.PublicKey {
				continue
			}
			want, err := tbls.Sign(secrets[d], depositRoot(d))
			require.NoError(t, err)
			require.Equal(t, tblsconv.SigToETH2(want), dd.Signature)
		}
	}

	for bad := 0; bad < dvs; bad++ {
		_, err = aggDepositData(partials(bad, depositRoot), shares, msgs, network)
		require.EqualError(t, err, "invalid deposit data partial signature from peer")
	}

	lockHash := []byte("cluster lock hash")
	lockMsg := func(int) []byte { return lockHash }
	_, pubkeys, err := aggLockHashSig(partials(-1, lockMsg), byPubkey, lockHash)
	require.NoError(t, err)
	require.Len(t, pubkeys, dvs*th)

	_, _, err = aggLockHashSig(partials(dvs-1, lockMsg), byPubkey, lockHash)
	require.EqualError(t, err, "invalid lock hash partial signature from peer: signature not verified")
}
