//go:build hipbls

package app

import (
	"context"

	"github.com/obolnetwork/charon/app/log"
	"github.com/obolnetwork/charon/app/z"
	"github.com/obolnetwork/charon/tbls"
	"github.com/obolnetwork/charon/tbls/hipbls"
)

// selectGPUBLS binds libhipbls to every GPU of the node (one charon process per node drives them all, one device
// context each) and installs it as the tbls implementation.  parsigex and sigagg then take their batch paths
// (wireCoreWorkflow type-asserts tbls.BatchVerifier).
func selectGPUBLS(ctx context.Context) error {
	impl, err := hipbls.New()
	if err != nil {
		return err
	}
	tbls.SetImplementation(impl)
	log.Info(ctx, "tbls backed by the GPU implementation", z.Str("impl", "hipbls"))

	return nil
}
