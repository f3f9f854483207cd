//go:build !hipbls

package app

import (
	"context"

	"github.com/obolnetwork/charon/app/errors"
)

// selectGPUBLS: this binary was built without the GPU implementation (-tags hipbls), so the gpu_bls feature cannot
// be honoured; failing at startup beats silently running on the CPU path the operator asked to replace.
func selectGPUBLS(context.Context) error {
	return errors.New("feature gpu_bls enabled but charon was built without -tags hipbls")
}
