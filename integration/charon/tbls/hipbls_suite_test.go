//go:build hipbls

package tbls_test

import (
	"testing"

	"github.com/stretchr/testify/require"

	"github.com/obolnetwork/charon/tbls"
	"github.com/obolnetwork/charon/tbls/hipbls"
)

// The reference's conformance hooks (tbls_test.go:170-216) with the GPU implementation added: the whole TestSuite
// against hipbls, and randomizedImpl choosing herumi or hipbls per call, so keys, shares and signatures made by one
// are consumed by the other.  FuzzRandomImplementations (tbls_test.go:342-346) drives TestRandomized; the fuzz target
// below drives the mixed one.

func newHipBLS(t testing.TB) tbls.Implementation {
	t.Helper()
	impl, err := hipbls.New()
	require.NoError(t, err)

	return impl
}

func TestHipBLSImplementation(t *testing.T) {
	runSuite(t, newHipBLS(t))
}

func TestRandomizedHipBLSHerumi(t *testing.T) {
	runSuite(t, randomizedImpl{
		implementations: []tbls.Implementation{
			tbls.Herumi{},
			newHipBLS(t),
		},
	})
}

func FuzzRandomImplementationsHipBLS(f *testing.F) {
	f.Fuzz(func(t *testing.T, _ byte) {
		TestRandomizedHipBLSHerumi(t)
	})
}

func BenchmarkHipBLSImplementation(b *testing.B) {
	runBenchmark(b, newHipBLS(b))
}
