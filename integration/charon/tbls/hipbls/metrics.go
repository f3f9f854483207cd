//go:build hipbls

package hipbls

/*
#include "hipbls.h"
*/
import "C"

import (
	"github.com/prometheus/client_golang/prometheus"

	"github.com/obolnetwork/charon/app/promauto"
)

// Engine metrics (SURVEY.md §5; the promauto pattern of core/parsigdb/metrics.go:10-16).  Every entry point records
// its calls by path: the batch size, the items and the items whose result is an error, and device failures.  The
// path label tells which GPU route charon's callers reach: "verify" (the submission queue behind tbls.Verify),
// "batch_verify" / "batch_verify_keys" (wire-format keys or the resident pubshare table), "batch_verify_rlc" /
// "batch_verify_rlc_keys" (random-linear-combination checks over shared roots), "threshold_aggregate",
// "fused_sigagg" (BatchThresholdAggregateVerify), "verify_aggregate", "batch_verify_aggregate" and "aggregate".
var (
	itemsCounter = promauto.NewCounterVec(prometheus.CounterOpts{
		Namespace: "tbls",
		Subsystem: "hipbls",
		Name:      "items_total",
		Help:      "Total number of items (signatures, aggregates or aggregate groups) processed on the GPU by path",
	}, []string{"path"})

	failedCounter = promauto.NewCounterVec(prometheus.CounterOpts{
		Namespace: "tbls",
		Subsystem: "hipbls",
		Name:      "failed_items_total",
		Help:      "Total number of items whose result is an error (not verified, not decodable, not combinable) by path",
	}, []string{"path"})

	batchSize = promauto.NewHistogramVec(prometheus.HistogramOpts{
		Namespace: "tbls",
		Subsystem: "hipbls",
		Name:      "batch_size",
		Help:      "Items per GPU call by path",
		Buckets:   prometheus.ExponentialBuckets(1, 4, 10), // 1 .. 262,144
	}, []string{"path"})

	deviceErrors = promauto.NewCounterVec(prometheus.CounterOpts{
		Namespace: "tbls",
		Subsystem: "hipbls",
		Name:      "device_errors_total",
		Help:      "Total number of GPU calls that failed as a whole (HIPBLS_ERR_DEVICE or a bad argument) by path",
	}, []string{"path"})

	rlcWindows = promauto.NewCounter(prometheus.CounterOpts{
		Namespace: "tbls",
		Subsystem: "hipbls",
		Name:      "rlc_windows_total",
		Help:      "Total number of RLC verdict windows checked (hipbls_rlc_stats)",
	})

	rlcWindowsFailed = promauto.NewCounter(prometheus.CounterOpts{
		Namespace: "tbls",
		Subsystem: "hipbls",
		Name:      "rlc_windows_failed_total",
		Help:      "Total number of RLC windows that failed and sent their items to per-item checks",
	})

	rlcFallbackItems = promauto.NewCounter(prometheus.CounterOpts{
		Namespace: "tbls",
		Subsystem: "hipbls",
		Name:      "rlc_fallback_items_total",
		Help:      "Total number of items re-verified one by one after their RLC window failed",
	})
)

// observe records one call of path that returned errs (one entry per item).
func observe(path string, errs []error) {
	batchSize.WithLabelValues(path).Observe(float64(len(errs)))
	itemsCounter.WithLabelValues(path).Add(float64(len(errs)))
	var failed int
	for _, e := range errs {
		if e != nil {
			failed++
		}
	}
	if failed > 0 {
		failedCounter.WithLabelValues(path).Add(float64(failed))
	}
}

// observeOne records a single-item call of path.
func observeOne(path string, err error) {
	batchSize.WithLabelValues(path).Observe(1)
	itemsCounter.WithLabelValues(path).Inc()
	if err != nil {
		failedCounter.WithLabelValues(path).Inc()
	}
}

// observeStatus records a call of path over n inputs with one result, failed or not.
func observeStatus(path string, n int, failed bool) {
	batchSize.WithLabelValues(path).Observe(float64(n))
	itemsCounter.WithLabelValues(path).Add(float64(n))
	if failed {
		failedCounter.WithLabelValues(path).Inc()
	}
}

// observeFailure records a call of n items that failed as a whole and returns its error.
func observeFailure(path string, n int, err error) error {
	batchSize.WithLabelValues(path).Observe(float64(n))
	deviceErrors.WithLabelValues(path).Inc()

	return err
}

// observeRLC adds the window counts of the RLC call that just returned (hipbls_rlc_stats reports the last call of the
// process, so with concurrent RLC calls the split between calls is approximate; the totals over time are not).
func observeRLC() {
	var windows, failed, fallback C.uint64_t
	if C.hipbls_rlc_stats(&windows, &failed, &fallback) != C.HIPBLS_OK {
		return
	}
	rlcWindows.Add(float64(windows))
	rlcWindowsFailed.Add(float64(failed))
	rlcFallbackItems.Add(float64(fallback))
}
