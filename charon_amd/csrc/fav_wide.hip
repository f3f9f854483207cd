// FastAggregateVerify's sixteen-lane check (verify_hex.hip k_fav_pair_lq16) in a translation unit of its own,
// namespace bls_hexw, compiled for two waves per SIMD: its out-of-line callees are private copies here, so the
// occupancy attribute holds them to 256 registers without touching the n = 1 Verify's check (k_verify_pair_lq16,
// verify_hex.hip), whose latency needs the full 512.
#define BLS_HEX_FAV_WIDE 1
#include "verify_hex.hip"
