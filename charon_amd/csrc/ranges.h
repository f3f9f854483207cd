// Splitting a batch across device contexts (host code only; hipbls.hip, and the sanitizer build of the host code,
// tests/native/sanitize_main.cpp).
#pragma once

#include <cstdint>
#include <vector>

namespace {

// Contiguous ranges: bounds[0] = 0 < ... < bounds[parts] = n, as equal as possible.  With run keys (e.g. the message
// index of each item, equal for all partials of one validator), an inner bound moves forward to the start of the
// next run, so a run never straddles two devices, unless that would move it by more than half a share.
inline std::vector<uint64_t> plan_ranges(uint64_t n, uint64_t parts, const uint32_t* keys) {
  if (parts < 1) parts = 1;
  if (parts > n && n > 0) parts = n;
  std::vector<uint64_t> b(parts + 1);
  b[0] = 0;
  b[parts] = n;
  const uint64_t share = parts ? n / parts : 0;
  for (uint64_t k = 1; k < parts; ++k) {
    uint64_t x = (uint64_t)((unsigned __int128)n * k / parts);
    if (keys && x > 0 && x < n) {
      const uint64_t lim = x + share / 2;
      uint64_t y = x;
      while (y < n && y < lim && keys[y] == keys[y - 1]) ++y;
      if (y == n || keys[y] != keys[y - 1]) x = y;  // the next run start, within half a share
    }
    b[k] = x < b[k - 1] ? b[k - 1] : x;
  }
  return b;
}

}  // namespace
