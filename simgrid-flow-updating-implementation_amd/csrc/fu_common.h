// Internal helpers shared by the libfu translation units.
#pragma once

#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

#include "fu.h"

namespace fu {

// Thread-local last error (fu_last_error).
void set_error(const std::string &msg);
int fail(int code, const std::string &msg);

constexpr uint64_t kGolden = 0x9E3779B97F4A7C15ull;

inline uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
// Element i of the SplitMix64 stream seeded with `seed` (counter form, thread-count free).
inline uint64_t splitmix_at(uint64_t seed, uint64_t i) { return mix64(seed + (i + 1) * kGolden); }
// Sequential SplitMix64 step (same as the Python oracle's splitmix64()).
inline uint64_t splitmix_next(uint64_t &state) {
  state += kGolden;
  return mix64(state);
}
inline double u01(uint64_t x) { return (double)(x >> 11) * 0x1.0p-53; }

}  // namespace fu

// Host graph: CSR with int64 row pointer on the host (device copies use int32).
struct fu_graph {
  int32_t n = 0;
  std::vector<int64_t> rowptr;  // n + 1
  std::vector<int32_t> col;     // E
  std::vector<int32_t> rev;     // E, empty if not symmetric
  int32_t max_deg = 0;
};

namespace fu {
// Builds rev for g (fails if some i->j lacks j->i). Parallel, deterministic.
int build_rev(fu_graph &g);
}  // namespace fu

#define FU_TRY_BEGIN try {
#define FU_TRY_END                                                   \
  }                                                                  \
  catch (const std::bad_alloc &) {                                   \
    return fu::fail(FU_ERR_ALLOC, "host allocation failed");         \
  }                                                                  \
  catch (const std::exception &ex) {                                 \
    return fu::fail(FU_ERR_ARG, std::string("exception: ") + ex.what()); \
  }
