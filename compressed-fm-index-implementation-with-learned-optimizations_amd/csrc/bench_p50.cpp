// bench_p50.cpp — bench helper (libcs_bench.so, not part of the product ABI): the
// p50 single-pattern latency exactly as SURVEY.md §8(d) prescribes it, "median over
// >= 1000 single-pattern calls through the C++ facade (end-to-end, the method of
// tools/benchmark.cpp:154-166)": each pattern is a host string_view into
// cs::FMIndex::count(), timed with std::chrono::steady_clock around the call.
// serve != 0: the same calls with the index in serving mode (FMIndex::serve).
#include <chrono>
#include <cstdint>
#include <stdexcept>
#include <string_view>

#include "../../include/cs/fm_index.hpp"

extern "C" int cs_bench_facade_count_latency(cs_fm_index* h, const uint8_t* pats, uint64_t m,
                                             uint64_t npat, uint64_t* counts, double* lat_us,
                                             int serve) {
  try {
    const cs::FMIndex idx = cs::FMIndex::borrow(h);
    if (serve) idx.serve(true);
    for (uint64_t q = 0; q < npat; ++q) {
      const std::string_view p(reinterpret_cast<const char*>(pats + q * m), m);
      const auto t0 = std::chrono::steady_clock::now();
      counts[q] = idx.count(p);
      const auto t1 = std::chrono::steady_clock::now();
      lat_us[q] = std::chrono::duration<double, std::micro>(t1 - t0).count();
    }
    if (serve) idx.serve(false);
  } catch (const std::exception&) {
    if (serve) {
      try {
        cs::FMIndex::borrow(h).serve(false);
      } catch (const std::exception&) {
      }
    }
    return 1;
  }
  return 0;
}
