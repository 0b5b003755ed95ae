// cs/fm_index.hpp — drop-in replacement for the reference's src/api/fm_index.hpp.
//
// Same namespace, class, member names, argument meaning, return types and
// exceptions as cs::FMIndex (src/api/fm_index.hpp:11-67); the work runs on the GPU
// through the C ABI in cs_fmindex.h (implementation: csrc/fm_facade.cpp inside
// libcs_fmindex.so).  Additions: count_batch / locate_batch (one launch for many
// patterns), save_directory (the on-disk format open_directory reads), handle()
// for the raw ABI, borrow() to wrap an ABI handle and serve() (resident
// single-pattern server).  Errors are
// std::runtime_error with the reference's message text ("locate: LF walk exceeded
// text length").
//
// Semantics kept from the reference: plain suffix order and a
// cyclic BWT, so callers append their own unique smallest terminator as before;
// count("") == n while locate("") is empty; locate returns BWT-row order, at most
// `limit` positions.  Copies share the immutable device index.
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <string_view>
#include <vector>

struct cs_fm_index;

namespace cs {

struct BuildParams {  // fm_index.hpp:11-14
  uint32_t S = 512, s = 64, ssa_stride = 32;
  double eps = 1.0;
};
struct IndexMeta {  // fm_index.hpp:15
  uint64_t n = 0;
  uint32_t sigma = 256;
};

class FMIndex {
 public:
  FMIndex() = default;
  // Builds on the current HIP device (hipGetDevice), or CS_FM_DEVICE if set.
  static FMIndex build_from_text(const std::string& text, const BuildParams& p);
  // Opens an index written by save_directory (the reference's TODO, fm_index.hpp:20;
  // it throws there).  Throws std::runtime_error("cannot open: ...") otherwise.
  static FMIndex open_directory(const std::string& dir);
  void save_directory(const std::string& dir) const;

  uint64_t count(std::string_view pattern) const;
  std::vector<uint64_t> locate(std::string_view pattern, size_t limit = 100000) const;
  std::string extract(uint64_t pos, uint64_t len) const;

  // Batched forms: one device launch for the whole batch.
  std::vector<uint64_t> count_batch(const std::vector<std::string_view>& patterns) const;
  std::vector<std::vector<uint64_t>> locate_batch(const std::vector<std::string_view>& patterns,
                                                  size_t limit = 100000) const;

  // Serving mode for single-pattern count(): a resident wave answers from a pinned
  // mailbox instead of one kernel launch per call (cs_fm_serve_start / _stop).
  void serve(bool on = true, uint32_t idle_us = 0) const;

  uint64_t size() const { return meta_.n; }
  const cs_fm_index* handle() const { return h_.get(); }
  // Wraps an index built or opened through the C ABI without taking ownership
  // (the caller keeps it alive and destroys it).
  static FMIndex borrow(cs_fm_index* h);

 private:
  IndexMeta meta_;
  std::shared_ptr<cs_fm_index> h_;
};

}  // namespace cs
