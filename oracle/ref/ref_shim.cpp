// ref_shim.cpp — extern "C" handle around the GENUINE reference cs::FMIndex.
//
// TEST INFRASTRUCTURE ONLY: built by `make -C oracle ref` into oracle/_ref/ from the
// reference sources in place.  Used in the build container to (a) time the real
// reference count() beside the C restatement (calibration) and (b)
// produce golden vectors at sizes where the reference's naive suffix sort
// (src/core/sais.hpp:8-16, O(n^2 log n)) is too slow: ref_build_from_sa fills the
// index members exactly as build_from_text does (src/api/fm_index.cpp:16-69) from
// a suffix array the caller supplies (checked equal to build_sa_naive at small n
// by tests/test_oracle_golden.py).  Technique per SURVEY.md §7 step 1.
#include <algorithm>
#include <array>
#include <chrono>
#include <thread>
#include <cstdint>
#include <cstring>
#include <filesystem>
#include <stdexcept>
#include <string>
#include <string_view>
#include <vector>

#define private public
#include "api/fm_index.hpp"
#undef private
#include "core/bwt.hpp"
#include "serialization/serialization.hpp"

extern "C" {

void* ref_build_from_text(const uint8_t* text, uint64_t n, uint32_t stride) {
  cs::BuildParams bp;
  bp.ssa_stride = stride;
  std::string t(reinterpret_cast<const char*>(text), n);
  return new cs::FMIndex(cs::FMIndex::build_from_text(t, bp));
}

void* ref_build_from_sa(const uint8_t* text, uint64_t n, const uint32_t* sa, uint32_t stride) {
  auto* idx = new cs::FMIndex();
  idx->text_.assign(reinterpret_cast<const char*>(text), n);
  idx->meta_.n = n;
  idx->sa_.assign(sa, sa + n);
  idx->bwt_ = cs::build_bwt_from_sa(idx->text_, idx->sa_);
  idx->C_.assign(257, 0u);
  std::array<uint32_t, 256> freq{};
  for (unsigned char ch : idx->bwt_) freq[ch]++;
  uint32_t cum = 0;
  for (int c = 0; c < 256; ++c) { idx->C_[c] = cum; cum += freq[c]; }
  idx->C_[256] = cum;
  std::vector<uint8_t> bwt_bytes(idx->bwt_.begin(), idx->bwt_.end());
  idx->wavelet_.build(bwt_bytes);
  idx->ssa_.stride = stride;
  const size_t ns = (idx->sa_.size() + stride - 1) / stride;
  idx->ssa_.samples.resize(ns);
  for (size_t i = 0; i < idx->sa_.size(); ++i)
    if (i % stride == 0) idx->ssa_.samples[i / stride] = idx->sa_[i];
  return idx;
}

void ref_free(void* h) { delete static_cast<cs::FMIndex*>(h); }

void ref_get_sa(void* h, uint32_t* out) {
  auto* idx = static_cast<cs::FMIndex*>(h);
  std::memcpy(out, idx->sa_.data(), idx->sa_.size() * 4);
}

uint64_t ref_count(void* h, const uint8_t* p, uint64_t m) {
  return static_cast<cs::FMIndex*>(h)->count(std::string_view(reinterpret_cast<const char*>(p), m));
}

// returns number of positions (<= cap), or -1 on exception
int64_t ref_locate(void* h, const uint8_t* p, uint64_t m, uint64_t limit, uint64_t* out, uint64_t cap) {
  try {
    auto v = static_cast<cs::FMIndex*>(h)->locate(
        std::string_view(reinterpret_cast<const char*>(p), m), limit);
    const uint64_t k = std::min<uint64_t>(v.size(), cap);
    std::memcpy(out, v.data(), k * 8);
    return (int64_t)v.size();
  } catch (...) {
    return -1;
  }
}

// Count-only reference index at sizes where the reference's own build (naive suffix
// sort, single-threaded wavelet partitions) cannot run: the eight wavelet levels'
// packed words (e.g. the oracle's levels of the same BWT, checked bit-equal by
// tests/test_oracle_golden.py) go through the genuine BitVector::build_from_words
// (src/core/bitvector.cpp:98-159), C_ as build_from_text computes it
// (src/api/fm_index.cpp:36-47); FMIndex::count (:79-101) then runs unmodified.
void* ref_build_count_only(const uint64_t* const* level_words, uint64_t nwords, uint64_t n,
                           const uint64_t* C257) {
  auto* idx = new cs::FMIndex();
  idx->meta_.n = n;
  idx->wavelet_.n_ = n;
  for (int l = 0; l < 8; ++l) {
    std::vector<uint64_t> w(level_words[l], level_words[l] + nwords);
    idx->wavelet_.levels_[l].build_from_words(w, n);
  }
  idx->C_.assign(257, 0u);
  for (int c = 0; c < 257; ++c) idx->C_[c] = static_cast<uint32_t>(C257[c]);
  return idx;
}

// locate() on such an index: the members it reads besides the wavelet levels and C_
// (src/api/fm_index.cpp:107-157) — bwt_ (LF, fm_index.hpp:62-66) and the row-sampled
// ssa_ (src/core/ssa.hpp:7-13) — taken from arrays of the same BWT.
void ref_attach_locate(void* h, const uint8_t* bwt, uint64_t n, const uint32_t* ssa,
                       uint64_t nsamples, uint32_t stride) {
  auto* idx = static_cast<cs::FMIndex*>(h);
  idx->bwt_.assign(reinterpret_cast<const char*>(bwt), n);
  idx->ssa_.stride = stride;
  idx->ssa_.samples.assign(ssa, ssa + nsamples);
}

// locate(pattern, limit) of npat patterns on nthreads host threads (disjoint slices):
// nout[q] = number of positions (-1: the reference threw), the first min(nout, cap)
// of them at out[q * cap ..], per-call latency in ns.
void ref_locate_batch(void* h, const uint8_t* pats, const uint64_t* offs, uint64_t npat,
                      uint64_t limit, int nthreads, uint64_t cap, int64_t* nout, uint64_t* out,
                      uint64_t* lat_ns) {
  const auto* idx = static_cast<const cs::FMIndex*>(h);
  if (nthreads < 1) nthreads = 1;
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; ++t) {
    th.emplace_back([=] {
      const uint64_t a = npat * t / nthreads, b = npat * (t + 1) / nthreads;
      for (uint64_t q = a; q < b; ++q) {
        const auto t0 = std::chrono::steady_clock::now();
        try {
          auto v = idx->locate(std::string_view(reinterpret_cast<const char*>(pats + offs[q]),
                                                offs[q + 1] - offs[q]), limit);
          nout[q] = (int64_t)v.size();
          std::memcpy(out + q * cap, v.data(), std::min<uint64_t>(v.size(), cap) * 8);
        } catch (...) {
          nout[q] = -1;
        }
        const auto t1 = std::chrono::steady_clock::now();
        if (lat_ns)
          lat_ns[q] = (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count();
      }
    });
  }
  for (auto& x : th) x.join();
}

// count() of npat patterns on nthreads host threads (disjoint contiguous slices; the
// reference's count is const and re-entrant), per-call latency in ns.
void ref_count_batch(void* h, const uint8_t* pats, const uint64_t* offs, uint64_t npat,
                     int nthreads, uint64_t* out, uint64_t* lat_ns) {
  const auto* idx = static_cast<const cs::FMIndex*>(h);
  if (nthreads < 1) nthreads = 1;
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; ++t) {
    th.emplace_back([=] {
      const uint64_t a = npat * t / nthreads, b = npat * (t + 1) / nthreads;
      for (uint64_t q = a; q < b; ++q) {
        const auto t0 = std::chrono::steady_clock::now();
        out[q] = idx->count(std::string_view(reinterpret_cast<const char*>(pats + offs[q]),
                                             offs[q + 1] - offs[q]));
        const auto t1 = std::chrono::steady_clock::now();
        if (lat_ns)
          lat_ns[q] = (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count();
      }
    });
  }
  for (auto& x : th) x.join();
}

uint64_t ref_wt_rank(void* h, uint8_t c, uint64_t i) {
  return static_cast<cs::FMIndex*>(h)->wavelet_.rank(c, i);
}

uint64_t ref_level_rank1(void* h, int level, uint64_t i) {
  return static_cast<cs::FMIndex*>(h)->wavelet_.levels_[level].rank1(i);
}

// CSIDX through the reference's own mmap reader (src/serialization/serialization.cpp:153-335):
// the file's sections exactly as cs::IndexReader returns them (pointers into its mapping).
// Returns a handle, or nullptr with the exception's text in err.
void* ref_csidx_open(const char* path, char* err, uint64_t errcap) {
  try {
    return new cs::IndexReader(path);
  } catch (const std::exception& e) {
    if (err && errcap) {
      std::strncpy(err, e.what(), errcap - 1);
      err[errcap - 1] = 0;
    }
    return nullptr;
  }
}
void ref_csidx_close(void* h) { delete static_cast<cs::IndexReader*>(h); }
// header fields: text_len, flags, version
void ref_csidx_header(void* h, uint64_t* text_len, uint32_t* flags, uint32_t* version) {
  const cs::IndexHeader* hd = static_cast<cs::IndexReader*>(h)->header();
  *text_len = hd->text_len;
  *flags = hd->flags;
  *version = hd->version;
}
// section `which` (0 text, 1 bwt, 2 C, 3 ssa): its element count and data pointer
// (null when absent); stride for the SSA
const void* ref_csidx_section(void* h, int which, uint64_t* count, uint32_t* stride) {
  auto* r = static_cast<cs::IndexReader*>(h);
  size_t k = 0;
  const void* p = nullptr;
  if (which == 0) p = r->get_text(&k);
  else if (which == 1) p = r->get_bwt(&k);
  else if (which == 2) p = r->get_c_array(&k);
  else p = r->get_ssa(&k, stride);
  *count = p ? k : 0;
  return p;
}

}  // extern "C"
