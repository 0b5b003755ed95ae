// ref_golden.cpp — golden-vector generator driven by the GENUINE reference.
//
// TEST INFRASTRUCTURE ONLY.  Compiled by oracle/Makefile against the reference
// sources where they lie under /root/reference (never copied); the binary lands
// in oracle/_ref/ (git-ignored) and is run only in the build container by
// tests/golden/make_golden.py.  It never travels to the GPU box as a dependency
// of anything: the GPU box uses the committed fixtures in tests/golden/.
//
// Modes (all inputs binary files written by make_golden.py):
//   fm <text> <patterns> <ssa_stride> <limit>
//        cs::FMIndex::build_from_text (src/api/fm_index.cpp:16-69), then per
//        pattern: count (:79-101) and locate (:107-157), exceptions reported.
//   bv <bits>           cs::BitVector::build + rank1/rank0 at every i in [0, n+2)
//                       (src/core/bitvector.cpp:14-92, :165-230)
//   wt <bytes> <syms>   cs::WaveletTree::build + rank(c, i) for every listed c and
//                       every i in [0, n+2), plus access(i) (src/core/wavelet.cpp)
//   lv <text>           per-level rank1 of the index's wavelet levels at a spread
//                       of positions (layout pin for the device re-layout)
// Pattern file: u32 count, then per pattern u32 length + bytes.
#include <cstdint>
#include <cstdio>
#include <fstream>
#include <iostream>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "api/fm_index.hpp"
#include "core/bitvector.hpp"
#include "core/wavelet.hpp"

static std::string slurp_file(const char* p) {
  std::ifstream f(p, std::ios::binary);
  if (!f) throw std::runtime_error(std::string("cannot open ") + p);
  return std::string((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

static std::vector<std::string> read_patterns(const char* p) {
  std::string raw = slurp_file(p);
  std::vector<std::string> out;
  size_t off = 0;
  auto rd32 = [&](void) {
    uint32_t v;
    std::memcpy(&v, raw.data() + off, 4);
    off += 4;
    return v;
  };
  uint32_t k = rd32();
  for (uint32_t i = 0; i < k; ++i) {
    uint32_t m = rd32();
    out.emplace_back(raw.data() + off, m);
    off += m;
  }
  return out;
}

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: ref_golden fm|bv|wt|lv ...\n");
    return 2;
  }
  std::string mode = argv[1];
  if (mode == "fm") {
    std::string text = slurp_file(argv[2]);
    auto pats = read_patterns(argv[3]);
    cs::BuildParams bp;
    bp.ssa_stride = (uint32_t)std::stoul(argv[4]);
    size_t limit = (size_t)std::stoull(argv[5]);
    cs::FMIndex idx = cs::FMIndex::build_from_text(text, bp);
    for (const auto& p : pats) {
      uint64_t c = idx.count(p);
      std::printf("C %llu\n", (unsigned long long)c);
      try {
        auto pos = idx.locate(p, limit);
        std::printf("L %zu", pos.size());
        for (auto v : pos) std::printf(" %llu", (unsigned long long)v);
        std::printf("\n");
      } catch (const std::exception& e) {
        std::printf("E %s\n", e.what());
      }
    }
    // extract at a few positions (fm_index.cpp:163-167)
    const uint64_t n = text.size();
    const uint64_t probes[][2] = {{0, 3}, {1, 3}, {n / 2, 5}, {n ? n - 1 : 0, 10}, {n, 1}, {n + 5, 2}};
    for (auto& pr : probes) {
      std::string s = idx.extract(pr[0], pr[1]);
      std::printf("X %llu %llu %zu", (unsigned long long)pr[0], (unsigned long long)pr[1], s.size());
      for (unsigned char ch : s) std::printf(" %u", ch);
      std::printf("\n");
    }
    return 0;
  }
  if (mode == "bv") {
    std::string raw = slurp_file(argv[2]);
    std::vector<uint8_t> bits(raw.begin(), raw.end());
    cs::BitVector bv;
    bv.build(bits);
    const size_t n = bits.size();
    std::printf("N %zu %zu\n", n, bv.count_ones());
    for (size_t i = 0; i < n + 2; ++i) std::printf("%zu %zu\n", bv.rank1(i), bv.rank0(i));
    return 0;
  }
  if (mode == "wt") {
    std::string raw = slurp_file(argv[2]);
    std::vector<uint8_t> seq(raw.begin(), raw.end());
    cs::WaveletTree wt;
    wt.build(seq);
    const size_t n = seq.size();
    std::printf("N %zu\n", n);
    std::stringstream ss(argv[3]);
    std::string tok;
    while (std::getline(ss, tok, ',')) {
      unsigned c = (unsigned)std::stoul(tok);
      std::printf("S %u", c);
      for (size_t i = 0; i < n + 2; ++i) std::printf(" %zu", wt.rank((uint8_t)c, i));
      std::printf("\n");
    }
    std::printf("A");
    for (size_t i = 0; i < n; ++i) std::printf(" %u", (unsigned)wt.access(i));
    std::printf("\n");
    return 0;
  }
  std::fprintf(stderr, "unknown mode\n");
  return 2;
}
