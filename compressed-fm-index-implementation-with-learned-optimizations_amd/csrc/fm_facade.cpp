// fm_facade.cpp — cs::FMIndex (include/cs/fm_index.hpp) over the C ABI.
#include "../../include/cs/fm_index.hpp"

#include <hip/hip_runtime.h>

#include <cstdlib>
#include <stdexcept>

#include "../../include/cs_fmindex.h"

namespace cs {
namespace {

[[noreturn]] void raise(cs_status s) {
  (void)s;
  throw std::runtime_error(cs_fm_last_error());
}

int pick_device() {
  if (const char* e = std::getenv("CS_FM_DEVICE")) return std::atoi(e);
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess) return 0;
  return d;
}

void pack(const std::vector<std::string_view>& pats, std::string& buf, std::vector<uint64_t>& offs) {
  offs.resize(pats.size() + 1);
  offs[0] = 0;
  size_t tot = 0;
  for (auto p : pats) tot += p.size();
  buf.clear();
  buf.reserve(tot);
  for (size_t i = 0; i < pats.size(); ++i) {
    buf.append(pats[i].data(), pats[i].size());
    offs[i + 1] = buf.size();
  }
}

}  // namespace

FMIndex FMIndex::build_from_text(const std::string& text, const BuildParams& p) {
  cs_build_params bp{p.S, p.s, p.ssa_stride, p.eps};
  cs_fm_index* h = nullptr;
  cs_status s = cs_fm_build_from_text(reinterpret_cast<const uint8_t*>(text.data()), text.size(),
                                      &bp, pick_device(), &h);
  if (s != CS_OK) raise(s);
  FMIndex idx;
  idx.meta_.n = text.size();
  idx.h_ = std::shared_ptr<cs_fm_index>(h, cs_fm_destroy);
  return idx;
}

FMIndex FMIndex::open_directory(const std::string& dir) {
  cs_fm_index* h = nullptr;
  cs_status s = cs_fm_open_directory_on(dir.c_str(), pick_device(), &h);
  if (s != CS_OK) raise(s);
  FMIndex idx;
  cs_fm_info info;
  (void)cs_fm_get_info(h, &info);
  idx.meta_.n = info.n;
  idx.h_ = std::shared_ptr<cs_fm_index>(h, cs_fm_destroy);
  return idx;
}

FMIndex FMIndex::borrow(cs_fm_index* h) {
  if (!h) throw std::runtime_error("borrow: null handle");
  FMIndex idx;
  cs_fm_info info;
  if (cs_fm_get_info(h, &info) != CS_OK) throw std::runtime_error(cs_fm_last_error());
  idx.meta_.n = info.n;
  idx.h_ = std::shared_ptr<cs_fm_index>(h, [](cs_fm_index*) {});
  return idx;
}

void FMIndex::save_directory(const std::string& dir) const {
  if (!h_) throw std::runtime_error("save_directory: empty index");
  cs_status s = cs_fm_save_directory(h_.get(), dir.c_str());
  if (s != CS_OK) raise(s);
}

uint64_t FMIndex::count(std::string_view pattern) const {
  if (!h_) return pattern.empty() ? meta_.n : 0;  // fm_index.cpp:80-81 on an empty index
  uint64_t c = 0;
  cs_status s = cs_fm_count(h_.get(), reinterpret_cast<const uint8_t*>(pattern.data()),
                            pattern.size(), &c);
  if (s != CS_OK) raise(s);
  return c;
}

void FMIndex::serve(bool on, uint32_t idle_us) const {
  if (!h_) return;
  cs_status s = on ? cs_fm_serve_start(h_.get(), idle_us) : cs_fm_serve_stop(h_.get());
  if (s != CS_OK) raise(s);
}

std::vector<uint64_t> FMIndex::locate(std::string_view pattern, size_t limit) const {
  std::vector<uint64_t> out;
  if (!h_ || pattern.empty()) return out;  // fm_index.cpp:109
  const uint8_t* p = reinterpret_cast<const uint8_t*>(pattern.data());
  const uint64_t offs[2] = {0, pattern.size()};
  uint64_t oo[2] = {0, 0}, total = 0;
  // size the output from the row range first (min(count, limit) positions)
  cs_status s = cs_fm_locate_batch(h_.get(), p, offs, 1, limit, oo, nullptr, 0, &total, nullptr);
  if (s == CS_OK) return out;
  if (s != CS_ERR_CAPACITY) raise(s);
  out.resize(total);
  s = cs_fm_locate_batch(h_.get(), p, offs, 1, limit, oo, out.data(), out.size(), &total, nullptr);
  if (s != CS_OK) raise(s);
  return out;
}

std::string FMIndex::extract(uint64_t pos, uint64_t len) const {
  if (!h_) return {};
  std::string out;
  if (pos >= meta_.n) return out;  // fm_index.cpp:164
  if (len > meta_.n - pos) len = meta_.n - pos;
  out.resize(len);
  uint64_t got = 0;
  cs_status s = cs_fm_extract(h_.get(), pos, len, reinterpret_cast<uint8_t*>(out.data()), &got);
  if (s != CS_OK) raise(s);
  out.resize(got);
  return out;
}

std::vector<uint64_t> FMIndex::count_batch(const std::vector<std::string_view>& pats) const {
  std::vector<uint64_t> out(pats.size(), 0);
  if (pats.empty()) return out;
  if (!h_) {
    for (size_t i = 0; i < pats.size(); ++i) out[i] = count(pats[i]);
    return out;
  }
  std::string buf;
  std::vector<uint64_t> offs;
  pack(pats, buf, offs);
  cs_status s = cs_fm_count_batch(h_.get(), reinterpret_cast<const uint8_t*>(buf.data()),
                                  offs.data(), pats.size(), out.data(), nullptr);
  if (s != CS_OK) raise(s);
  return out;
}

std::vector<std::vector<uint64_t>> FMIndex::locate_batch(const std::vector<std::string_view>& pats,
                                                         size_t limit) const {
  std::vector<std::vector<uint64_t>> res(pats.size());
  if (pats.empty() || !h_) return res;
  std::string buf;
  std::vector<uint64_t> offs, oo(pats.size() + 1, 0), pos;
  pack(pats, buf, offs);
  uint64_t total = 0;
  const uint8_t* p = reinterpret_cast<const uint8_t*>(buf.data());
  cs_status s = cs_fm_locate_batch(h_.get(), p, offs.data(), pats.size(), limit, oo.data(), nullptr,
                                   0, &total, nullptr);
  if (s == CS_ERR_CAPACITY) {
    pos.resize(total);
    s = cs_fm_locate_batch(h_.get(), p, offs.data(), pats.size(), limit, oo.data(), pos.data(),
                           pos.size(), &total, nullptr);
  }
  if (s != CS_OK) raise(s);
  for (size_t q = 0; q < pats.size(); ++q) res[q].assign(pos.begin() + oo[q], pos.begin() + oo[q + 1]);
  return res;
}

}  // namespace cs
