// fm_csidx.cpp — the reference's designed on-disk format, CSIDX
// (src/serialization/serialization.hpp:1-83, writer serialization.cpp:26-147, mmap reader
// :153-335), read and written over the C ABI.  The reference never wired it to FMIndex and
// its writer does not terminate (align_to never advances, serialization.cpp:44-54), so no
// reference-written file exists; this follows the documented layout:
//
//   IndexHeader (88 B): magic "CSIDX\0\0\0", u16 version = 1, u16 reserved, u32 flags,
//                       u64 text_len, u64 offsets[8] (header, text, bwt, C, ssa, wavelet,
//                       vEB, footer; 0 = absent)
//   text    [u64 len][len bytes]                       (8-B aligned, as every section)
//   bwt     [u64 count][count bytes]
//   C       [u64 count][count x u32]                   (the reference's C_, 257 entries)
//   ssa     [u32 stride][pad to 8][u64 count][count x u32]
//   footer  u64 0x444E4553435300 ("CSEND")
//
// The wavelet and vEB sections (the reference's BitVector tables and node layout) are not
// written — the engine rebuilds its own rank structures from the BWT — and are ignored on
// reading.  Opening takes the BWT and the SSA as cs_fm_create does (no suffix sorting) and
// the text, when present, for extract.
#include <hip/hip_runtime.h>

#include <sys/stat.h>

#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/cs_fmindex.h"
#include "../../include/cs_fmindex_diag.h"

namespace fmx {
void set_error(const std::string& msg);  // fm_capi.hip: cs_fm_last_error()'s text
}

namespace {

cs_status report(cs_status s, const std::string& msg) {
  fmx::set_error(msg);
  return s;
}

constexpr uint64_t kFooter = 0x444E4553435300ull;
constexpr int kSections = 8;
enum { kText = 1, kBwt = 2, kCArr = 3, kSsa = 4 };

struct Header {
  char magic[8];
  uint16_t version;
  uint16_t reserved;
  uint32_t flags;
  uint64_t text_len;
  uint64_t offsets[kSections];
};
static_assert(sizeof(Header) == 88, "CSIDX header is 88 bytes (serialization.hpp:81)");

cs_status fail(cs_status s, const std::string& msg, std::string* err) {
  if (err) *err = msg;
  return s;
}

bool section(const std::vector<uint8_t>& f, uint64_t off, uint64_t elem, uint64_t& count,
             const uint8_t*& data) {
  if (off == 0 || off % 8 || off + 8 > f.size()) return false;
  std::memcpy(&count, f.data() + off, 8);
  if (elem && count > (f.size() - off - 8) / elem) return false;
  data = f.data() + off + 8;
  return true;
}

struct Writer {
  std::FILE* f = nullptr;
  uint64_t at = 0;
  bool ok = true;
  void raw(const void* p, uint64_t n) {
    if (n && std::fwrite(p, 1, n, f) != n) ok = false;
    at += n;
  }
  void align8() {
    static const uint8_t z[8] = {0};
    raw(z, (8 - at % 8) % 8);  // the padding the reference's align_to meant to write
  }
  template <class T>
  void array(const T* p, uint64_t count) {
    raw(&count, 8);
    raw(p, count * sizeof(T));
  }
};

// parse + validate; on success fills the arrays (shared by open and the CPU-side check)
cs_status csidx_parse(const std::vector<uint8_t>& f, std::vector<uint8_t>& bwt, std::vector<uint32_t>& ssa,
                         uint32_t& stride, std::vector<uint8_t>& text, bool& has_text, std::string* err) {
  Header hd;
  if (f.size() < sizeof hd) return fail(CS_ERR_INVALID, "CSIDX: file too small to contain header", err);
  std::memcpy(&hd, f.data(), sizeof hd);
  if (std::memcmp(hd.magic, "CSIDX", 5) != 0 || hd.version != 1)
    return fail(CS_ERR_INVALID, "Invalid index file: bad magic or version", err);  // serialization.cpp:174
  uint64_t nb = 0, ns = 0;
  const uint8_t *pb = nullptr, *ps = nullptr;
  if (!section(f, hd.offsets[kBwt], 1, nb, pb)) return fail(CS_ERR_INVALID, "CSIDX: no BWT section", err);
  if (hd.text_len != nb) return fail(CS_ERR_INVALID, "CSIDX: text_len differs from the BWT's length", err);
  const uint64_t so = hd.offsets[kSsa];
  if (so == 0 || so % 8 || so + 8 > f.size()) return fail(CS_ERR_INVALID, "CSIDX: no SSA section", err);
  std::memcpy(&stride, f.data() + so, 4);
  if (!section(f, so + 8, 4, ns, ps)) return fail(CS_ERR_INVALID, "CSIDX: truncated SSA section", err);
  if (stride == 0 || ns != (nb + stride - 1) / stride)
    return fail(CS_ERR_INVALID, "CSIDX: the SSA must hold ceil(n / stride) samples", err);
  if (nb >= (1ull << 32)) return fail(CS_ERR_UNSUPPORTED, "CSIDX: u32 samples need n < 2^32", err);
  bwt.assign(pb, pb + nb);
  ssa.resize(ns);
  if (ns) std::memcpy(ssa.data(), ps, ns * 4);
  for (uint64_t k = 0; k < ns; ++k)
    if (ssa[k] >= nb) return fail(CS_ERR_INVALID, "CSIDX: an SSA sample past the text", err);
  // C[] when present must be the BWT's cumulative histogram (fm_index.cpp:36-47)
  uint64_t nc = 0;
  const uint8_t* pc = nullptr;
  if (hd.offsets[kCArr]) {
    if (!section(f, hd.offsets[kCArr], 4, nc, pc)) return fail(CS_ERR_INVALID, "CSIDX: truncated C section", err);
    if (nc) {
      uint64_t hist[256] = {0};
      for (uint64_t i = 0; i < nb; ++i) ++hist[bwt[i]];
      uint64_t cum = 0;
      for (uint64_t c = 0; c < nc && c <= 256; ++c) {
        uint32_t v;
        std::memcpy(&v, pc + 4 * c, 4);
        if (v != cum) return fail(CS_ERR_INVALID, "CSIDX: the C array does not match the BWT", err);
        if (c < 256) cum += hist[c];
      }
    }
  }
  has_text = false;
  uint64_t nt = 0;
  const uint8_t* pt = nullptr;
  if (hd.offsets[kText]) {
    if (!section(f, hd.offsets[kText], 1, nt, pt) || nt != nb)
      return fail(CS_ERR_INVALID, "CSIDX: the text section does not hold text_len bytes", err);
    text.assign(pt, pt + nt);
    has_text = true;
  }
  return CS_OK;
}

// the whole file, sized by fstat and read in one pass (no growth by repeated
// insert, read errors reported)
bool read_file(const char* path, std::vector<uint8_t>& f) {
  std::FILE* fp = std::fopen(path, "rb");
  if (!fp) return false;
  struct stat sb;
  if (fstat(fileno(fp), &sb) != 0 || sb.st_size < 0) {
    std::fclose(fp);
    return false;
  }
  // a regular file: its size, then one read; anything else (a FIFO, /dev/stdin, a procfs
  // file, whose st_size says nothing) in chunks until the end
  bool ok;
  if (S_ISREG(sb.st_mode)) {
    f.resize((size_t)sb.st_size);
    const size_t k = f.empty() ? 0 : std::fread(f.data(), 1, f.size(), fp);
    ok = k == f.size() && !std::ferror(fp);
  } else {
    f.clear();
    uint8_t buf[1 << 16];
    size_t k;
    while ((k = std::fread(buf, 1, sizeof buf, fp)) > 0) f.insert(f.end(), buf, buf + k);
    ok = !std::ferror(fp);
  }
  std::fclose(fp);
  return ok;
}

// The file IndexWriter would write for these members (serialization.cpp:64-147): header,
// text (optional), BWT, C_ (the BWT's cumulative histogram, fm_index.cpp:36-47), SSA, footer.
cs_status csidx_write(const char* path, const uint8_t* bwt, uint64_t n, const uint32_t* ssa, uint64_t ns,
                      uint32_t stride, const uint8_t* text) {
  if (n >= (1ull << 32)) return report(CS_ERR_UNSUPPORTED, "CSIDX: u32 samples need n < 2^32");
  if (stride == 0 || ns != (n + stride - 1) / stride)
    return report(CS_ERR_INVALID, "CSIDX: the SSA must hold ceil(n / stride) samples");
  uint64_t hist[256] = {0};
  for (uint64_t i = 0; i < n; ++i) ++hist[bwt[i]];
  uint32_t c32[257];
  uint64_t cum = 0;
  for (int c = 0; c < 257; ++c) {
    c32[c] = (uint32_t)cum;
    if (c < 256) cum += hist[c];
  }
  Writer w;
  w.f = std::fopen(path, "wb");
  if (!w.f) return report(CS_ERR_INVALID, std::string("cannot write: ") + path);
  Header hd;
  std::memset(&hd, 0, sizeof hd);
  std::memcpy(hd.magic, "CSIDX", 5);
  hd.version = 1;
  hd.text_len = n;
  w.raw(&hd, sizeof hd);  // rewritten with the offsets at the end (IndexWriter::finalize)
  if (text) {
    w.align8();
    hd.offsets[kText] = w.at;
    w.array(text, n);
  }
  w.align8();
  hd.offsets[kBwt] = w.at;
  w.array(bwt, n);
  w.align8();
  hd.offsets[kCArr] = w.at;
  w.array(c32, 257);
  w.align8();
  hd.offsets[kSsa] = w.at;
  w.raw(&stride, 4);
  w.align8();
  w.array(ssa, ns);
  w.align8();
  hd.offsets[7] = w.at;
  w.raw(&kFooter, 8);
  if (std::fseek(w.f, 0, SEEK_SET) != 0) w.ok = false;
  else if (std::fwrite(&hd, sizeof hd, 1, w.f) != 1) w.ok = false;
  if (std::fclose(w.f) != 0) w.ok = false;
  if (!w.ok) return report(CS_ERR_INVALID, std::string("cannot write: ") + path);
  return CS_OK;
}

}  // namespace

extern "C" {

cs_status cs_csidx_check(const char* path, uint64_t* n, uint32_t* ssa_stride, int* has_text) {
  if (!path) return report(CS_ERR_INVALID, "null argument");
  std::vector<uint8_t> f, bwt, text;
  if (!read_file(path, f)) return report(CS_ERR_INVALID, std::string("cannot open: ") + path);
  std::vector<uint32_t> ssa;
  uint32_t stride = 0;
  bool ht = false;
  std::string err;
  const cs_status s = csidx_parse(f, bwt, ssa, stride, text, ht, &err);
  if (s != CS_OK) return report(s, err);
  if (n) *n = bwt.size();
  if (ssa_stride) *ssa_stride = stride;
  if (has_text) *has_text = ht ? 1 : 0;
  return CS_OK;
}

cs_status cs_fm_open_csidx(const char* path, int device, cs_fm_index** out) {
  if (!path || !out) return report(CS_ERR_INVALID, "null argument");
  *out = nullptr;
  std::vector<uint8_t> f;
  if (!read_file(path, f)) return report(CS_ERR_INVALID, std::string("cannot open: ") + path);
  std::vector<uint8_t> bwt, text;
  std::vector<uint32_t> ssa;
  uint32_t stride = 0;
  bool has_text = false;
  std::string err;
  cs_status s = csidx_parse(f, bwt, ssa, stride, text, has_text, &err);
  if (s != CS_OK) return report(s, err);
  return cs_fm_create(bwt.data(), bwt.size(), ssa.data(), ssa.size(), stride,
                      has_text ? text.data() : nullptr, device, out);
}

cs_status cs_fm_save_csidx(const cs_fm_index* h, const char* path) {
  if (!h || !path) return report(CS_ERR_INVALID, "null argument");
  cs_fm_info info;
  cs_status s = cs_fm_get_info(h, &info);
  if (s != CS_OK) return s;
  const uint64_t n = info.n;
  if (n >= (1ull << 32)) return report(CS_ERR_UNSUPPORTED, "CSIDX: u32 samples need n < 2^32");
  // the BWT (device), the SSA, C[], the text (extract; absent when the index cannot give it)
  std::vector<uint8_t> bwt(n ? n : 1), text(n ? n : 1);
  if (n) {  // on the index's device, the caller's current device restored after
    int prev = 0;
    if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(info.device) != hipSuccess)
      return report(CS_ERR_HIP, "hipSetDevice (save_csidx)");
    void* d = nullptr;
    if (hipMalloc(&d, n) != hipSuccess) s = CS_ERR_HIP;
    if (s == CS_OK) s = cs_fm_bwt_device(h, static_cast<uint8_t*>(d), nullptr);
    if (s == CS_OK && hipMemcpy(bwt.data(), d, n, hipMemcpyDeviceToHost) != hipSuccess) s = CS_ERR_HIP;
    if (d) (void)hipFree(d);
    (void)hipSetDevice(prev);
    if (s != CS_OK) return s == CS_ERR_HIP ? report(s, "device copy of the BWT (save_csidx)") : s;
  }
  uint64_t ns = 0;
  s = cs_fm_get_ssa(h, nullptr, 0, &ns);
  if (s != CS_OK && s != CS_ERR_CAPACITY) return s;
  std::vector<uint64_t> s64(ns ? ns : 1);
  if ((s = cs_fm_get_ssa(h, s64.data(), ns, &ns)) != CS_OK) return s;
  std::vector<uint32_t> ssa(ns);
  for (uint64_t k = 0; k < ns; ++k) ssa[k] = (uint32_t)s64[k];
  uint64_t nt = 0;
  const bool has_text = !n || cs_fm_extract(h, 0, n, text.data(), &nt) == CS_OK;
  return csidx_write(path, bwt.data(), n, ssa.data(), ns, info.ssa_stride, has_text ? text.data() : nullptr);
}

cs_status cs_csidx_write(const char* path, const uint8_t* bwt, uint64_t n, const uint32_t* ssa,
                         uint64_t nsamples, uint32_t ssa_stride, const uint8_t* text) {
  if (!path || (n && !bwt) || (nsamples && !ssa)) return report(CS_ERR_INVALID, "null argument");
  return csidx_write(path, bwt, n, ssa, nsamples, ssa_stride, text);
}

}  // extern "C"
