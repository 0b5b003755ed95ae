// fm_io.hip — on-disk index format and FMIndex::open_directory, and the same image
// exported to / imported from device buffers (index replication across GPUs).
//
// The reference declares open_directory (src/api/fm_index.hpp:20, "TODO: on-disk
// format") and throws (src/api/fm_index.cpp:71-73); its CSIDX serializer
// (src/serialization/serialization.{hpp,cpp}) is unwired and its writer never
// terminates (align_to, serialization.cpp:44-54).  SURVEY.md §8(f) item 2: an
// on-disk format so a prebuilt multi-GB index is uploaded instead of rebuilt.
//
// Directory layout (all little-endian raw arrays, exactly the HBM images):
//   cs_fmindex.meta  "key value" lines: format, n, stride, line_bytes, line_bits,
//                    nlines, nsamples, nisa, ptab_k, ptab_sigma, lf_exact, has_text,
//                    wide, line_fmt, levels, nwalk, walk_marks, has_wssa, nlctx, lctx_q/sb/eb, pstride, nlmodel, lmodel_shift, ptab_rec, has_sa, has_dtext,
//                    xstride (inverse-SA sample stride), nwssa (walk position samples),
//                    wssa_eb (their bytes per entry: 4, 5 = 40-bit, 8 = older wide images),
//                    active <symbol> <mask>
//   table.bin        NodeTable (fm_device.hpp)
//   lines.bin        the rank lines (8 wavelet levels, or one occurrence-line array)
//   ssa.bin          sampled SA              isa.bin   inverse-SA samples (u32; u64 if wide)
//   ptab.bin         prefix table (if k > 0) text.bin  the text (if kept, for extract)
//   walk.bin         walk lines                      wssa.bin  their position samples
//   lctx.bin         left contexts (if built)    lmodel.bin  learned-line models
//   sa.bin           full suffix array (if kept)     dtext.bin  the text in HBM (if kept)
// The device image (cs_fm_export_* / cs_fm_import) is the same meta text plus the
// parts table, lines, ssa, isa[, ptab][, walk][, wssa][, lctx] as device buffers.
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <sstream>
#include <string>
#include <vector>
#include <sys/stat.h>

#include "fm_internal.hpp"

namespace fmx {
namespace {

constexpr const char* kFormat = "cs_fmindex/3";  // 3: packed wide prefix-table entries
constexpr size_t kChunk = 256ull << 20;

std::string join(const std::string& dir, const char* f) { return dir + "/" + f; }

cs_status io_fail(const std::string& what) {
  set_error(what + (errno ? std::string(": ") + std::strerror(errno) : std::string()));
  return CS_ERR_INVALID;
}

// device -> file through a pinned bounce buffer
cs_status dump_dev(const std::string& path, const void* d, size_t bytes, void* pinned) {
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) return io_fail("cannot write: " + path);
  for (size_t off = 0; off < bytes; off += kChunk) {
    const size_t c = bytes - off < kChunk ? bytes - off : kChunk;
    hipError_t e = hipMemcpy(pinned, static_cast<const uint8_t*>(d) + off, c, hipMemcpyDeviceToHost);
    if (e != hipSuccess) {
      std::fclose(f);
      return hip_fail(e, "hipMemcpy D2H (save)");
    }
    if (std::fwrite(pinned, 1, c, f) != c) {
      std::fclose(f);
      return io_fail("short write: " + path);
    }
  }
  if (std::fclose(f) != 0) return io_fail("cannot close: " + path);
  return CS_OK;
}

cs_status load_dev(const std::string& path, void* d, size_t bytes, void* pinned) {
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) return io_fail("cannot open: " + path);
  for (size_t off = 0; off < bytes; off += kChunk) {
    const size_t c = bytes - off < kChunk ? bytes - off : kChunk;
    if (std::fread(pinned, 1, c, f) != c) {
      std::fclose(f);
      return io_fail("truncated file: " + path);
    }
    hipError_t e = hipMemcpy(static_cast<uint8_t*>(d) + off, pinned, c, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
      std::fclose(f);
      return hip_fail(e, "hipMemcpy H2D (open)");
    }
  }
  std::fclose(f);
  return CS_OK;
}

struct Pinned {
  void* p = nullptr;
  ~Pinned() { if (p) (void)hipHostFree(p); }
};

// One device array of the index image.
struct Part {
  const char* file;
  void** dptr;
  uint64_t bytes;
};

// The index's device arrays in image order; sizes from the geometry fields, so the
// exporting and the importing side derive the same list from the same meta.
std::vector<Part> index_parts(cs_fm_index* h, bool with_table, bool has_wssa, bool has_sa,
                              bool has_dtext) {
  std::vector<Part> v;
  const uint64_t sb = h->sample_bytes();
  if (with_table) v.push_back({"table.bin", reinterpret_cast<void**>(&h->d_table), sizeof(NodeTable)});
  v.push_back({"lines.bin", &h->d_lines, (uint64_t)h->nlevels * h->nlines * h->line_bytes});
  v.push_back({"ssa.bin", &h->d_ssa, h->nsamples * sb});
  v.push_back({"isa.bin", &h->d_isa, h->nisa * sb});
  if (h->ptab_k) v.push_back({"ptab.bin", &h->d_ptab, h->ptab_entries() * h->ptab_entry_bytes()});
  if (h->nwalk) v.push_back({"walk.bin", &h->d_walk, h->nwalk * 32});
  if (has_wssa) v.push_back({"wssa.bin", &h->d_wssa, h->nwssa * h->wssa_bytes()});
  if (h->nlctx) v.push_back({"lctx.bin", &h->d_lctx, h->nlctx * h->lctx_eb});
  if (h->nlmodel) v.push_back({"lmodel.bin", &h->d_lmodel, h->nlmodel * sizeof(LOccModel)});
  if (has_sa) v.push_back({"sa.bin", &h->d_sa, h->n * 4});
  if (has_dtext) v.push_back({"dtext.bin", &h->d_dtext, h->n});
  return v;
}

std::string meta_text(const cs_fm_index* h, bool has_text) {
  char buf[1024];
  std::snprintf(buf, sizeof buf,
                "format %s\nn %llu\nstride %u\nline_bytes %u\nline_bits %u\nnlines %llu\n"
                "nsamples %llu\nnisa %llu\nptab_k %u\nptab_sigma %u\nlf_exact %d\nhas_text %d\n"
                "wide %d\nline_fmt %u\nlevels %u\nnwalk %llu\nwalk_marks %u\nhas_wssa %d\n"
                "nlctx %llu\nlctx_q %u\nlctx_sb %u\nlctx_eb %u\npstride %u\nnlmodel %llu\n"
                "lmodel_shift %u\nptab_rec %d\nhas_sa %d\nhas_dtext %d\nxstride %u\nnwssa %llu\n"
                "wssa_eb %u\n",
                kFormat, (unsigned long long)h->n, h->stride, h->line_bytes, h->line_bits,
                (unsigned long long)h->nlines, (unsigned long long)h->nsamples,
                (unsigned long long)h->nisa, h->ptab_k, h->ptab_sigma, h->lf_exact ? 1 : 0,
                has_text ? 1 : 0, h->wide ? 1 : 0, h->line_fmt, h->nlevels,
                (unsigned long long)(h->d_walk ? h->nwalk : 0), h->walk_marks, h->d_wssa ? 1 : 0,
                (unsigned long long)(h->d_lctx ? h->nlctx : 0), h->lctx_q, h->lctx_sb, h->lctx_eb,
                h->pstride, (unsigned long long)h->nlmodel, h->lmodel_shift, (int)h->ptab_rec,
                h->d_sa ? 1 : 0, h->d_dtext ? 1 : 0, h->xstride,
                (unsigned long long)(h->d_wssa ? h->nwssa : 0), h->wssa_bytes());
  std::string m(buf);
  for (int c = 0; c < 256; ++c) {
    std::snprintf(buf, sizeof buf, "active %d %u\n", c, h->active_levels[c]);
    m += buf;
  }
  return m;
}

// Fills h's geometry from a meta text; kv receives the flags (has_text, has_wssa).
cs_status meta_parse(const std::string& text, cs_fm_index* h,
                     std::map<std::string, unsigned long long>& kv, const std::string& what) {
  std::istringstream in(text);
  std::string key, val, format;
  while (in >> key >> val) {
    if (key == "format") {
      format = val;
    } else if (key == "active") {
      const int c = std::atoi(val.c_str());
      unsigned m = 0;
      if ((in >> m) && c >= 0 && c < 256) h->active_levels[c] = m;
    } else {
      kv[key] = std::strtoull(val.c_str(), nullptr, 10);
    }
  }
  if (format != kFormat) {
    set_error("not a " + std::string(kFormat) + " index: " + what);
    return CS_ERR_INVALID;
  }
  h->n = kv["n"];
  h->stride = (uint32_t)kv["stride"];
  h->line_bytes = (uint32_t)kv["line_bytes"];
  h->line_bits = (uint32_t)kv["line_bits"];
  h->nlines = kv["nlines"];
  h->nsamples = kv["nsamples"];
  h->nisa = kv["nisa"];
  h->ptab_k = (uint32_t)kv["ptab_k"];
  h->ptab_sigma = (uint32_t)kv["ptab_sigma"];
  h->lf_exact = kv["lf_exact"] != 0;
  h->wide = kv["wide"] != 0;
  h->line_fmt = (uint32_t)kv["line_fmt"];
  h->nlevels = (uint32_t)kv["levels"];
  h->nwalk = kv["nwalk"];
  h->walk_marks = (uint32_t)kv["walk_marks"];
  h->nlctx = kv["nlctx"];  // absent in indexes saved before left contexts: none
  h->lctx_q = (uint32_t)kv["lctx_q"];
  h->lctx_sb = (uint32_t)kv["lctx_sb"];
  h->lctx_eb = (uint32_t)kv["lctx_eb"];
  h->pstride = kv["pstride"] ? (uint32_t)kv["pstride"] : h->stride;  // older images: the SSA's
  h->xstride = kv["xstride"] ? (uint32_t)kv["xstride"] : h->pstride;  // older images: one stride
  h->nwssa = kv.count("nwssa") ? kv["nwssa"] : (kv["has_wssa"] ? h->nisa : 0);
  h->wssa_eb = (uint32_t)kv["wssa_eb"];  // absent in older images: sample_bytes()
  if (h->wssa_eb != 0 && h->wssa_eb != 4 && h->wssa_eb != 5 && h->wssa_eb != 8) {
    set_error("bad wssa_eb in " + what);
    return CS_ERR_INVALID;
  }
  h->nlmodel = kv["nlmodel"];
  h->lmodel_shift = (uint32_t)kv["lmodel_shift"];
  h->ptab_rec = (uint32_t)kv["ptab_rec"];
  if (h->ptab_rec > 3) {
    set_error("bad ptab_rec in " + what);
    return CS_ERR_INVALID;
  }
  return CS_OK;
}

cs_status need_device() {
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count == 0) {
    (void)hipGetLastError();
    set_error("no HIP device: the FM-index engine runs only on the GPU");
    return CS_ERR_NO_DEVICE;
  }
  return CS_OK;
}

// allocate every part (and the overrun flag) of a handle whose geometry is set
cs_status alloc_parts(cs_fm_index* h, const std::vector<Part>& parts) {
  for (const Part& p : parts)  // + kPartPad zeroed bytes: word reads past a part's end
    if (hipMalloc(p.dptr, p.bytes + kPartPad) != hipSuccess ||
        hipMemset(static_cast<uint8_t*>(*p.dptr) + p.bytes, 0, kPartPad) != hipSuccess)
      return hip_fail(hipGetLastError(), "hipMalloc (index image)");
  if (hipMalloc(&h->d_err, 8) != hipSuccess || hipMemset(h->d_err, 0xFF, 8) != hipSuccess)
    return hip_fail(hipGetLastError(), "hipMalloc (index image)");
  return CS_OK;
}

}  // namespace

uint64_t index_hbm_bytes(const cs_fm_index* hc) {
  cs_fm_index* h = const_cast<cs_fm_index*>(hc);  // sizes only
  uint64_t b = 0;
  for (const Part& p : index_parts(h, true, h->d_wssa != nullptr, h->d_sa != nullptr, h->d_dtext != nullptr))
    if (*p.dptr) b += p.bytes;
  if (h->d_ptext) b += h->ptext_bytes();  // derived, not an image part
  b += h->lrec_bytes();                    // the same
  return b;
}

uint64_t device_bytes(const cs_fm_index* hc) {
  cs_fm_index* h = const_cast<cs_fm_index*>(hc);  // sizes only
  uint64_t b = 0;
  // every image part (each allocated with kPartPad zeroed bytes after it), the node table
  // among them
  for (const Part& p : index_parts(h, true, h->d_wssa != nullptr, h->d_sa != nullptr, h->d_dtext != nullptr))
    if (*p.dptr) b += p.bytes + (p.dptr == reinterpret_cast<void**>(&h->d_table) ? 0 : kPartPad);
  if (h->d_ptext) b += h->ptext_bytes() + kPartPad;  // derived parts
  b += h->lrec_bytes();
  if (h->d_prare) b += kMaxExc * 4;
  if (h->d_prare64) b += kMaxExc * 8;
  if (h->d_err) b += 8;
  if (h->scratch.d) b += cs_fm_index::kScratchBytes;  // the small-batch arena
  return b;
}

bool hbm_room(const cs_fm_index* h, uint64_t bytes, uint64_t freed, uint64_t transient) {
  size_t free_b = 0, total_b = 0;
  if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) return false;
  // the built index leaves an eighth free; a replacement (freed > 0) needs both copies
  // for a moment, within 2 GB of the device's free memory
  const uint64_t net = bytes > freed ? bytes - freed : 0;
  if (net + total_b / 8 > free_b + transient || bytes + (2ull << 30) > free_b) return false;
  if (!h->hbm_budget) return true;
  const uint64_t have = index_hbm_bytes(h);
  return have + bytes <= h->hbm_budget + freed;
}

uint64_t hbm_budget_env() {
  const char* e = build_opt("CS_FM_HBM_BUDGET");
  if (!e || !*e) return 0;
  char* end = nullptr;
  const double v = std::strtod(e, &end);
  double mul = 1;
  switch (end && *end ? *end : ' ') {
    case 'K': case 'k': mul = 1e3; break;
    case 'M': case 'm': mul = 1e6; break;
    case 'G': case 'g': mul = 1e9; break;
    case 'T': case 't': mul = 1e12; break;
    default: break;
  }
  return v > 0 ? (uint64_t)(v * mul) : 0;
}

}  // namespace fmx

using namespace fmx;

extern "C" {

cs_status cs_fm_save_directory(const cs_fm_index* hc, const char* dir) {
  if (!hc || !dir) {
    set_error("null argument");
    return CS_ERR_INVALID;
  }
  cs_fm_index* h = const_cast<cs_fm_index*>(hc);  // parts are only read
  DeviceScope ds;
  FMX_HIP(ds.enter(h->device));
  errno = 0;
  if (mkdir(dir, 0755) != 0 && errno != EEXIST) return io_fail(std::string("cannot create: ") + dir);
  errno = 0;
  const std::string d(dir);
  Pinned pin;
  FMX_HIP(hipHostMalloc(&pin.p, kChunk, hipHostMallocDefault));
  cs_status s;
  for (const Part& p : index_parts(h, false, h->d_wssa != nullptr, h->d_sa != nullptr, h->d_dtext != nullptr))
    if ((s = dump_dev(join(d, p.file), *p.dptr, p.bytes, pin.p)) != CS_OK) return s;
  {
    FILE* f = std::fopen(join(d, "table.bin").c_str(), "wb");
    if (!f || std::fwrite(&h->h_table, sizeof h->h_table, 1, f) != 1) {
      if (f) std::fclose(f);
      return io_fail("cannot write: " + join(d, "table.bin"));
    }
    std::fclose(f);
  }
  // the host text_ copy, unless the text travels as the device part dtext.bin
  const bool has_text = h->h_text.size() == h->n && h->n && !h->d_dtext;
  if (has_text) {
    FILE* f = std::fopen(join(d, "text.bin").c_str(), "wb");
    if (!f || std::fwrite(h->h_text.data(), 1, h->n, f) != h->n) {
      if (f) std::fclose(f);
      return io_fail("cannot write: " + join(d, "text.bin"));
    }
    std::fclose(f);
  }
  const std::string meta = meta_text(h, has_text);
  FILE* f = std::fopen(join(d, "cs_fmindex.meta").c_str(), "w");
  if (!f || std::fwrite(meta.data(), 1, meta.size(), f) != meta.size()) {
    if (f) std::fclose(f);
    return io_fail("cannot write: " + join(d, "cs_fmindex.meta"));
  }
  std::fclose(f);
  return CS_OK;
}

cs_status cs_fm_open_directory_on(const char* dir, int device, cs_fm_index** out) {
  if (!dir || !out) {
    set_error("null argument");
    return CS_ERR_INVALID;
  }
  *out = nullptr;
  {  // a single file: the reference's CSIDX format (fm_csidx.cpp)
    struct stat sb;
    if (stat(dir, &sb) == 0 && S_ISREG(sb.st_mode)) return cs_fm_open_csidx(dir, device, out);
  }
  const std::string d(dir);
  errno = 0;
  std::string meta;
  {
    FILE* f = std::fopen(join(d, "cs_fmindex.meta").c_str(), "r");
    if (!f) {
      // a reference-style index directory holding only its source text (the shipped
      // sample.csidx/text.txt): built here as tools/build_index.cpp does — '$' appended
      // unless the text ends in '$' or '\0', ssa_stride 32
      FILE* t = std::fopen(join(d, "text.txt").c_str(), "rb");
      if (!t) return io_fail("cannot open: " + join(d, "cs_fmindex.meta"));
      std::vector<uint8_t> text;
      uint8_t buf[1 << 16];
      size_t k;
      while ((k = std::fread(buf, 1, sizeof buf, t)) > 0) text.insert(text.end(), buf, buf + k);
      std::fclose(t);
      if (text.empty()) {
        set_error("empty text: " + join(d, "text.txt"));
        return CS_ERR_INVALID;
      }
      if (text.back() != '$' && text.back() != '\0') text.push_back('$');
      cs_build_params bp;
      cs_default_build_params(&bp);
      return cs_fm_build_from_text(text.data(), text.size(), &bp, device, out);
    }
    char buf[4096];
    size_t k;
    while ((k = std::fread(buf, 1, sizeof buf, f)) > 0) meta.append(buf, k);
    std::fclose(f);
  }
  auto* h = new cs_fm_index();
  read_tuning(h);
  std::map<std::string, unsigned long long> kv;
  cs_status s = meta_parse(meta, h, kv, d);
  if (s == CS_OK) s = need_device();
  if (s != CS_OK) {
    delete h;
    return s;
  }
  h->device = device;
  auto fail = [&](cs_status st) {
    cs_fm_destroy(h);
    return st;
  };
  DeviceScope ds;
  if (ds.enter(device) != hipSuccess) return fail(hip_fail(hipGetLastError(), "hipSetDevice"));
  {
    FILE* t = std::fopen(join(d, "table.bin").c_str(), "rb");
    if (!t || std::fread(&h->h_table, sizeof h->h_table, 1, t) != 1) {
      if (t) std::fclose(t);
      return fail(io_fail("cannot read: " + join(d, "table.bin")));
    }
    std::fclose(t);
  }
  const std::vector<Part> parts = index_parts(h, true, kv["has_wssa"] != 0, kv["has_sa"] != 0, kv["has_dtext"] != 0);
  if ((s = alloc_parts(h, parts)) != CS_OK) return fail(s);
  Pinned pin;
  if (hipHostMalloc(&pin.p, kChunk, hipHostMallocDefault) != hipSuccess)
    return fail(hip_fail(hipGetLastError(), "hipHostMalloc"));
  for (const Part& p : parts) {
    if (p.dptr == reinterpret_cast<void**>(&h->d_table)) continue;  // from the host copy below
    if ((s = load_dev(join(d, p.file), *p.dptr, p.bytes, pin.p)) != CS_OK) return fail(s);
  }
  if (hipMemcpy(h->d_table, &h->h_table, sizeof(NodeTable), hipMemcpyHostToDevice) != hipSuccess)
    return fail(hip_fail(hipGetLastError(), "hipMemcpy (open)"));
  if (kv["has_text"]) {
    FILE* t = std::fopen(join(d, "text.bin").c_str(), "rb");
    h->h_text.resize(h->n);
    if (!t || std::fread(h->h_text.data(), 1, h->n, t) != h->n) {
      if (t) std::fclose(t);
      return fail(io_fail("cannot read: " + join(d, "text.bin")));
    }
    std::fclose(t);
  }
  if ((s = derive_parts(h, nullptr)) != CS_OK) return fail(s);
  *out = h;
  return CS_OK;
}

cs_status cs_fm_export_meta(const cs_fm_index* hc, char* meta, uint64_t cap, uint64_t* meta_len,
                            uint64_t* part_bytes, uint32_t* nparts) {
  if (!hc || !meta_len || !nparts) {
    set_error("null argument");
    return CS_ERR_INVALID;
  }
  cs_fm_index* h = const_cast<cs_fm_index*>(hc);
  const std::string m = meta_text(h, false);
  const std::vector<Part> parts = index_parts(h, true, h->d_wssa != nullptr, h->d_sa != nullptr, h->d_dtext != nullptr);
  *meta_len = m.size();
  *nparts = (uint32_t)parts.size();
  if (!meta || cap < m.size() || !part_bytes) {
    set_error("export: meta buffer too small");
    return CS_ERR_CAPACITY;
  }
  std::memcpy(meta, m.data(), m.size());
  for (size_t i = 0; i < parts.size(); ++i) part_bytes[i] = parts[i].bytes;
  return CS_OK;
}

cs_status cs_fm_export_parts(const cs_fm_index* hc, void* const* d_dst, void* stream) {
  if (!hc || !d_dst) {
    set_error("null argument");
    return CS_ERR_INVALID;
  }
  cs_fm_index* h = const_cast<cs_fm_index*>(hc);
  DeviceScope ds;
  FMX_HIP(ds.enter(h->device));
  const std::vector<Part> parts = index_parts(h, true, h->d_wssa != nullptr, h->d_sa != nullptr, h->d_dtext != nullptr);
  for (size_t i = 0; i < parts.size(); ++i)
    if (parts[i].bytes)
      FMX_HIP(hipMemcpyAsync(d_dst[i], *parts[i].dptr, parts[i].bytes, hipMemcpyDeviceToDevice,
                             (hipStream_t)stream));
  return CS_OK;
}

cs_status cs_fm_import(const char* meta, uint64_t meta_len, const void* const* d_src,
                       uint32_t nparts, int device, cs_fm_index** out) {
  if (!meta || !d_src || !out) {
    set_error("null argument");
    return CS_ERR_INVALID;
  }
  *out = nullptr;
  auto* h = new cs_fm_index();
  read_tuning(h);
  std::map<std::string, unsigned long long> kv;
  cs_status s = meta_parse(std::string(meta, meta_len), h, kv, "device image");
  if (s == CS_OK) s = need_device();
  if (s != CS_OK) {
    delete h;
    return s;
  }
  h->device = device;
  auto fail = [&](cs_status st) {
    cs_fm_destroy(h);
    return st;
  };
  DeviceScope ds;
  if (ds.enter(device) != hipSuccess) return fail(hip_fail(hipGetLastError(), "hipSetDevice"));
  const std::vector<Part> parts = index_parts(h, true, kv["has_wssa"] != 0, kv["has_sa"] != 0, kv["has_dtext"] != 0);
  if (parts.size() != nparts) {
    set_error("import: the image has a different number of parts than its meta");
    return fail(CS_ERR_INVALID);
  }
  if ((s = alloc_parts(h, parts)) != CS_OK) return fail(s);
  for (size_t i = 0; i < parts.size(); ++i)
    if (parts[i].bytes &&
        hipMemcpy(*parts[i].dptr, d_src[i], parts[i].bytes, hipMemcpyDeviceToDevice) != hipSuccess)
      return fail(hip_fail(hipGetLastError(), "hipMemcpy (import)"));
  if (hipMemcpy(&h->h_table, h->d_table, sizeof(NodeTable), hipMemcpyDeviceToHost) != hipSuccess)
    return fail(hip_fail(hipGetLastError(), "hipMemcpy (import table)"));
  if ((s = derive_parts(h, nullptr)) != CS_OK) return fail(s);
  *out = h;
  return CS_OK;
}

cs_status cs_fm_export_part_ptrs(const cs_fm_index* hc, const void** d_parts, uint32_t cap) {
  if (!hc || !d_parts) {
    set_error("null argument");
    return CS_ERR_INVALID;
  }
  cs_fm_index* h = const_cast<cs_fm_index*>(hc);  // parts are only read
  const std::vector<Part> parts = index_parts(h, true, h->d_wssa != nullptr, h->d_sa != nullptr, h->d_dtext != nullptr);
  if (cap < parts.size()) {
    set_error("export: part pointer array too small");
    return CS_ERR_CAPACITY;
  }
  for (size_t i = 0; i < parts.size(); ++i) d_parts[i] = *parts[i].dptr;
  return CS_OK;
}

cs_status cs_fm_import_alloc(const char* meta, uint64_t meta_len, int device, cs_fm_index** out,
                             void** d_parts, uint32_t nparts) {
  if (!meta || !out || !d_parts) {
    set_error("null argument");
    return CS_ERR_INVALID;
  }
  *out = nullptr;
  auto* h = new cs_fm_index();
  read_tuning(h);
  std::map<std::string, unsigned long long> kv;
  cs_status s = meta_parse(std::string(meta, meta_len), h, kv, "device image");
  if (s == CS_OK) s = need_device();
  if (s != CS_OK) {
    delete h;
    return s;
  }
  h->device = device;
  auto fail = [&](cs_status st) {
    cs_fm_destroy(h);
    return st;
  };
  DeviceScope ds;
  if (ds.enter(device) != hipSuccess) return fail(hip_fail(hipGetLastError(), "hipSetDevice"));
  const std::vector<Part> parts = index_parts(h, true, kv["has_wssa"] != 0, kv["has_sa"] != 0, kv["has_dtext"] != 0);
  if (parts.size() != nparts) {
    set_error("import: the image has a different number of parts than its meta");
    return fail(CS_ERR_INVALID);
  }
  if ((s = alloc_parts(h, parts)) != CS_OK) return fail(s);
  for (size_t i = 0; i < parts.size(); ++i) d_parts[i] = *parts[i].dptr;
  *out = h;
  return CS_OK;
}

cs_status cs_fm_import_commit(cs_fm_index* h) {
  if (!h) {
    set_error("null index handle");
    return CS_ERR_INVALID;
  }
  DeviceScope ds;
  FMX_HIP(ds.enter(h->device));
  FMX_HIP(hipDeviceSynchronize());  // the caller's copies into the parts (any stream)
  FMX_HIP(hipMemcpy(&h->h_table, h->d_table, sizeof(NodeTable), hipMemcpyDeviceToHost));
  return derive_parts(h, nullptr);
}

}  // extern "C"
