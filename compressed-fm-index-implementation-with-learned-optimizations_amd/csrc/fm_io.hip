// fm_io.hip — on-disk index format and FMIndex::open_directory.
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
//                    wide, line_fmt, levels, nwalk, walk_marks, has_wssa,
//                    active <symbol> <mask>
//   table.bin        NodeTable (fm_device.hpp)
//   lines.bin        the rank lines (8 wavelet levels, or one occurrence-line array)
//   ssa.bin          sampled SA              isa.bin   inverse-SA samples (u32; u64 if wide)
//   ptab.bin         prefix table (if k > 0) text.bin  the text (if kept, for extract)
//   walk.bin         walk lines (occurrence engine)  wssa.bin  their position samples
#include <cerrno>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <sys/stat.h>

#include "fm_internal.hpp"

namespace fmx {
namespace {

constexpr const char* kFormat = "cs_fmindex/2";
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

}  // namespace
}  // namespace fmx

using namespace fmx;

extern "C" {

cs_status cs_fm_save_directory(const cs_fm_index* h, const char* dir) {
  if (!h || !dir) {
    set_error("null argument");
    return CS_ERR_INVALID;
  }
  DeviceScope ds;
  FMX_HIP(ds.enter(h->device));
  errno = 0;
  if (mkdir(dir, 0755) != 0 && errno != EEXIST) return io_fail(std::string("cannot create: ") + dir);
  errno = 0;
  const std::string d(dir);
  Pinned pin;
  FMX_HIP(hipHostMalloc(&pin.p, kChunk, hipHostMallocDefault));
  cs_status s;
  const uint64_t lbytes = (uint64_t)h->nlevels * h->nlines * h->line_bytes;
  if ((s = dump_dev(join(d, "lines.bin"), h->d_lines, lbytes, pin.p)) != CS_OK) return s;
  const uint64_t sb = h->sample_bytes();
  if ((s = dump_dev(join(d, "ssa.bin"), h->d_ssa, h->nsamples * sb, pin.p)) != CS_OK) return s;
  if ((s = dump_dev(join(d, "isa.bin"), h->d_isa, h->nisa * sb, pin.p)) != CS_OK) return s;
  if (h->ptab_k) {
    const uint64_t pb = h->ptab_entries() * h->ptab_entry_bytes();
    if ((s = dump_dev(join(d, "ptab.bin"), h->d_ptab, pb, pin.p)) != CS_OK) return s;
  }
  if (h->d_walk && (s = dump_dev(join(d, "walk.bin"), h->d_walk, h->nwalk * 32, pin.p)) != CS_OK)
    return s;
  if (h->d_wssa && (s = dump_dev(join(d, "wssa.bin"), h->d_wssa, h->nisa * sb, pin.p)) != CS_OK)
    return s;
  {
    FILE* f = std::fopen(join(d, "table.bin").c_str(), "wb");
    if (!f || std::fwrite(&h->h_table, sizeof h->h_table, 1, f) != 1) {
      if (f) std::fclose(f);
      return io_fail("cannot write: " + join(d, "table.bin"));
    }
    std::fclose(f);
  }
  const bool has_text = h->h_text.size() == h->n && h->n;
  if (has_text) {
    FILE* f = std::fopen(join(d, "text.bin").c_str(), "wb");
    if (!f || std::fwrite(h->h_text.data(), 1, h->n, f) != h->n) {
      if (f) std::fclose(f);
      return io_fail("cannot write: " + join(d, "text.bin"));
    }
    std::fclose(f);
  }
  FILE* f = std::fopen(join(d, "cs_fmindex.meta").c_str(), "w");
  if (!f) return io_fail("cannot write: " + join(d, "cs_fmindex.meta"));
  std::fprintf(f, "format %s\nn %llu\nstride %u\nline_bytes %u\nline_bits %u\nnlines %llu\n"
                  "nsamples %llu\nnisa %llu\nptab_k %u\nptab_sigma %u\nlf_exact %d\nhas_text %d\n"
                  "wide %d\nline_fmt %u\nlevels %u\nnwalk %llu\nwalk_marks %u\nhas_wssa %d\n",
               kFormat, (unsigned long long)h->n, h->stride, h->line_bytes, h->line_bits,
               (unsigned long long)h->nlines, (unsigned long long)h->nsamples,
               (unsigned long long)h->nisa, h->ptab_k, h->ptab_sigma, h->lf_exact ? 1 : 0,
               has_text ? 1 : 0, h->wide ? 1 : 0, h->line_fmt, h->nlevels,
               (unsigned long long)(h->d_walk ? h->nwalk : 0), h->walk_marks, h->d_wssa ? 1 : 0);
  for (int c = 0; c < 256; ++c) std::fprintf(f, "active %d %u\n", c, h->active_levels[c]);
  std::fclose(f);
  return CS_OK;
}

cs_status cs_fm_open_directory_on(const char* dir, int device, cs_fm_index** out) {
  if (!dir || !out) {
    set_error("null argument");
    return CS_ERR_INVALID;
  }
  *out = nullptr;
  const std::string d(dir);
  errno = 0;
  FILE* f = std::fopen(join(d, "cs_fmindex.meta").c_str(), "r");
  if (!f) return io_fail("cannot open: " + join(d, "cs_fmindex.meta"));
  std::map<std::string, unsigned long long> kv;
  std::string format;
  auto* h = new cs_fm_index();
  char key[64], val[128];
  while (std::fscanf(f, "%63s %127s", key, val) == 2) {
    if (!std::strcmp(key, "format")) {
      format = val;
    } else if (!std::strcmp(key, "active")) {
      const int c = std::atoi(val);
      unsigned m = 0;
      if (std::fscanf(f, "%u", &m) == 1 && c >= 0 && c < 256) h->active_levels[c] = m;
    } else {
      kv[key] = std::strtoull(val, nullptr, 10);
    }
  }
  std::fclose(f);
  if (format != kFormat) {
    delete h;
    set_error("not a " + std::string(kFormat) + " index: " + d);
    return CS_ERR_INVALID;
  }
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count == 0) {
    delete h;
    (void)hipGetLastError();
    set_error("no HIP device: the FM-index engine runs only on the GPU");
    return CS_ERR_NO_DEVICE;
  }
  h->device = device;
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
  auto fail = [&](cs_status s) {
    cs_fm_destroy(h);
    return s;
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
  Pinned pin;
  if (hipHostMalloc(&pin.p, kChunk, hipHostMallocDefault) != hipSuccess)
    return fail(hip_fail(hipGetLastError(), "hipHostMalloc"));
  const uint64_t lbytes = (uint64_t)h->nlevels * h->nlines * h->line_bytes;
  if (hipMalloc(&h->d_lines, lbytes ? lbytes : 16) != hipSuccess ||
      hipMalloc(&h->d_ssa, h->nsamples ? h->nsamples * h->sample_bytes() : 16) != hipSuccess ||
      hipMalloc(&h->d_isa, h->nisa ? h->nisa * h->sample_bytes() : 16) != hipSuccess ||
      hipMalloc(&h->d_table, sizeof(NodeTable)) != hipSuccess ||
      hipMalloc(&h->d_err, 8) != hipSuccess)
    return fail(hip_fail(hipGetLastError(), "hipMalloc (open)"));
  cs_status s;
  if ((s = load_dev(join(d, "lines.bin"), h->d_lines, lbytes, pin.p)) != CS_OK) return fail(s);
  const uint64_t sb = h->sample_bytes();
  if ((s = load_dev(join(d, "ssa.bin"), h->d_ssa, h->nsamples * sb, pin.p)) != CS_OK) return fail(s);
  if ((s = load_dev(join(d, "isa.bin"), h->d_isa, h->nisa * sb, pin.p)) != CS_OK) return fail(s);
  if (h->ptab_k) {
    const uint64_t pb = h->ptab_entries() * h->ptab_entry_bytes();
    if (hipMalloc(&h->d_ptab, pb) != hipSuccess)
      return fail(hip_fail(hipGetLastError(), "hipMalloc (ptab)"));
    if ((s = load_dev(join(d, "ptab.bin"), h->d_ptab, pb, pin.p)) != CS_OK) return fail(s);
  }
  if (kv["nwalk"]) {
    h->nwalk = kv["nwalk"];
    h->walk_marks = (uint32_t)kv["walk_marks"];
    if (hipMalloc(&h->d_walk, h->nwalk * 32) != hipSuccess)
      return fail(hip_fail(hipGetLastError(), "hipMalloc (walk)"));
    if ((s = load_dev(join(d, "walk.bin"), h->d_walk, h->nwalk * 32, pin.p)) != CS_OK) return fail(s);
  }
  if (kv["has_wssa"]) {
    if (hipMalloc(&h->d_wssa, (h->nisa ? h->nisa : 1) * sb) != hipSuccess)
      return fail(hip_fail(hipGetLastError(), "hipMalloc (wssa)"));
    if ((s = load_dev(join(d, "wssa.bin"), h->d_wssa, h->nisa * sb, pin.p)) != CS_OK) return fail(s);
  }
  if (hipMemcpy(h->d_table, &h->h_table, sizeof(NodeTable), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemset(h->d_err, 0xFF, 8) != hipSuccess)
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
  *out = h;
  return CS_OK;
}

}  // extern "C"
