// fm_internal.hpp — host-side handle and shared helpers of libcs_fmindex.so.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <string>
#include <mutex>
#include <utility>
#include <vector>

#include "../../include/cs_fmindex.h"
#include "../../include/cs_fmindex_tuning.h"
#include "../../include/cs_fmindex_diag.h"
#include "../../include/cs_fmindex_replica.h"
#include "fm_device.hpp"

struct cs_fm_index {
  int device = 0;
  // HBM budget of the whole index (CS_FM_HBM_BUDGET at build time; 0 = none): the optional
  // speed structures are added in build order while they fit (fm_io.hip hbm_room)
  uint64_t hbm_budget = 0;
  uint64_t n = 0;
  uint32_t stride = 32;
  void* d_lines = nullptr;            // 8 levels x nlines rank lines
  uint64_t nlines = 0;
  uint32_t line_fmt = fmx::kFmtLine32; // Line32 (n < 2^32), Line32W (wide), Line64 or Occ
  uint32_t line_bytes = 32;
  uint32_t line_bits = 224;
  uint32_t nlevels = fmx::kLevels;     // rank-line sequences (1 for occurrence lines)
  bool wide = false;                  // n >= 2^32 (or forced): u64 samples and table entries
  void* d_ssa = nullptr;
  uint64_t nsamples = 0;
  fmx::NodeTable* d_table = nullptr;
  fmx::NodeTable h_table{};
  uint64_t* d_err = nullptr;          // locate: min failing item (UINT64_MAX = none)
  void* d_ptab = nullptr;             // prefix table (DevIndex::ptab)
  void* d_sa = nullptr;               // full suffix array, u32 (lf_exact prefix-doubling builds)
  void* d_isa = nullptr;              // inverse-SA samples (extract, walk-line marks)
  uint64_t nisa = 0;
  uint32_t pstride = 32;              // walk-mark text-position stride (position_stride())
  uint32_t xstride = 32;              // the inverse-SA samples' stride (pstride; 2 pstride wide)
  uint64_t nwssa = 0;                 // walk position samples (n / pstride with position marks)
  uint32_t wssa_eb = 0;               // their bytes per entry: 4 narrow, 5 wide (40 bits); 0 = sample_bytes()
  bool lf_exact = false;              // unique smallest last symbol: LF inverts SA
  void* d_walk = nullptr;             // walk lines (occurrence engine; WalkLine / WalkLineW)
  uint64_t nwalk = 0;
  void* d_wssa = nullptr;             // position samples by mark (lf_exact), else d_ssa is used
  uint32_t walk_marks = 0;            // 0 no walk lines, 1 row marks, 2 text-position marks
  uint32_t ptab_k = 0, ptab_sigma = 0;
  void* d_lctx = nullptr;             // left contexts (DevIndex::lctx)
  uint64_t nlctx = 0;                 // entries allocated (rows rounded up + a pad sector)
  uint32_t lctx_q = 0, lctx_sb = 0;   // symbols per entry, bits per symbol
  uint32_t lctx_eb = 0;               // bytes per entry (2 occurrence lines, 4 quaternary matrix)
  void* d_lmodel = nullptr;           // learned occurrence lines: superblock models
  uint64_t nlmodel = 0;
  uint32_t lmodel_shift = 0;
  std::vector<uint8_t> h_text;        // fm_index.hpp:41 text_ (extract only)
  void* d_dtext = nullptr;            // the same text in HBM: extract as a copy (fm_index.cpp:163-167)
  // 2-bit copy of d_dtext (occurrence codes, 32 characters per u64, rare symbols as code 0)
  // and the sorted text positions of the rare symbols (<= kMaxExc): long-pattern
  // verification (fm_query.hip k_count_long); derived on build / open / import, not saved
  void* d_ptext = nullptr;
  void* d_prare = nullptr;
  uint32_t nrare = 0;
  // (round 6) the same as u64 positions for an index whose long patterns are verified at
  // their walks' positions (walk_verify()): n may pass 2^32 there
  void* d_prare64 = nullptr;
  uint32_t nrare64 = 0;
  // lf_exact occurrence lines with walk lines and text-position marks and no full SA (C5):
  // k_count_long positions a long pattern's candidate rows by their short walks and verifies
  // them against the text (the 2-bit text d_ptext, else the byte text d_dtext)
  bool walk_verify() const {
    return !d_sa && d_walk && d_wssa && walk_marks == 2 && lf_exact && line_fmt == fmx::kFmtOcc;
  }
  uint64_t ptext_bytes() const { return ((n + 31) / 32) * 8; }
  // Locate records (fmx::DevIndex::lrec): 64 B per ptab_k-mer (lrec_w 64, the default) or
  // 16 B per (ptab_k + 1)-mer (lrec_w 16), derived from the context records, the left
  // contexts and the full SA on build / open / import, not saved
  void* d_lrec = nullptr;
  uint32_t lrec_w = 0;
  uint64_t lrec_bytes() const {
    return !d_lrec ? 0 : lrec_w == 64 ? (64ull << (2 * ptab_k)) : (16ull << (2 * (ptab_k + 1)));
  }
  uint32_t active_levels[256] = {};
  // Tuning defaults (CS_QT_* bits, cs_fmindex.h) and the host-batch chunk (patterns; 0 = the
  // default), read from the environment once when the handle is created (read_tuning); every
  // query ORs its flags over `tune` (fm_query.hip call_flags) and reads no environment
  uint32_t tune = 0;
  uint64_t host_chunk = 0;
  // the routed count: a wave lists its general searches for the list kernel when it holds
  // at least this many (CS_FM_GENERAL_LIST_MIN; fm_device.hpp LongList::gen_list)
  uint32_t gen_list_min = 2;
  // the list kernels' grid (CS_FM_LIST_GRID; 0 = fm_query.hip kLongListGrid)
  uint32_t list_grid = 0;

  // Small host batches (single-pattern queries, p50 latency) stage through a
  // per-handle pinned + HBM arena instead of per-call hipMalloc/hipFree and
  // pageable copies; the lock serialises calls that share it.
  struct Scratch {
    std::mutex mu;
    uint8_t* h = nullptr;  // pinned host
    uint8_t* d = nullptr;  // HBM
  };
  static constexpr size_t kScratchBytes = 1u << 20;
  mutable Scratch scratch;

  // Resident single-pattern server (cs_fm_serve_start): one wave on a private
  // stream polls `mbox` and answers into `resp`; single-pattern counts go through it
  // while `enabled`.  The kernel exits on a stop request, after idle_us without
  // requests, or after a lifetime cap; the next request relaunches it.
  struct Server {
    std::mutex mu;
    hipStream_t st = nullptr;
    uint64_t* mbox = nullptr;  // pinned, fine-grained: kServeWords request words
    uint64_t* resp = nullptr;  // pinned, fine-grained: [0] count, [1] tag served, [2] exit mark
    uint32_t seq = 0;          // tag of the last request written
    uint32_t idle_us = 0;
    uint64_t ticks_per_us = 100;
    std::atomic<bool> enabled{false};  // read without mu on the count path
    bool launched = false;     // a kernel was launched and its exit not yet observed
  };
  mutable Server server;

  uint32_t sample_bytes() const { return wide ? 8 : 4; }
  uint32_t wssa_bytes() const { return wssa_eb ? wssa_eb : sample_bytes(); }
  uint32_t ptab_rec = 0;             // prefix-table entries: 0 plain, 1 32-B / 2 16-B context records
  uint32_t ptab_entry_bytes() const { return ptab_rec == 1 ? 32 : ptab_rec >= 2 ? 16 : 8; }  // plain: 2 x u32 / packed wide
  uint64_t ptab_entries() const {
    if (!ptab_k) return 0;
    uint64_t e = 1;
    for (uint32_t i = 0; i < ptab_k; ++i) e *= ptab_sigma;
    return e;
  }

  fmx::DevIndex dev() const {
    fmx::DevIndex d;
    d.lines = d_lines;
    d.nlines = nlines;
    d.n = n;
    d.wide = wide ? 1u : 0u;
    d.ssa = d_ssa;
    d.nsamples = nsamples;
    d.stride = stride;
    d.stride_shift = 0xFFFFFFFFu;
    if (stride && (stride & (stride - 1)) == 0) {
      uint32_t s = 0;
      while ((1u << s) != stride) ++s;
      d.stride_shift = s;
    }
    d.table = d_table;
    d.ptab = d_ptab;
    d.ptab_k = ptab_k;
    d.ptab_sigma = ptab_sigma;
    d.ptab_rec = ptab_rec;
    d.isa = d_isa;
    d.nisa = nisa;
    d.pstride = xstride;  // device code reads it only with the inverse-SA samples (extract)
    d.lf_exact = lf_exact ? 1u : 0u;
    d.walk = d_walk;
    d.wssa = d_wssa ? d_wssa : d_ssa;
    d.wssa_eb = d_wssa ? wssa_bytes() : sample_bytes();
    d.lctx = d_lctx;
    d.lctx_q = d_lctx ? lctx_q : 0u;
    d.lctx_sb = lctx_sb;
    d.lmodel = d_lmodel;
    d.lmodel_shift = lmodel_shift;
    const bool ver = d_sa && d_dtext && lf_exact && !wide;
    d.vsa = ver ? static_cast<const uint32_t*>(d_sa) : nullptr;
    d.vtext = ver ? static_cast<const uint8_t*>(d_dtext) : nullptr;
    d.wtext = walk_verify() && d_dtext ? static_cast<const uint8_t*>(d_dtext) : nullptr;
    d.ptext = (ver || walk_verify()) && d_ptext ? static_cast<const uint64_t*>(d_ptext) : nullptr;
    d.wrare = static_cast<const uint64_t*>(d_prare64);
    d.nwrare = nrare64;
    d.prare = static_cast<const uint32_t*>(d_prare);
    d.lrec = d_sa && lf_exact && !wide ? d_lrec : nullptr;
    d.lrec64 = lrec_w == 64 ? 1u : 0u;
    d.dna_std = 0;
    if ((line_fmt == fmx::kFmtOcc || line_fmt == fmx::kFmtLOcc) && ptab_sigma == 4) {
      bool std_map = true;
      for (int c = 0; c < 256 && std_map; ++c) {
        const uint8_t want = c == 'A' ? 0 : c == 'C' ? 1 : c == 'G' ? 2 : c == 'T' ? 3 : fmx::kNoCode;
        std_map = h_table.code[c] == want && h_table.occ_code[c] == want;
      }
      d.dna_std = std_map ? 1u : 0u;
    }
    d.nrare = nrare;
    return d;
  }
};

namespace fmx {

// thread-local last-error text (cs_fm_last_error)
void set_error(const std::string& msg);
cs_status hip_fail(hipError_t e, const char* what);

#define FMX_HIP(call)                                          \
  do {                                                         \
    hipError_t _e = (call);                                    \
    if (_e != hipSuccess) return ::fmx::hip_fail(_e, #call);   \
  } while (0)

// Index construction on the device (fm_build.hip).
cs_status build_sa_device(const uint8_t* d_text, uint64_t n, uint32_t* d_sa, hipStream_t st);

// Rank structures from a BWT in HBM (fm_build_rank.hip).
struct CodeMap {
  uint8_t c[256];  // 2-bit code per symbol, kNoCode for the rare ones
};
cs_status build_wm_levels(uint8_t* bwt, uint64_t n, cs_fm_index* h, hipStream_t st);
bool occ_feasible(const unsigned long long* hist, uint64_t n, CodeMap& map, uint8_t occ_sym[4]);
cs_status build_occ(const uint8_t* bwt, uint64_t n, const CodeMap& map, cs_fm_index* h,
                    hipStream_t st);
cs_status build_locc(const uint8_t* bwt, uint64_t n, const CodeMap& map, cs_fm_index* h,
                     hipStream_t st);
cs_status build_qwm(const uint8_t* bwt, uint64_t n, const unsigned long long* hist,
                    cs_fm_index* h, hipStream_t st);
cs_status build_walk(const uint8_t* bwt, uint64_t n, const CodeMap& map, cs_fm_index* h,
                     hipStream_t st);
cs_status launch_node_ranks(const cs_fm_index* h, uint64_t* d_R, hipStream_t st);
cs_status build_index_from_bwt(const uint8_t* bwt_host, uint64_t n, const uint32_t* ssa_host,
                               uint64_t nsamples, uint32_t stride, cs_fm_index* h, hipStream_t st);
cs_status build_bwt_bucketed(const uint8_t* d_text, uint64_t n, uint32_t stride, uint32_t pstride,
                             bool wide,
                             uint8_t* d_bwt, void* d_ssa, void* d_isa, hipStream_t st);
cs_status build_index_device(const uint8_t* d_text, uint64_t n, uint32_t stride, cs_fm_index* h,
                             hipStream_t st);

// A caller's device workspace (cs_fm_*_ws entry points, cs_fm_workspace_bytes): null = none
// (the call allocates what it needs, stream-ordered)
struct Work {
  void* p = nullptr;
  uint64_t bytes = 0;
};
// workspace bytes of a routed count / a one-call locate of npat patterns (fm_query.hip)
uint64_t count_workspace_bytes(const cs_fm_index* h, uint64_t npat);
uint64_t locate_workspace_bytes(const cs_fm_index* h, uint64_t npat);
// the tuning defaults of a new handle from the CS_FM_* environment (cs_fm_index::tune,
// host_chunk; fm_capi.hip): read once when a handle is created, never by a query
void read_tuning(cs_fm_index* h);

// Build options (cs_fmindex_tuning.h cs_fm_build_with_options, round 6): the CS_FM_* build and
// tuning variables as NAME=VALUE pairs.  Every builder reads its variables through build_opt():
// inside a build started with an options string that is the string's value (or none), otherwise
// the environment — the shim cs_fm_build_from_text and the older callers rely on.  The scope is
// per thread; a build runs in its caller's thread.
struct BuildOptions {
  std::vector<std::pair<std::string, std::string>> kv;
};
const char* build_opt(const char* name);
class BuildOptScope {
 public:
  explicit BuildOptScope(const BuildOptions* o);
  ~BuildOptScope();
  BuildOptScope(const BuildOptScope&) = delete;
  BuildOptScope& operator=(const BuildOptScope&) = delete;

 private:
  const BuildOptions* prev_;
};
// "ENGINE=wavelet, FULL_SA=0" -> o (names with or without CS_FM_, upper-cased); false and the
// offending token in err for a malformed pair or a name no builder reads
bool parse_build_options(const char* text, BuildOptions& o, std::string& err);

// Query launches (fm_query.hip).
// d_offs == nullptr: npat patterns of length fixed_m at stride fixed_m; flags CS_Q_*
cs_status launch_count(const cs_fm_index* h, const uint8_t* d_pats, const uint64_t* d_offs,
                       uint64_t npat, uint64_t* d_out, hipStream_t st, uint64_t fixed_m = 0,
                       uint32_t flags = 0);
// A batch whose patterns are all longer than this takes the long-pattern count kernel
// (CS_Q_LONG): fixed-length device batches and host batches, whose lengths are known
// before the launch: 32 characters and more (k_count_long reads a pattern's last 32).
constexpr uint64_t kLongPatternM = 31;
// Slack after every index part in HBM (zeroed): the text verification and extract read
// whole aligned 8-B words, up to 7 bytes past the text's last byte (fm_query.hip
// window_eq / verify_filter / k_extract_text), so the allocation covers them.
constexpr uint64_t kPartPad = 64;
// the general form: output width (fmx::CountOut), query flags (CS_Q_*), packed DNA input
// (d_pats = one uint64 per pattern of fixed_m 2-bit characters)
cs_status launch_count_ex(const cs_fm_index* h, const uint8_t* d_pats, const uint64_t* d_offs,
                          uint64_t npat, const fmx::CountOut& co, uint32_t flags, hipStream_t st,
                          uint64_t fixed_m, bool packed, const Work& work = Work{});
cs_status launch_count_one(const cs_fm_index* h, const fmx::OnePattern& p, uint64_t* out_host,
                           hipStream_t st);
cs_status launch_count_bytes(const cs_fm_index* h, const uint8_t* d_pats, const uint64_t* d_offs,
                             uint64_t npat, uint64_t* d_out, hipStream_t st, uint32_t flags = 0);
// the resident server kernel (one wave) on the handle's server stream
cs_status launch_count_server(const cs_fm_index* h, uint32_t seq_done, uint64_t idle_ticks,
                              uint64_t life_ticks);
// measurement twin of the one-call locate's locate records (cs_fm_locate_record_hits_device)
cs_status launch_locrec_hits(const cs_fm_index* h, const uint8_t* d_pats, const uint64_t* d_offs,
                             uint64_t npat, uint8_t* d_hit, hipStream_t st);
cs_status launch_locate_ranges(const cs_fm_index* h, const uint8_t* d_pats,
                               const uint64_t* d_offs, uint64_t npat, uint64_t limit,
                               uint64_t* d_sp, uint64_t* d_out_offs, uint64_t* total,
                               hipStream_t st, uint32_t flags = 0);
// err: device word receiving the smallest overrunning row index (UINT64_MAX = none);
// null = the handle's shared flag (the asynchronous API, cs_fm_locate_check)
cs_status launch_locate_onepass(const cs_fm_index* h, const uint8_t* d_pats, const uint64_t* d_offs,
                                uint64_t npat, uint64_t limit, uint64_t* d_out_offs,
                                uint64_t* d_out_pos, uint64_t cap, uint64_t* total, hipStream_t st,
                                bool* done, uint32_t flags = 0, const Work& work = Work{});
cs_status launch_locate_walk(const cs_fm_index* h, const uint64_t* d_sp,
                             const uint64_t* d_out_offs, uint64_t npat, uint64_t total,
                             uint64_t* d_out_pos, hipStream_t st,
                             unsigned long long* err = nullptr, uint32_t flags = 0,
                             uint32_t steps_only = 0);
// reads (and re-arms) the overrun word `err` (null = the handle's shared flag)
cs_status check_locate_error(const cs_fm_index* h, unsigned long long* err, hipStream_t st);
cs_status launch_level_rank1(const cs_fm_index* h, int level, const uint64_t* d_pos, uint64_t k,
                             uint64_t* d_out, hipStream_t st);
cs_status launch_wt_rank(const cs_fm_index* h, const uint8_t* d_syms, const uint64_t* d_pos,
                         uint64_t k, uint64_t* d_out, hipStream_t st);
cs_status launch_wt_access(const cs_fm_index* h, const uint64_t* d_pos, uint64_t k,
                           uint8_t* d_out, hipStream_t st);
cs_status launch_bwt(const cs_fm_index* h, uint8_t* d_out, hipStream_t st);
cs_status launch_extract(const cs_fm_index* h, const uint64_t* d_pos, const uint64_t* d_len,
                         const uint64_t* d_out_offs, uint64_t k, uint8_t* d_out, hipStream_t st);
cs_status build_prefix_table(cs_fm_index* h, hipStream_t st);
cs_status build_left_contexts(cs_fm_index* h, hipStream_t st);
cs_status build_context_records(cs_fm_index* h, hipStream_t st);
cs_status keep_device_text(cs_fm_index* h, const uint8_t* src, bool src_on_device, hipStream_t st);
// the 2-bit text of d_dtext (cs_fm_index::d_ptext), when the index can use it (fm_query.hip)
// (src: the build's device text when the index does not keep one — its 2-bit form is still
// derived for walk_verify() indexes; the buffer is the caller's input, not counted against the
// eighth of HBM the built index leaves free)
cs_status derive_packed_text(cs_fm_index* h, hipStream_t st, const uint8_t* src = nullptr);
// the locate records (cs_fm_index::d_lrec, fm_device.hpp kLocRec*) when the index can use them
cs_status derive_locate_records(cs_fm_index* h, hipStream_t st);
// both derived parts (open / import)
inline cs_status derive_parts(cs_fm_index* h, hipStream_t st) {
  cs_status s = derive_packed_text(h, st);
  return s == CS_OK ? derive_locate_records(h, st) : s;
}
// HBM held by the index's device arrays so far (the image parts, fm_io.hip)
uint64_t index_hbm_bytes(const cs_fm_index* h);
// every device allocation the handle owns (cs_fm_info.device_bytes, fm_io.hip)
uint64_t device_bytes(const cs_fm_index* h);
// Whether an optional structure of `bytes` may be allocated: the device keeps an eighth
// of its HBM free (query buffers), and with a budget the index stays within it — `freed`
// bytes of the index are released once the structure is built (a replacement).
// `transient`: device bytes in use now that are not the index's and go away after the build
// (the caller's text): counted as free for the eighth, not for the allocation itself.
bool hbm_room(const cs_fm_index* h, uint64_t bytes, uint64_t freed = 0, uint64_t transient = 0);
// CS_FM_HBM_BUDGET: bytes, with an optional K / M / G / T suffix (powers of 1000); 0 = none
uint64_t hbm_budget_env();
cs_status launch_lf(const cs_fm_index* h, const uint64_t* d_rows, uint64_t k, uint64_t* d_out,
                    hipStream_t st);

// RAII device buffer for temporaries.
struct DevBuf {
  void* p = nullptr;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { if (p) (void)hipFree(p); }
  hipError_t alloc(size_t bytes) {
    if (p) { (void)hipFree(p); p = nullptr; }
    return hipMalloc(&p, bytes ? bytes : 16);
  }
  template <class T> T* as() const { return static_cast<T*>(p); }
  void release() { if (p) (void)hipFree(p); p = nullptr; }
};

// Entry points select the index's device and restore the caller's current device on
// return, so a process driving several GPUs keeps its own device selection.
struct DeviceScope {
  int prev = -1;
  DeviceScope() = default;
  DeviceScope(const DeviceScope&) = delete;
  DeviceScope& operator=(const DeviceScope&) = delete;
  hipError_t enter(int dev) {
    int cur = 0;
    hipError_t e = hipGetDevice(&cur);
    if (e != hipSuccess) return e;
    if (cur == dev) return hipSuccess;
    e = hipSetDevice(dev);
    if (e == hipSuccess) prev = cur;
    return e;
  }
  ~DeviceScope() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

// Stream-ordered scratch for the query paths: hipMallocAsync / hipFreeAsync on the
// launch stream, so a call allocates and frees without a device synchronisation
// and the device's default pool keeps the memory cached between calls.
void keep_pool(int device);
struct StreamBuf {
  void* p = nullptr;
  hipStream_t st = nullptr;
  StreamBuf() = default;
  StreamBuf(const StreamBuf&) = delete;
  StreamBuf& operator=(const StreamBuf&) = delete;
  ~StreamBuf() { if (p) (void)hipFreeAsync(p, st); }
  hipError_t alloc(size_t bytes, hipStream_t s) {
    if (p) (void)hipFreeAsync(p, st);
    p = nullptr;
    st = s;
    int dev = 0;
    if (hipGetDevice(&dev) == hipSuccess) keep_pool(dev);
    return hipMallocAsync(&p, bytes ? bytes : 16, s);
  }
  template <class T> T* as() const { return static_cast<T*>(p); }
};

inline unsigned grid_for(uint64_t work, unsigned block, unsigned cap = 1u << 20) {
  uint64_t g = (work + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

}  // namespace fmx
