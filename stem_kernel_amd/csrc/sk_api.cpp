// C ABI of the stem-kernel engine (include/stem_kernel.h): host runtime.
//
// Owns: example sets (host build + device packing), per-GPU contexts
// (stream, scratch, work lists) and the orchestration of the HIP kernels
// that replace KernelMatrix::calculate's per-pair loop
// (common/kernel_matrix.cpp:42-56, 485-575).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <functional>
#include <memory>
#include <mutex>
#include <new>
#include <numeric>
#include <queue>
#include <sstream>
#include <thread>
#include <type_traits>
#include <atomic>
#include <string>
#include <system_error>
#include <vector>

#include "../../include/stem_kernel.h"
#include "host/fold_params.h"
#include "host/sk_internal.h"
#include "kernels/device_set.h"
#include "kernels/launch.h"
#include "ribosum85_60.inc"

using sk::DevSet;
using sk::Example;

namespace {

struct DeviceBuffers {
  std::vector<void*> ptrs;
  size_t bytes = 0;  // (SK_HOST_STATS)
  ~DeviceBuffers() { release(); }
  void release() {
    for (void* p : ptrs) (void)hipFree(p);
    ptrs.clear();
  }
};

template <class V, class T = typename V::value_type>
hipError_t upload(DeviceBuffers& db, const V& v, const T** out) {
  void* p = nullptr;
  const size_t bytes = std::max<size_t>(v.size() * sizeof(T), 16);
  hipError_t e = hipMalloc(&p, bytes);
  if (e != hipSuccess) return e;
  db.ptrs.push_back(p);
  db.bytes += bytes;
  if (!v.empty()) e = hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice);
  *out = static_cast<const T*>(p);
  return e;
}

// BPLA fill_weight (bpla_kernel/data.cpp:19-45) over the averaged bp matrix:
// float accumulators with each add rounded from double, then sqrt.
float4 bpla_weight(const Example& X, int i) {
  if (!X.has_bp) return make_float4(0.f, 0.f, 1.f, 0.f);
  float pl = 0.0f, pr = 0.0f;
  for (int j = 0; j < i; ++j) pr = (float)((double)pr + X.bpp[sk::tri_index(X.len, j, i)]);
  for (int j = i + 1; j < X.len; ++j) pl = (float)((double)pl + X.bpp[sk::tri_index(X.len, i, j)]);
  float pu = (float)(1.0 - (double)(pl + pr));
  if (pu < 0.0f) pu = 0.0f;
  return make_float4(std::sqrt(pl), std::sqrt(pr), std::sqrt(pu), 0.f);
}

// every position's bpla_weight, appended to out, in one pass over the
// triangle's rows: the same float sums in the same order (pl[i] over j > i,
// pr[i] over j < i, both by increasing j), O(L^2) with contiguous reads
void bpla_weights(const Example& X, std::vector<float4>& out) {
  const int L = X.len;
  const size_t base = out.size();
  out.resize(base + (size_t)std::max(L, 0));
  if (!X.has_bp) {
    for (int i = 0; i < L; ++i) out[base + i] = make_float4(0.f, 0.f, 1.f, 0.f);
    return;
  }
  std::vector<float> pr((size_t)L, 0.0f);
  for (int i = 0; i < L; ++i) {
    float pl = 0.0f;
    if (i + 1 < L) {
      const double* row = X.bpp.data() + sk::tri_index(L, i, i + 1);
      for (int j = i + 1; j < L; ++j) {
        const double b = row[j - i - 1];
        pl = (float)((double)pl + b);
        pr[j] = (float)((double)pr[j] + b);
      }
    }
    float pu = (float)(1.0 - (double)(pl + pr[i]));  // pr[i] is final: rows j < i came first
    if (pu < 0.0f) pu = 0.0f;
    out[base + i] = make_float4(std::sqrt(pl), std::sqrt(pr[i]), std::sqrt(pu), 0.f);
  }
}

// Packed host image of a dataset (device_set.h layout).
// vectors whose resize() leaves new elements uninitialised (trivial types):
// the packed arrays are sized once and filled on host threads, which then
// also take the page faults, instead of one thread zero-filling them first
template <class T>
struct NoInitAlloc : std::allocator<T> {
  template <class U>
  struct rebind {
    using other = NoInitAlloc<U>;
  };
  NoInitAlloc() = default;
  template <class U>
  NoInitAlloc(const NoInitAlloc<U>&) noexcept {}
  template <class U>
  void construct(U* p) noexcept {
    ::new ((void*)p) U;
  }
  template <class U, class... A>
  void construct(U* p, A&&... a) {
    ::new ((void*)p) U(std::forward<A>(a)...);
  }
};
template <class T>
using pvec = std::vector<T, NoInitAlloc<T>>;

struct HostPack {
  std::vector<int32_t> ex_nl, ex_node_base, ex_edge_base, ex_bpf_base, ex_lvl_base, ex_nlev,
      ex_len, ex_pos_base, ex_has_w;
  // every profile entry of the example a multiple of 1/256 (BPLA fast path)
  std::vector<uint8_t> ex_dyadic;
  // dyadic and no empty profile column: the string kernel's fast path;
  // every column one residue: its one-hot variant
  std::vector<uint8_t> ex_str_fast, ex_onehot;
  // y examples the register-class stem kernel cannot take (2,048 non-leaf
  // nodes or more -- each class keeps its last slot free --, or a stem edge
  // gap over 1023: its packed 11/11/10-bit records); they go to
  // sk_dag_stem_big_kernel (level-order arrays)
  std::vector<uint8_t> ex_big;
  std::vector<float> ex_nseqs;
  pvec<uint32_t> nd_a, nd_b, nd_c;
  pvec<float> nd_w, nd_nbp;
  pvec<double> nd_P;
  pvec<uint2> ed;
  pvec<uint32_t> bpf_code;
  pvec<float> bpf_p;
  pvec<int32_t> lvl;
  pvec<float4> pos_prof;
  pvec<float> pos_w;
  pvec<uint8_t> pos_chr;
  pvec<float4> pos_lru;
  std::vector<int32_t> ex_nslots, ex_xch_base;
  pvec<sk::XRow> xrow;
  pvec<uint32_t> yn_a, yn_b, yn_c, ye2, ysc;
  pvec<uint4> yrec;
  pvec<float> yn_w, yn_nbp, yn_p0;
  pvec<double> yn_P;
  pvec<int32_t> ycs;
  std::vector<int32_t> ex_ysc_base, ex_nch, ex_ycs_base;
  pvec<uint32_t> xr_node, xr_ch;
  // gamma schedule (device_set.h): the x rows without the gamma rows, the
  // gamma rows' K inputs, the dataset's gamma keys and the y gapless flags
  pvec<sk::XRow> xgrow;
  std::vector<uint32_t> gam_key;
  pvec<uint32_t> xg_node, xg_ch, xg_clg, gr_info;
  pvec<float> xg_cpf, gr_pf;
  pvec<double> gr_P;
  std::vector<int32_t> ex_xg_base, ex_nlxg, ex_xgch_base, ex_gr_base, ex_gapless;
  // phi rows (combination rows of the gamma schedule): per child record its
  // weight recipe, the rows' Gamma_{code,len} K inputs, each example's phi
  // components (phi key per type-2 record, in record order), the phi keys
  pvec<uint8_t> xg_cty;
  std::vector<uint32_t> phi_al, phi_g;
  pvec<uint32_t> gra_gidx, gra_row, phk_idx;
  std::vector<int32_t> ex_gra_base, ex_phk_base;
  pvec<uint64_t> ex_phi_bits;  // per example, the phi keys it uses (bitset)
  int32_t max_nl = 0, max_edges = 0, max_bpf = 0, max_nlev = 0, max_len = 0, max_slots = 0;
  int32_t max_nch = 0;
};
// every packed array: the y-role records (SK_YBIG and their bases) and the
// x-role / per-example arrays (SK_BIG, the ex_* vectors, the key tables) --
// sk_dataset_pack_digest and tools/pack_compare.cpp hash them in this order
#define SK_PACK_Y_ARRAYS(X) X(yn_a) X(yn_b) X(yn_c) X(ye2) X(ysc) X(yrec) X(yn_w) X(yn_nbp) X(yn_p0) X(yn_P) \
  X(ycs) X(ex_ysc_base) X(ex_nch) X(ex_ycs_base)
#define SK_PACK_X_ARRAYS(X) X(nd_a) X(nd_b) X(nd_c) X(nd_w) X(nd_nbp) X(nd_P) X(ed) X(bpf_code) X(bpf_p)     \
  X(lvl) X(xr_ch) X(xrow) X(xr_node) X(gr_info) X(gr_pf) X(gr_P) X(xg_ch) X(xg_clg) X(xg_cpf) X(xg_cty)     \
  X(phk_idx) X(gra_gidx) X(gra_row) X(xgrow) X(xg_node) X(pos_prof) X(pos_w) X(pos_chr) X(pos_lru)          \
  X(ex_phi_bits) X(ex_nl) X(ex_node_base) X(ex_edge_base) X(ex_bpf_base) X(ex_lvl_base) X(ex_nlev) X(ex_len) \
  X(ex_pos_base) X(ex_has_w) X(ex_dyadic) X(ex_str_fast) X(ex_onehot) X(ex_big) X(ex_nseqs) X(ex_nslots)    \
  X(ex_xch_base) X(gam_key) X(ex_xg_base) X(ex_nlxg) X(ex_xgch_base) X(ex_gr_base) X(ex_gapless) X(phi_al)   \
  X(phi_g) X(ex_gra_base) X(ex_phk_base)

}  // namespace

// 4-D stem kernel tables of every example of a dataset, resident on the
// device: one set per (device, bp model, loop), built on the first 4-D call
// for it and rebuilt when examples were added since (examples are
// append-only); stem4d_tables.  A call holds its sets through shared_ptrs, and
// a replaced set synchronizes its own device before its buffers are freed,
// so kernels of any context still reading it finish first.
struct Stem4dTables {
  Stem4dTables() = default;
  Stem4dTables(const Stem4dTables&) = delete;
  Stem4dTables& operator=(const Stem4dTables&) = delete;
  ~Stem4dTables() {
    if (device < 0 || buf.ptrs.empty()) return;
    int cur = -1;
    if (hipGetDevice(&cur) != hipSuccess) cur = -1;
    if (hipSetDevice(device) == hipSuccess) (void)hipDeviceSynchronize();
    buf.release();
    if (cur >= 0) (void)hipSetDevice(cur);
  }
  DeviceBuffers buf;
  int device = -1, model = -1;
  unsigned loop = 0;
  size_t n_ex = 0;
  const float* bp = nullptr;
  const uint8_t* ch = nullptr;
  std::vector<int64_t> bp_off, ch_off;
  // per example: 0 usable, 1 several rows, 2 no base pairs (bp_model 0);
  // acgu: only A/C/G/U residues (the PairHMM constraints need them)
  std::vector<uint8_t> why, acgu;
};

struct sk_dataset {
  std::vector<Example> ex;
  std::vector<std::string> labels;
  // device image (per device ordinal; one context uploads)
  int device = -1;
  bool uploaded = false;
  DevSet dev;
  DeviceBuffers buf;
  HostPack pack;
  std::string err;
  // x-role leaf-column closed forms (sk_prep_kernel) for one loop_gap: they
  // depend only on the dataset (immutable once uploaded) and loop_gap
  double* prep = nullptr;
  double prep_loop_gap = -1.0;
  // 4-D tables per (device, bp model, loop), at most kS4Sets (oldest dropped)
  std::mutex s4_mu;
  std::vector<std::shared_ptr<Stem4dTables>> s4;
};
constexpr size_t kS4Sets = 4;

struct Stem4dBatch {
  sk::Stem4dPair* pairs = nullptr;
  int2* items = nullptr;
  int32_t* band = nullptr;  // c_low | c_high (cap_band each)
  size_t cap_pairs = 0, cap_items = 0, cap_band = 0;
};

struct sk_context {
  Stem4dBatch s4d;
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  int n_cu = 0;
  std::string err;
  // reusable device buffers
  double* scratch = nullptr;
  size_t scratch_bytes = 0;
  void* work = nullptr;
  size_t work_bytes = 0;
  hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr, ev3 = nullptr;
  // side stream: the string kernel of a stem+string kind runs beside the
  // persistent stem launches and fills the CUs their tails free
  hipStream_t side = nullptr;
  hipEvent_t evf = nullptr, evj = nullptr;
  // second class stream: DAG stem register classes alternate between the
  // main stream and this one, so a class's fill overlaps the previous one's
  // tail
  hipStream_t cls = nullptr;
  hipEvent_t evk = nullptr, evx = nullptr;
  // a fourth stream: the 4-D kernel's span launches run in parts on all four
  hipStream_t aux = nullptr;
  hipEvent_t eva = nullptr;
  // Timing of a compute call: its span events (ev0..ev3 are the current
  // set's) and per-launch events of the dominant kernel (sk_last_launch_ms: a
  // start and an end event around each launch on the launch's own stream).
  // Synchronous calls use set 0 and are resolved before they return; with
  // sk_set_async the sets rotate through a ring and a call returns once its
  // work is enqueued: its set stays pending until sk_sync_timing, or until
  // the ring comes round to it, and is then added to the acc_* totals.
  struct TSet {
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    std::vector<hipEvent_t> lev;
    size_t lev_used = 0;
    bool pending = false, stem = false, str = false;
    double cells = 0.0;
    int32_t launches = 0;
  };
  static constexpr int kTSets = 4;
  TSet tset[kTSets];
  int tk = 0;
  bool async = false;
  double acc_stem_ms = 0.0, acc_str_ms = 0.0, acc_cells = 0.0, acc_launch_ms = 0.0;
  int32_t acc_launch_n = 0, acc_launches = 0;
  // pinned staging of an asynchronous call's host-to-device uploads (the
  // host buffers die when the call returns; pageable copies would wait for
  // the stream): one ring slot per call parity, reused once its copies are
  // done (its event)
  struct Stage {
    std::vector<std::pair<char*, size_t>> blocks;
    size_t blk = 0, off = 0;
    hipEvent_t ev = nullptr;
    bool recorded = false;
    // device copy of a call's inputs uploaded on the copy stream (up_reserve)
    char* dbuf = nullptr;
    size_t dcap = 0;
    hipEvent_t uev = nullptr;
  };
  Stage stage[2];
  hipStream_t cps = nullptr;  // copy stream of the asynchronous uploads
  uint64_t ncalls = 0;
  double last_launch_ms_sum = 0.0;
  int32_t last_launch_n = 0;
  double last_stem_ms = 0.0, last_str_ms = 0.0, last_cells = 0.0;
  int32_t last_launches = 0;
  // kernel instantiations the last compute call launched (sk_last_classes):
  // bit MAXK/4 per DAG stem register class; bit log2(CPL) (+4 when banded)
  // per 4-D stem class
  uint32_t last_stem_classes = 0, last_s4d_classes = 0;
  // RCCL communicator of sk_comm_init (ncclComm_t, csrc/host/shard.cpp)
  void* comm = nullptr;
};

// Host thread pools: f(t) for t = 1..n-1 on new threads, f(0) on the calling
// thread; a slice whose thread cannot be created (std::system_error) runs on
// the calling thread too, so a pool never escapes through the C ABI.  The
// no-index form is for workers that share an atomic cursor.
template <class F>
void run_slices(int n, F&& f) {
  std::vector<std::thread> th;
  std::vector<int> here;
  for (int t = 1; t < n; ++t) {
    try {
      th.emplace_back(f, t);
    } catch (const std::system_error&) {
      here.push_back(t);
    }
  }
  f(0);
  for (int t : here) f(t);
  for (auto& x : th) x.join();
}
// host threads of a call's planning passes (the box gives a job 16)
int plan_threads(int want) {
  return std::max(1, std::min({want, 16, (int)std::max(1u, std::thread::hardware_concurrency())}));
}
template <class F>
void run_pool(int n, F&& work) {
  std::vector<std::thread> th;
  for (int t = 1; t < n; ++t) {
    try {
      th.emplace_back(work);
    } catch (const std::system_error&) {
      break;  // the calling thread's share drains the cursor
    }
  }
  work();
  for (auto& x : th) x.join();
}

namespace sk {
hipStream_t ctx_stream(sk_context* ctx) { return ctx->stream; }

// start or end event of one dominant-kernel launch, on the launch's stream
hipError_t lev_mark(sk_context* ctx, hipStream_t s) {
  sk_context::TSet& T = ctx->tset[ctx->tk];
  if (T.lev_used == T.lev.size()) {
    hipEvent_t e = nullptr;
    const hipError_t r = hipEventCreate(&e);
    if (r != hipSuccess) return r;
    T.lev.push_back(e);
  }
  return hipEventRecord(T.lev[T.lev_used++], s);
}

// after the launch streams are synchronized: adds the marked launches'
// durations to the call's sum
hipError_t lev_collect(sk_context* ctx) {
  sk_context::TSet& T = ctx->tset[ctx->tk];
  for (size_t i = 0; i + 1 < T.lev_used; i += 2) {
    float ms = 0.f;
    const hipError_t r = hipEventElapsedTime(&ms, T.lev[i], T.lev[i + 1]);
    if (r != hipSuccess) return r;
    ctx->last_launch_ms_sum += ms;
    ++ctx->last_launch_n;
  }
  T.lev_used = 0;
  return hipSuccess;
}

// A pending asynchronous call's timing, into the acc_* totals (waits for it).
hipError_t tset_resolve(sk_context* ctx, int k) {
  sk_context::TSet& T = ctx->tset[k];
  if (!T.pending) return hipSuccess;
  T.pending = false;
  float ms = 0.f;
  hipError_t r;
  if (T.stem) {
    if ((r = hipEventSynchronize(T.ev[1])) != hipSuccess) return r;
    if ((r = hipEventElapsedTime(&ms, T.ev[0], T.ev[1])) != hipSuccess) return r;
    ctx->acc_stem_ms += ms;
  }
  if (T.str) {
    if ((r = hipEventSynchronize(T.ev[3])) != hipSuccess) return r;
    if ((r = hipEventElapsedTime(&ms, T.ev[2], T.ev[3])) != hipSuccess) return r;
    ctx->acc_str_ms += ms;
  }
  for (size_t i = 0; i + 1 < T.lev_used; i += 2) {
    if ((r = hipEventSynchronize(T.lev[i + 1])) != hipSuccess) return r;
    if ((r = hipEventElapsedTime(&ms, T.lev[i], T.lev[i + 1])) != hipSuccess) return r;
    ctx->acc_launch_ms += ms;
    ++ctx->acc_launch_n;
  }
  T.lev_used = 0;
  ctx->acc_cells += T.cells;
  ctx->acc_launches += T.launches;
  return hipSuccess;
}

// Start of a compute call: its timing set (and, async, its staging slot).
hipError_t call_begin(sk_context* ctx) {
  hipError_t r;
  if (ctx->async) {
    const int k = (ctx->tk + 1) % sk_context::kTSets;
    if ((r = tset_resolve(ctx, k)) != hipSuccess) return r;  // the ring came round
    ctx->tk = k;
    sk_context::Stage& G = ctx->stage[ctx->ncalls++ & 1];
    if (G.recorded) {
      if ((r = hipEventSynchronize(G.ev)) != hipSuccess) return r;
    } else if (G.blk || G.off) {
      // the slot's call staged copies but failed before call_finish recorded
      // its event: the copy engine may still read the pinned bytes
      if ((r = hipStreamSynchronize(ctx->stream)) != hipSuccess) return r;
      if (ctx->cps && (r = hipStreamSynchronize(ctx->cps)) != hipSuccess) return r;
    }
    G.recorded = false;
    G.blk = G.off = 0;
  } else {
    ctx->tk = 0;
  }
  sk_context::TSet& T = ctx->tset[ctx->tk];
  for (int i = 0; i < 4; ++i)
    if (!T.ev[i] && (r = hipEventCreate(&T.ev[i])) != hipSuccess) return r;
  T.lev_used = 0;
  T.pending = false;
  ctx->ev0 = T.ev[0];
  ctx->ev1 = T.ev[1];
  ctx->ev2 = T.ev[2];
  ctx->ev3 = T.ev[3];
  return hipSuccess;
}

// Host-to-device upload of a compute call: straight from the caller's memory
// (synchronous calls), or through the call's pinned staging slot (async).
hipError_t h2d(sk_context* ctx, void* dst, const void* src, size_t bytes, hipStream_t s) {
  if (bytes == 0) return hipSuccess;
  if (!ctx->async) return hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s);
  sk_context::Stage& G = ctx->stage[(ctx->ncalls - 1) & 1];
  const size_t need = (bytes + 255) & ~(size_t)255;
  while (G.blk < G.blocks.size() && G.off + need > G.blocks[G.blk].second) {
    ++G.blk;
    G.off = 0;
  }
  if (G.blk == G.blocks.size()) {
    const size_t cap = std::max(need, (size_t)8 << 20);
    void* p = nullptr;
    const hipError_t r = hipHostMalloc(&p, cap, hipHostMallocDefault);
    if (r != hipSuccess) return r;
    G.blocks.push_back({static_cast<char*>(p), cap});
    G.off = 0;
  }
  char* p = G.blocks[G.blk].first + G.off;
  G.off += need;
  std::memcpy(p, src, bytes);
  return hipMemcpyAsync(dst, p, bytes, hipMemcpyHostToDevice, s);
}

// Asynchronous calls (BPLA): the call's host inputs go to a device buffer of
// the call's parity on a copy stream that the call's stream then waits for,
// so the upload overlaps the previous call's kernels instead of following
// them.  The buffer's last user is the call two back, which call_begin has
// waited for.
hipError_t up_reserve(sk_context* ctx, size_t bytes, char** dst) {
  sk_context::Stage& G = ctx->stage[(ctx->ncalls - 1) & 1];
  hipError_t r;
  if (G.dcap < bytes) {
    if (G.dbuf && (r = hipFree(G.dbuf)) != hipSuccess) return r;
    G.dbuf = nullptr;
    G.dcap = 0;
    const size_t cap = bytes + bytes / 4 + 4096;
    void* p = nullptr;
    if ((r = hipMalloc(&p, cap)) != hipSuccess) return r;
    G.dbuf = static_cast<char*>(p);
    G.dcap = cap;
  }
  *dst = G.dbuf;
  return hipSuccess;
}

hipError_t up_copy(sk_context* ctx, const void* src, size_t bytes, hipStream_t s) {
  sk_context::Stage& G = ctx->stage[(ctx->ncalls - 1) & 1];
  hipError_t r;
  if (!ctx->cps && (r = hipStreamCreateWithFlags(&ctx->cps, hipStreamNonBlocking)) != hipSuccess) return r;
  if (!G.uev && (r = hipEventCreateWithFlags(&G.uev, hipEventDisableTiming)) != hipSuccess) return r;
  if ((r = h2d(ctx, G.dbuf, src, bytes, ctx->cps)) != hipSuccess) return r;  // (pinned staging)
  if ((r = hipEventRecord(G.uev, ctx->cps)) != hipSuccess) return r;
  return hipStreamWaitEvent(s, G.uev, 0);
}

// End of a compute call whose span events (ev0/ev1: stem, ev2/ev3: string)
// and launch events were recorded on streams joined into `s`: synchronous,
// its timing becomes last_*; async, it stays pending.
hipError_t call_finish(sk_context* ctx, hipStream_t s, bool stem, bool str) {
  sk_context::TSet& T = ctx->tset[ctx->tk];
  T.stem = stem;
  T.str = str;
  T.cells = ctx->last_cells;
  T.launches = ctx->last_launches;
  hipError_t r;
  if (ctx->async) {
    sk_context::Stage& G = ctx->stage[(ctx->ncalls - 1) & 1];
    if ((r = hipEventRecord(G.ev, s)) != hipSuccess) return r;
    G.recorded = true;
    T.pending = true;
    return hipSuccess;
  }
  if ((r = hipStreamSynchronize(s)) != hipSuccess) return r;
  float ms = 0.f;
  if (stem) {
    if ((r = hipEventElapsedTime(&ms, T.ev[0], T.ev[1])) != hipSuccess) return r;
    ctx->last_stem_ms = ms;
  }
  if (str) {
    if ((r = hipEventElapsedTime(&ms, T.ev[2], T.ev[3])) != hipSuccess) return r;
    ctx->last_str_ms = ms;
  }
  return lev_collect(ctx);
}

void lev_reset(sk_context* ctx) {  // (the call's launch events: call_begin)
  ctx->last_launch_ms_sum = 0.0;
  ctx->last_launch_n = 0;
}
int ctx_device(sk_context* ctx) { return ctx->device; }
void*& ctx_comm(sk_context* ctx) { return ctx->comm; }
void comm_destroy(void* comm);
}  // namespace sk

namespace {

int fail(sk_context* ctx, int code, const std::string& msg) {
  if (ctx) ctx->err = msg;
  return code;
}


// Lane placement of one IY sweep chunk (records child:11 | parent:11 |
// gaps:10, sorted ids).  The kernel reads R[child] (ds_read_b64: banks by
// element mod 32 within each 32-lane half) and adds into R[parent]
// (ds_add_f64: taken as 16-lane groups, element mod 16), so the edges are
// dealt to the four 16-lane groups greedily to spread both, the parents with
// most edges in the chunk first; dummies (child == parent, weight 0) take
// the emptiest slots.
static void assign_sweep_lanes(const std::vector<int>& take, const std::vector<uint32_t>& er, int nl,
                               uint32_t lanes[64]) {
  const int n = (int)take.size();  // <= 64: fixed arrays, no allocation per chunk
  // edges per parent in the chunk (a per-thread count table over the 11-bit
  // parent ids, cleared again after use)
  thread_local uint8_t npar[2048];
  int cntp[64];
  for (int i = 0; i < n; ++i) ++npar[(er[take[i]] >> 11) & 0x7ff];
  for (int i = 0; i < n; ++i) cntp[i] = npar[(er[take[i]] >> 11) & 0x7ff];
  for (int i = 0; i < n; ++i) npar[(er[take[i]] >> 11) & 0x7ff] = 0;
  // edges by that count, largest first, chunk order among equals (a
  // counting sort: stable)
  int ord[64];
  {
    int cstart[66] = {0};
    for (int i = 0; i < n; ++i) ++cstart[64 - cntp[i] + 1];
    for (int k = 0; k < 65; ++k) cstart[k + 1] += cstart[k];
    for (int i = 0; i < n; ++i) ord[cstart[64 - cntp[i]]++] = i;
  }
  int fill[4] = {0, 0, 0, 0};
  int at[4][16];         // group -> parent slot load
  uint32_t rd[2][32][4];  // half -> child slot -> distinct children (up to 4 kept)
  int rdn[2][32];
  std::memset(at, 0, sizeof(at));
  std::memset(rdn, 0, sizeof(rdn));
  auto child_load = [&](int h, uint32_t c) {
    const int sl = c & 31;
    for (int t = 0; t < std::min(rdn[h][sl], 4); ++t)
      if (rd[h][sl][t] == c) return rdn[h][sl];
    return rdn[h][sl] + 1;
  };
  auto put = [&](int g, uint32_t r) {
    const uint32_t c = r & 0x7ff, q = (r >> 11) & 0x7ff;
    const int h = g >> 1, sl = c & 31;
    bool seen = false;
    for (int t = 0; t < std::min(rdn[h][sl], 4); ++t) seen |= rd[h][sl][t] == c;
    if (!seen) {
      if (rdn[h][sl] < 4) rd[h][sl][rdn[h][sl]] = c;
      ++rdn[h][sl];
    }
    at[g][q & 15]++;
    lanes[16 * g + fill[g]++] = r;
  };
  for (int oi = 0; oi < n; ++oi) {
    const int i = ord[oi];
    const uint32_t r = er[take[i]];
    const uint32_t c = r & 0x7ff, q = (r >> 11) & 0x7ff;
    int best = -1, bc = 1 << 30;
    for (int g = 0; g < 4; ++g) {
      if (fill[g] == 16) continue;
      const int cost = 4 * (child_load(g >> 1, c) + at[g][q & 15] + 1) + fill[g];
      if (cost < bc) {
        bc = cost;
        best = g;
      }
    }
    put(best, r);
  }
  const int nl1 = std::max(nl, 1);
  for (int g = 0; g < 4; ++g) {
    while (fill[g] < 16) {
      int bs = 0, bc = 1 << 30;
      for (int sl = 0; sl < 32 && sl < nl1; ++sl) {
        const int cost = rdn[g >> 1][sl] + at[g][sl & 15];
        if (cost < bc) {
          bc = cost;
          bs = sl;
        }
      }
      const uint32_t d = (uint32_t)(bs % nl1);
      put(g, d | (d << 11));
    }
  }
}

#define SK_HIP(ctx, expr)                                                              \
  do {                                                                                 \
    hipError_t _e = (expr);                                                            \
    if (_e != hipSuccess)                                                              \
      return fail((ctx), SK_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

// --------------------------------------------------------------- packing
int pack_dataset(sk_dataset* ds, std::string& err, const std::function<void()>* after_x = nullptr) {
  HostPack& P = ds->pack;
  const bool tstats = std::getenv("SK_HOST_STATS") != nullptr;
  auto tnow = [] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
  const double tp0 = tnow();
  // SK_SWEEP_LANES=0: sweep chunks in schedule order (A/B diagnostics)
  const char* lanes_env = SK_KNOB("SK_SWEEP_LANES");
  const bool sweep_lanes_greedy = !lanes_env || std::atoi(lanes_env) != 0;
  P = HostPack();
  const int n = (int)ds->ex.size();
  // Gamma rows: x loop rows (one leaf child) with one bp-frequency entry and
  // no gap column.  Their G0 row is (g^gaps pf) x Gamma_{code,len}(y), the
  // IY sweep of a y-only vector (dag_stem.hip), so the gamma schedule skips
  // them; the dataset's (code, len) keys index the per-y Gamma rows.
  auto is_gamma = [&](const Example& X, int v) {
    const uint32_t e0 = X.edge_off[v], e1 = X.edge_off[v + 1];
    if (e1 - e0 != 1) return false;
    const uint32_t c = X.edge_to[e0];
    if (X.edge_off[c + 1] != X.edge_off[c]) return false;  // the child is not a leaf: a stem
    return X.bpf_off[v + 1] - X.bpf_off[v] == 1 && X.prof5[(size_t)X.first[v] * 5 + 4] == 0.0f;
  };
  auto gamma_key = [&](const Example& X, int v) {
    return ((uint32_t)X.bpf_code[X.bpf_off[v]] << 16) | (uint32_t)(X.last[v] - X.first[v]);
  };
  // Phi rows: stem rows with one bp-frequency entry and no gap column whose
  // children are all gamma rows.  Their G0 row is linear in per-y tables
  // (dag_stem.hip): pf [sum_c w_c Phi_{code,len,key(c)} + xSL Gamma_{code,len}]
  // + xwg sum_c w_c Gamma_{key(c)}, so the gamma schedule holds them as
  // combination rows (no MATCH, no sweep).
  auto is_phi = [&](const Example& X, int v) {
    const uint32_t e0 = X.edge_off[v], e1 = X.edge_off[v + 1];
    if (e1 == e0 || 2 * (e1 - e0) + 1 > 255) return false;
    if (X.bpf_off[v + 1] - X.bpf_off[v] != 1 || X.prof5[(size_t)X.first[v] * 5 + 4] != 0.0f) return false;
    for (uint32_t k = e0; k < e1; ++k)
      if (!is_gamma(X, X.edge_to[k])) return false;
    return !is_gamma(X, v);
  };
  std::vector<uint64_t> phi_raw;  // child gamma key:32 | code:16 | len:16 (sorted: by child key)
  // host threads of the packing passes (SK_PACK_THREADS caps them: the
  // packed arrays do not depend on it, tests/test_pack_threads.py)
  const size_t pcap = std::getenv("SK_PACK_THREADS") ? (size_t)std::max(1, std::atoi(std::getenv("SK_PACK_THREADS")))
                                                     : (size_t)16;
  const int nthr = (int)std::max<size_t>(1, std::min<size_t>({(size_t)n / 8 + 1, pcap,
                                                              (size_t)std::max(1u, std::thread::hardware_concurrency())}));
  {  // every example's keys (host threads, one slice each), then one sorted set
    std::vector<std::vector<uint32_t>> tk(nthr);
    std::vector<std::vector<uint64_t>> tp(nthr);
    auto keys = [&](int t) {
      for (int e = (int)((int64_t)n * t / nthr); e < (int)((int64_t)n * (t + 1) / nthr); ++e) {
        const Example& X = ds->ex[e];
        for (int v = 0; v < X.n_nodes(); ++v) {
          if (is_gamma(X, v)) tk[t].push_back(gamma_key(X, v));
          if (is_phi(X, v)) {
            tk[t].push_back(gamma_key(X, v));
            for (uint32_t k = X.edge_off[v]; k < X.edge_off[v + 1]; ++k)
              tp[t].push_back(((uint64_t)gamma_key(X, X.edge_to[k]) << 32) | gamma_key(X, v));
          }
        }
        auto& k1 = tk[t];  // keep each slice's lists short
        if (k1.size() > 4096) {
          std::sort(k1.begin(), k1.end());
          k1.erase(std::unique(k1.begin(), k1.end()), k1.end());
        }
        auto& p1 = tp[t];
        if (p1.size() > 4096) {
          std::sort(p1.begin(), p1.end());
          p1.erase(std::unique(p1.begin(), p1.end()), p1.end());
        }
      }
    };
    run_slices(nthr, keys);
    for (int t = 0; t < nthr; ++t) {
      P.gam_key.insert(P.gam_key.end(), tk[t].begin(), tk[t].end());
      phi_raw.insert(phi_raw.end(), tp[t].begin(), tp[t].end());
    }
  }
  std::sort(P.gam_key.begin(), P.gam_key.end());
  P.gam_key.erase(std::unique(P.gam_key.begin(), P.gam_key.end()), P.gam_key.end());
  const bool gam_on = !P.gam_key.empty() && P.gam_key.size() <= 512 && !SK_KNOB("SK_NO_GAMMA");
  if (!gam_on) P.gam_key.clear();
  auto gamma_idx = [&](uint32_t key) {
    return (uint32_t)(std::lower_bound(P.gam_key.begin(), P.gam_key.end(), key) - P.gam_key.begin());
  };
  std::sort(phi_raw.begin(), phi_raw.end());
  phi_raw.erase(std::unique(phi_raw.begin(), phi_raw.end()), phi_raw.end());
  const bool phi_on = gam_on && !phi_raw.empty() && phi_raw.size() < 0x4000 && !SK_KNOB("SK_NO_PHI");
  if (phi_on)
    for (uint64_t k : phi_raw) {
      P.phi_al.push_back((uint32_t)k);
      P.phi_g.push_back(gamma_idx((uint32_t)(k >> 32)));
    }
  auto phi_idx = [&](uint32_t key_p, uint32_t key_c) {
    const uint64_t k = ((uint64_t)key_c << 32) | key_p;
    return (uint32_t)(std::lower_bound(phi_raw.begin(), phi_raw.end(), k) - phi_raw.begin());
  };
  // y-role records of one example (its nodes sorted by length, the IY sweep
  // schedule, node-major edges), formed from its x-role arrays once the loop
  // below has packed them: independent per example, so they run on host
  // threads and are appended in example order (bit-identical to a serial pass)
  struct YJob {
    int nb0, ebase, bbase, nl;
    bool big;
  };
  struct YOut {
    std::vector<uint32_t> ysc, ye2, yn_a, yn_b, yn_c;
    std::vector<int32_t> ycs;
    std::vector<uint4> yrec;
    std::vector<float> yn_w, yn_nbp, yn_p0;
    std::vector<double> yn_P;
    int nch = 0;
    std::string err;
  };
  std::vector<YJob> yjobs;
  yjobs.reserve(n);
  auto pack_y = [&](const YJob& J, YOut& Y) {
    const int nl = J.nl, ebase = J.ebase, bbase = J.bbase;
    const bool big = J.big;
    // y-role numbering for the stem kernel: nodes sorted by length (span
    // last - first), so the nodes inside a row's length band are one index
    // range and a node's children (strictly shorter) come before it; edges
    // grouped by parent level (the IY sweep walks levels) and contiguous per
    // parent, packed child:11 | parent:11 | gaps:10 in sorted ids.
    {
      std::vector<int> srt(nl);
      std::iota(srt.begin(), srt.end(), 0);
      auto len_of = [&](int k) { return P.nd_b[J.nb0 + k] & 0xffff; };
      std::stable_sort(srt.begin(), srt.end(), [&](int a, int b) { return len_of(a) < len_of(b); });
      std::vector<int> pos(nl);
      for (int i = 0; i < nl; ++i) pos[srt[i]] = i;
      const int nb0 = J.nb0;
      // IY sweep schedule.  The sweep is a stream of chunks of 64 edges: a
      // chunk's R[child] reads are issued after the previous chunk's
      // atomics, so an edge may go into any chunk after the one holding the
      // last edge of its child (every node's value is final by then).  List
      // scheduling, priority = height of the parent (longest path up to a
      // root; the critical chain first), then the child's length; chunks
      // are padded with dummy records (child == parent: weight 0).
      if (big) {  // no sweep schedule: the big-y kernel walks the levels
        const int lmax = nl ? (int)(P.nd_b[nb0 + srt[nl - 1]] & 0xffff) : 0;
        for (int v = 0; v <= lmax + 1; ++v) Y.ycs.push_back(0);
        Y.nch = 0;
      } else {
        std::vector<uint32_t> er;       // records child:11 | parent:11 | gaps:10
        std::vector<int> epar, ech;
        for (int k = 0; k < nl; ++k) {
          const uint32_t a = P.nd_a[nb0 + k];
          const uint32_t ne = (a >> 16) & 0xff, el = a & 0xffff;
          for (uint32_t t = 0; t < ne; ++t) {
            const uint2 rec = P.ed[ebase + el + t];  // {child | gaps<<16, parent}
            const int c = pos[rec.x & 0xffff], q = pos[k];
            epar.push_back(q);
            ech.push_back(c);
            er.push_back((uint32_t)c | ((uint32_t)q << 11) | ((rec.x >> 16) << 22));
          }
        }
        const int ne_all = (int)er.size();
        // a child's edges in edge order (CSR: one allocation, not one per node)
        std::vector<int> cb(nl + 1, 0), by_child(ne_all);
        for (int f = 0; f < ne_all; ++f) cb[ech[f] + 1]++;
        for (int i = 0; i < nl; ++i) cb[i + 1] += cb[i];
        {
          std::vector<int> fillc(cb.begin(), cb.end() - 1);
          for (int f = 0; f < ne_all; ++f) by_child[fillc[ech[f]]++] = f;
        }
        // sorted ids: a parent is strictly longer, so it has a larger id
        std::vector<int> h(nl, 0), rem(nl, 0);
        for (int i = nl - 1; i >= 0; --i)
          for (int t = cb[i]; t < cb[i + 1]; ++t) h[i] = std::max(h[i], h[epar[by_child[t]]] + 1);
        for (int f = 0; f < ne_all; ++f) rem[epar[f]]++;
        // key (-height, child len, edge) packed into one integer, smallest
        // first: 2^20 - 1 - height:20 | len:16 | edge:28 (nl < 2^16, edges < 2^28)
        std::priority_queue<uint64_t, std::vector<uint64_t>, std::greater<uint64_t>> ready;
        auto push_edges_of = [&](int c) {
          const uint64_t len = P.nd_b[nb0 + srt[c]] & 0xffff;
          for (int t = cb[c]; t < cb[c + 1]; ++t) {
            const int f = by_child[t];
            ready.push(((uint64_t)((1 << 20) - 1 - h[epar[f]]) << 44) | (len << 28) | (uint64_t)f);
          }
        };
        for (int c = 0; c < nl; ++c)
          if (rem[c] == 0) push_edges_of(c);
        std::vector<int32_t> cm;  // prefix maximum of the children's lengths
        int32_t run = -1, placed = 0;
        // done: parents completed by the chunk just formed; their edges are
        // ready from the next chunk on
        std::vector<int> take, done;
        while (!ready.empty()) {
          take.clear();
          done.clear();
          while (!ready.empty() && (int)take.size() < 64) {
            take.push_back((int)(ready.top() & 0xfffffffu));
            ready.pop();
          }
          for (int f : take) {
            run = std::max<int32_t>(run, (int32_t)(P.nd_b[nb0 + srt[ech[f]]] & 0xffff));
            if (--rem[epar[f]] == 0) done.push_back(epar[f]);
          }
          if (sweep_lanes_greedy) {
            uint32_t lanes[64];
            assign_sweep_lanes(take, er, nl, lanes);
            Y.ysc.insert(Y.ysc.end(), lanes, lanes + 64);
          } else {
            for (int f : take) Y.ysc.push_back(er[f]);
            for (int j = (int)take.size(); j < 64; ++j) {
              const uint32_t d = (uint32_t)(j % std::max(nl, 1));
              Y.ysc.push_back(d | (d << 11));
            }
          }
          placed += (int)take.size();
          cm.push_back(run);
          for (int q : done) push_edges_of(q);  // ready from the next chunk on
        }
        if (placed != ne_all) {
          Y.err = "IY sweep schedule: DAG has a cycle";
          return;
        }
        const int nch = (int)cm.size();
        // first chunk whose prefix maximum reaches v, v = 0 .. lmax+1
        const int lmax = nl ? (int)(P.nd_b[nb0 + srt[nl - 1]] & 0xffff) : 0;
        for (int v = 0, c = 0; v <= lmax + 1; ++v) {
          while (c < nch && cm[c] < v) ++c;
          Y.ycs.push_back(c);
        }
        Y.nch = nch;
      }
      // node-major copy of the edges in sorted order (the MATCH sums of a
      // run of consecutive nodes read one contiguous edge range); a node's
      // record keeps its first edge there, E(q) = prefix sum of n_edges
      const int ye2_base = (int)Y.ye2.size();
      for (int i = 0; i < nl; ++i) {
        const int k = srt[i];
        const uint32_t a = P.nd_a[nb0 + k];
        const uint32_t ne = (a >> 16) & 0xff, el = a & 0xffff;
        const uint32_t nbf = a >> 24, bl = P.nd_b[nb0 + k] >> 16;
        Y.yn_a.push_back(((uint32_t)Y.ye2.size() - ye2_base) | (a & 0xffff0000u));
        for (uint32_t t = 0; t < ne; ++t) {
          const uint2 rec = P.ed[ebase + el + t];
          Y.ye2.push_back(big ? 0u : (uint32_t)pos[rec.x & 0xffff] | ((uint32_t)i << 11) |
                                         ((rec.x >> 16) << 22));
        }
        // c = loop leaf-edge gaps:16 | first bp-freq code:4 | single-entry flag
        // (one bp-freq entry, no gap column: the closed-form node score)
        const bool one = nbf == 1 && P.nd_nbp[nb0 + k] == 0.0f;
        const uint32_t bc0 = nbf ? P.bpf_code[bbase + bl] & 0xf : 0u;
        Y.yn_c.push_back((P.nd_c[nb0 + k] & 0xffff) | (bc0 << 16) | ((one ? 1u : 0u) << 24));
        Y.yn_p0.push_back(nbf ? P.bpf_p[bbase + bl] : 0.0f);
        {
          uint4 r;
          r.x = Y.yn_a.back();
          r.y = Y.yn_c.back();
          std::memcpy(&r.z, &P.nd_w[nb0 + k], 4);
          std::memcpy(&r.w, &Y.yn_p0.back(), 4);
          Y.yrec.push_back(r);
        }
        Y.yn_b.push_back(P.nd_b[nb0 + k]);
        Y.yn_w.push_back(P.nd_w[nb0 + k]);
        Y.yn_nbp.push_back(P.nd_nbp[nb0 + k]);
        Y.yn_P.push_back(P.nd_P[nb0 + k]);
      }
    }

  };
  // x-role records of one example (nodes in level order, the x schedules,
  // per-position tables), formed per example on host threads and appended
  // in example order below (bit-identical to one serial pass; example-local
  // offsets, the dataset's bases added when appending)
  struct XOut {
    std::vector<uint32_t> nd_a, nd_b, nd_c, xr_ch, xr_node, gr_info, xg_ch, xg_clg, phk_idx, gra_gidx,
        gra_row, xg_node;
    std::vector<float> nd_w, nd_nbp, bpf_p, gr_pf, xg_cpf, ex_nseqs, pos_w;
    std::vector<double> nd_P, gr_P;
    std::vector<uint2> ed;
    std::vector<uint32_t> bpf_code;
    std::vector<int32_t> lvl, ex_nslots, ex_nlxg, ex_gapless, ex_nl, ex_nlev, ex_len, ex_has_w;
    std::vector<uint8_t> ex_big, xg_cty, pos_chr, ex_dyadic, ex_str_fast, ex_onehot;
    std::vector<sk::XRow> xrow, xgrow;
    std::vector<float4> pos_prof, pos_lru;
    std::vector<uint64_t> ex_phi_bits;
    int nl = 0, nlev = 0, max_slots = 0, n_nostore = 0, n_nodes = 0, gslots = 0;
    bool big = false;
    int rc = SK_OK;
    std::string err;
  };
  auto pack_x = [&](int e, XOut& O) {
    const Example& X = ds->ex[e];
    const int nn = X.n_nodes();
    // level of every node (children first in reference numbering)
    std::vector<int> level(nn, -1);
    int nlev = 0;
    for (int v = 0; v < nn; ++v) {
      const uint32_t e0 = X.edge_off[v], e1 = X.edge_off[v + 1];
      if (e0 == e1) continue;  // leaf
      int lv = 0;
      bool any_leaf = false;
      for (uint32_t k = e0; k < e1; ++k) {
        const int c = level[X.edge_to[k]];
        if (c < 0) any_leaf = true;
        else lv = std::max(lv, c + 1);
      }
      if (any_leaf && e1 - e0 != 1) {
        O.err = "unexpected DAG shape: stem with a leaf child";
        O.rc = SK_ERR_INVALID;
        return;
      }
      level[v] = lv;
      nlev = std::max(nlev, lv + 1);
    }
    std::vector<int> order;  // non-leaf nodes by (level, reference index): a counting sort
    {
      std::vector<int> lstart(nlev + 1, 0);
      for (int v = 0; v < nn; ++v)
        if (level[v] >= 0) ++lstart[level[v] + 1];
      for (int l = 0; l < nlev; ++l) lstart[l + 1] += lstart[l];
      order.resize(lstart[nlev]);
      for (int v = 0; v < nn; ++v)
        if (level[v] >= 0) order[lstart[level[v]]++] = v;
    }
    const int nl = (int)order.size();
    if (nl >= 0xffff) {
      O.err = "example too large: more than 65534 non-leaf DAG nodes";
      O.rc = SK_ERR_UNSUPPORTED;
      return;
    }
    std::vector<int> nid(nn, -1);
    for (int k = 0; k < nl; ++k) nid[order[k]] = k;
    // per-node gamma (bit 0) / phi (bit 1) row flags, tested once here: the
    // passes below ask repeatedly
    // and their (code, len) key's index (looked up once per node)
    std::vector<uint8_t> fl(nn, 0);
    std::vector<uint32_t> gix(nn, 0);
    if (gam_on)
      for (int v = 0; v < nn; ++v) fl[v] |= is_gamma(X, v) ? 1 : 0;
    if (phi_on)
      for (int v = 0; v < nn; ++v) fl[v] |= is_phi(X, v) ? 2 : 0;
    for (int v = 0; v < nn; ++v)
      if (fl[v]) gix[v] = gamma_idx(gamma_key(X, v));
    {
      const size_t ne_x = (size_t)X.n_edges();
      for (auto* q : {&O.nd_a, &O.nd_b, &O.nd_c, &O.xr_node, &O.xg_node}) q->reserve(nl);
      O.nd_w.reserve(nl);
      O.nd_nbp.reserve(nl);
      O.nd_P.reserve(nl);
      O.ed.reserve(ne_x);
      O.xr_ch.reserve(ne_x);
      O.xrow.reserve(nl);
      O.xgrow.reserve(nl);
      O.xg_ch.reserve(2 * ne_x + nl);
      O.xg_clg.reserve(2 * ne_x + nl);
      O.xg_cpf.reserve(2 * ne_x + nl);
      O.xg_cty.reserve(2 * ne_x + nl);
      O.bpf_code.reserve(X.bpf_off[nn]);
      O.bpf_p.reserve(X.bpf_off[nn]);
    }
    // path weights: number of root->v paths (parents have larger reference ids)
    std::vector<double> Pw(nn, 0.0);
    for (uint32_t r : X.roots) Pw[r] += 1.0;
    for (int v = nn - 1; v >= 0; --v)
      for (uint32_t k = X.edge_off[v]; k < X.edge_off[v + 1]; ++k) Pw[X.edge_to[k]] += Pw[v];


    bool big_gap = false;
    for (int k = 0; k < nl; ++k) {
      const int v = order[k];
      const uint32_t e0 = X.edge_off[v], e1 = X.edge_off[v + 1];
      const uint32_t b0 = X.bpf_off[v], b1 = X.bpf_off[v + 1];
      const bool loop = level[v] == 0;  // single leaf child
      const uint32_t eloc = (uint32_t)O.ed.size(), bloc = (uint32_t)O.bpf_code.size();
      const uint32_t ne = loop ? 0u : e1 - e0;
      if (eloc > 0xffff || bloc > 0xffff || ne > 0xff || b1 - b0 > 0xff ||
          X.last[v] - X.first[v] > 0xffff) {
        O.err = "example too large for the 16-bit packed DAG layout";
        O.rc = SK_ERR_UNSUPPORTED;
        return;
      }
      O.nd_a.push_back(eloc | (ne << 16) | ((b1 - b0) << 24));
      O.nd_b.push_back((X.last[v] - X.first[v]) | (bloc << 16));
      O.nd_c.push_back(loop ? X.edge_gaps[e0] : 0u);
      O.nd_w.push_back(X.weight[v]);
      O.nd_nbp.push_back(X.prof5[(size_t)X.first[v] * 5 + 4]);
      O.nd_P.push_back(Pw[v]);
      if (!loop) {
        for (uint32_t t = e0; t < e1; ++t) {
          const int c = nid[X.edge_to[t]];
          if (c < 0 || X.edge_gaps[t] > 0xffff) {
            O.err = c < 0 ? "unexpected DAG shape: stem with a leaf child" : "gap count exceeds 65535";
            O.rc = c < 0 ? SK_ERR_INVALID : SK_ERR_UNSUPPORTED;
            return;
          }
          big_gap |= X.edge_gaps[t] > 1023;
          O.ed.push_back(make_uint2((uint32_t)c | (X.edge_gaps[t] << 16), (uint32_t)k));
        }
      }
      for (uint32_t t = b0; t < b1; ++t) {
        O.bpf_code.push_back(X.bpf_code[t]);
        O.bpf_p.push_back(X.bpf_p[t]);
      }
    }
    std::vector<int32_t> lv(nlev + 1, 0);
    for (int k = 0; k < nl; ++k) lv[level[order[k]] + 1]++;
    for (int l = 0; l < nlev; ++l) lv[l + 1] += lv[l];
    O.lvl.insert(O.lvl.end(), lv.begin(), lv.end());
    // the register-class kernel's y records: child:11 | parent:11 | gaps:10
    // (at most 2,047 nodes: every register class keeps its last slot free,
    // the dummy records' target, dag_stem.hip)
    const bool big = nl > 2047 || big_gap;
    O.ex_big.push_back(big ? 1 : 0);

    // (the y-role records are formed after the x-role pass: pack_y below)
    O.nl = nl;
    O.big = big;

    // x-role schedule: rows in reference (post-)order; a row's HBM slot is
    // recycled once its last parent has been produced (LIFO free list keeps
    // hot addresses hot).  Rows nobody reads (roots) get no slot.
    {
      std::vector<int> last_parent(nn, -1);
      for (int v = 0; v < nn; ++v)
        for (uint32_t k = X.edge_off[v]; k < X.edge_off[v + 1]; ++k)
          last_parent[X.edge_to[k]] = std::max(last_parent[X.edge_to[k]], v);
      std::vector<uint32_t> slot(nn, 0xffff);
      std::vector<int> free_list;
      int nslots = 0;
      for (int v = 0; v < nn; ++v) {
        if (level[v] < 0) continue;
        const bool loop = level[v] == 0;
        const uint32_t e0 = X.edge_off[v], e1 = X.edge_off[v + 1];
        const uint32_t b0 = X.bpf_off[v], b1 = X.bpf_off[v + 1];
        uint32_t nch = 0;
        if (!loop) {
          for (uint32_t k = e0; k < e1; ++k) {
            const int c = X.edge_to[k];
            O.xr_ch.push_back(slot[c] | (X.edge_gaps[k] << 16));
            ++nch;
          }
        }
        for (uint32_t k = e0; k < e1; ++k) {
          const int c = X.edge_to[k];
          if (level[c] >= 0 && last_parent[c] == v && slot[c] != 0xffff) free_list.push_back(slot[c]);
        }
        if (last_parent[v] >= 0) {
          int sl;
          if (!free_list.empty()) {
            sl = free_list.back();
            free_list.pop_back();
          } else {
            sl = nslots++;
          }
          slot[v] = (uint32_t)sl;
        }
        sk::XRow xr;
        xr.a = nch | ((b1 - b0) << 8) | ((loop ? X.edge_gaps[e0] : 0u) << 16);
        xr.b = (X.last[v] - X.first[v]) | (slot[v] << 16);
        xr.w = X.weight[v];
        xr.nbp = X.prof5[(size_t)X.first[v] * 5 + 4];
        xr.bp0 = b1 > b0 ? X.bpf_p[b0] : 0.0f;
        xr.P = Pw[v];
        // bpf_beg in the level-order bpf array of this example (see nd_b)
        xr.c = (O.nd_b[nid[v]] >> 16) | ((b1 > b0 ? (uint32_t)X.bpf_code[b0] : 0u) << 16);
        O.xrow.push_back(xr);
        O.xr_node.push_back((uint32_t)nid[v]);
      }
      if (nslots >= 0xffff) {
        O.err = "too many live DAG rows";
        O.rc = SK_ERR_UNSUPPORTED;
        return;
      }
      O.ex_nslots.push_back(nslots);
      O.max_slots = std::max(O.max_slots, nslots);

      // the gamma schedule: the same post-order without the gamma rows
      // (slots only among the remaining rows; a gamma child is a record
      // 0x8000 | gamma index, its weight factors g^lg pf in xg_clg / xg_cpf)
      std::vector<uint32_t> gslot(nn, 0xffff);
      std::vector<int> gfree;
      int gslots = 0, nlxg = 0;
      // row order: a depth-first post-order whose last-visited child of a
      // row is, where it can be, one that row alone reads among its first
      // four records (stored nowhere: the row takes it from registers; see
      // below), the reference numbering with SK_REF_ORDER; then each phi row
      // moved to just before its first parent (it has no row children, so
      // any earlier place is valid): the parent takes it from registers too
      // (distance 1), and the row before it, usually a swept one, prefetches
      // its first components
      std::vector<int> order;
      {
        std::vector<int> npar(nn, 0), cand(nn, -1);
        for (int v = 0; v < nn; ++v)
          for (uint32_t k = X.edge_off[v]; k < X.edge_off[v + 1]; ++k) ++npar[X.edge_to[k]];
        for (int v = 0; v < nn; ++v) {
          if (level[v] <= 0 || (fl[v] & 2)) continue;
          for (uint32_t k = X.edge_off[v]; k < X.edge_off[v + 1] && k < X.edge_off[v] + 4; ++k) {
            const int c = X.edge_to[k];
            if (npar[c] == 1 && level[c] >= 0 && !(fl[c] & 1)) {
              cand[v] = c;
              break;
            }
          }
        }
        if (SK_KNOB("SK_REF_ORDER")) {
          for (int v = 0; v < nn; ++v)
            if (level[v] >= 0) order.push_back(v);
        } else {
          std::vector<uint8_t> seen(nn, 0);
          std::vector<std::pair<int, int>> st;  // (row, next child index; -1: candidate done)
          auto dfs = [&](int s) {
            if (seen[s] || level[s] < 0) return;
            seen[s] = 1;
            st.push_back({s, 0});
            while (!st.empty()) {
              auto& [v, i] = st.back();
              const int ne = (int)(X.edge_off[v + 1] - X.edge_off[v]);
              int next = -1;
              while (i >= 0 && i < ne && next < 0) {
                const int c = X.edge_to[X.edge_off[v] + i++];
                if (c != cand[v] && !seen[c] && level[c] >= 0) next = c;
              }
              if (next < 0 && i >= 0) {
                i = -1;
                if (cand[v] >= 0 && !seen[cand[v]]) next = cand[v];
              }
              if (next < 0) {
                order.push_back(v);
                st.pop_back();
              } else {
                seen[next] = 1;
                st.push_back({next, 0});
              }
            }
          };
          for (uint32_t r : X.roots) dfs((int)r);
          for (int v = nn - 1; v >= 0; --v) dfs(v);
        }
        std::vector<int> pos(nn, nn), first_parent(nn, nn);
        for (int i = 0; i < (int)order.size(); ++i) pos[order[i]] = i;
        for (int v = 0; v < nn; ++v)
          for (uint32_t k = X.edge_off[v]; k < X.edge_off[v + 1]; ++k) {
            const int c = X.edge_to[k];
            if (pos[v] < nn && (first_parent[c] == nn || pos[v] < pos[first_parent[c]])) first_parent[c] = v;
          }
        // the phi rows moved before each row (first parent nn: the roots'),
        // in order, as one CSR list
        const bool move = phi_on && !SK_KNOB("SK_PHI_POSTORDER");
        std::vector<int> o1, boff(nn + 2, 0), bl;
        o1.reserve(order.size());
        for (int v : order) {
          if (move && (fl[v] & 2)) ++boff[first_parent[v] + 1];
          else o1.push_back(v);
        }
        for (int i = 0; i <= nn; ++i) boff[i + 1] += boff[i];
        bl.resize(boff[nn + 1]);
        {
          std::vector<int> bf(boff.begin(), boff.end() - 1);
          for (int v : order)
            if (move && (fl[v] & 2)) bl[bf[first_parent[v]]++] = v;
        }
        std::vector<int> o2;
        o2.reserve(order.size() + 8);
        for (int v : o1) {
          const auto bb = bl.begin() + boff[v], be = bl.begin() + boff[v + 1];
          const auto it = std::find(bb, be, cand[v]);
          if (it != be) {
            std::rotate(it, it + 1, be);  // the candidate last
            o2.insert(o2.end(), bb, be);
          } else if (bb != be && cand[v] >= 0 && !o2.empty() && o2.back() == cand[v]) {
            o2.pop_back();
            o2.insert(o2.end(), bb, be);
            o2.push_back(cand[v]);
          } else {
            o2.insert(o2.end(), bb, be);
          }
          o2.push_back(v);
        }
        o2.insert(o2.end(), bl.begin() + boff[nn], bl.begin() + boff[nn + 1]);  // roots
        order.swap(o2);
      }
      // each row's slot is freed at its last parent in this order
      std::vector<int> glast(nn, -1);
      {
        std::vector<int> gpos(nn, -1);
        for (int i = 0; i < (int)order.size(); ++i) gpos[order[i]] = i;
        for (int v : order)
          for (uint32_t k = X.edge_off[v]; k < X.edge_off[v + 1]; ++k) {
            const int c = X.edge_to[k];
            if (glast[c] < 0 || gpos[v] > gpos[glast[c]]) glast[c] = v;
          }
      }
      // rows read only by the next row, among its first four children, are
      // never stored: the next row takes them from registers (slot 0xfffe)
      std::vector<uint8_t> nostore(nn, 0);
      if (!SK_KNOB("SK_STORE_ALL")) {
        std::vector<int> npar(nn, 0), emitted;
        for (int v = 0; v < nn; ++v)
          for (uint32_t k = X.edge_off[v]; k < X.edge_off[v + 1]; ++k) ++npar[X.edge_to[k]];
        for (int v : order)
          if (!(fl[v] & 1)) emitted.push_back(v);
        for (size_t i = 0; i + 1 < emitted.size(); ++i) {
          const int v = emitted[i], r = emitted[i + 1];
          if (npar[v] != 1 || level[r] <= 0 || level[v] < 0 || (fl[r] & 2)) continue;
          for (uint32_t k = X.edge_off[r]; k < X.edge_off[r + 1] && k < X.edge_off[r] + 4; ++k)
            if (X.edge_to[k] == v) nostore[v] = 1;
        }
      }
      for (int v : order) {
        const uint32_t e0 = X.edge_off[v], e1 = X.edge_off[v + 1];
        const uint32_t b0 = X.bpf_off[v], b1 = X.bpf_off[v + 1];
        if (fl[v] & 1) {
          O.gr_info.push_back(gix[v] | (X.edge_gaps[e0] << 16));
          O.gr_pf.push_back(X.bpf_p[b0]);
          O.gr_P.push_back(Pw[v]);
          continue;
        }
        const bool loop = level[v] == 0;
        const bool phi = (fl[v] & 2) != 0;
        uint32_t nch = 0;
        if (phi) {
          // components: per child c a Phi row (type 2) and its Gamma row
          // (type 4), then Gamma_{code,len} of the row itself (type 3)
          const uint32_t kp = gamma_key(X, v);
          for (uint32_t k = e0; k < e1; ++k) {
            const int c = X.edge_to[k];
            const uint32_t kc = gamma_key(X, c);
            const uint32_t pi = phi_idx(kp, kc);
            for (int ty : {2, 4}) {
              O.xg_ch.push_back(((ty == 2 ? 0x4000u | pi : 0x8000u | gix[c])) | (X.edge_gaps[k] << 16));
              O.xg_clg.push_back(X.edge_gaps[X.edge_off[c]]);
              O.xg_cpf.push_back(X.bpf_p[X.bpf_off[c]]);
              O.xg_cty.push_back((uint8_t)ty);
            }
            O.phk_idx.push_back(pi);
          }
          O.xg_ch.push_back(0x8000u | gix[v]);
          O.xg_clg.push_back(0u);
          O.xg_cpf.push_back(0.0f);
          O.xg_cty.push_back(3);
          O.gra_gidx.push_back(gix[v]);
          O.gra_row.push_back((uint32_t)O.xgrow.size());  // (+ the example's xgrow base)
          nch = 2 * (e1 - e0) + 1;
        } else if (!loop) {
          for (uint32_t k = e0; k < e1; ++k) {
            const int c = X.edge_to[k];
            if (fl[c] & 1) {
              O.xg_ch.push_back((0x8000u | gix[c]) | (X.edge_gaps[k] << 16));
              O.xg_clg.push_back(X.edge_gaps[X.edge_off[c]]);
              O.xg_cpf.push_back(X.bpf_p[X.bpf_off[c]]);
              O.xg_cty.push_back(1);
            } else {
              O.xg_ch.push_back(gslot[c] | (X.edge_gaps[k] << 16));
              O.xg_clg.push_back(0u);
              O.xg_cpf.push_back(1.0f);
              O.xg_cty.push_back(0);
            }
            ++nch;
          }
        }
        for (uint32_t k = e0; k < e1; ++k) {
          const int c = X.edge_to[k];
          if (level[c] >= 0 && glast[c] == v && gslot[c] < 0x4000) {
            gfree.push_back(gslot[c]);
            gslot[c] |= 0x10000;  // freed (a second edge to c must not free it again)
          }
        }
        if (nostore[v]) {
          gslot[v] = 0xfffe;
        } else if (last_parent[v] >= 0) {
          int sl;
          if (!gfree.empty()) {
            sl = gfree.back();
            gfree.pop_back();
          } else {
            sl = gslots++;
          }
          gslot[v] = (uint32_t)sl;
        }
        sk::XRow xr;
        xr.a = nch | ((b1 - b0) << 8) | ((loop ? X.edge_gaps[e0] : 0u) << 16);
        xr.b = (X.last[v] - X.first[v]) | (gslot[v] << 16);
        xr.w = X.weight[v];
        xr.nbp = X.prof5[(size_t)X.first[v] * 5 + 4];
        xr.bp0 = b1 > b0 ? X.bpf_p[b0] : 0.0f;
        xr.P = Pw[v];
        xr.c = (O.nd_b[nid[v]] >> 16) | ((b1 > b0 ? (uint32_t)X.bpf_code[b0] : 0u) << 16) |
               (phi ? 0x80000000u : 0u);
        O.xgrow.push_back(xr);
        O.xg_node.push_back((uint32_t)nid[v]);
        ++nlxg;
      }
      if (phi_on) {  // this example's phi keys as a bitset (items take unions)
        const size_t W = (P.phi_al.size() + 63) / 64;
        O.ex_phi_bits.assign(W, 0ull);
        for (size_t j = 0; j < O.phk_idx.size(); ++j)
          O.ex_phi_bits[O.phk_idx[j] / 64] |= 1ull << (O.phk_idx[j] % 64);
      }
      if (gslots >= 0x4000) {  // slot ids share the record with the gamma / phi flags
        O.err = "too many live DAG rows";
        O.rc = SK_ERR_UNSUPPORTED;
        return;
      }
      O.ex_nlxg.push_back(nlxg);
      O.max_slots = std::max(O.max_slots, gslots);
      O.n_nostore = 0;
      for (int v = 0; v < nn; ++v) O.n_nostore += nostore[v];
      O.n_nodes = nn;
      O.gslots = gslots;
    }
    {  // y role: no gap column in any non-leaf node (the Gamma rows need it)
      bool gl = true;
      for (int k = 0; k < nl; ++k) gl &= O.nd_nbp[k] == 0.0f;
      O.ex_gapless.push_back(gl ? 1 : 0);
    }
    O.ex_nl.push_back(nl);
    O.ex_nlev.push_back(nlev);
    O.nlev = nlev;
    O.ex_nseqs.push_back(X.n_seqs);
    O.ex_len.push_back(X.len);
    O.ex_has_w.push_back(X.has_bp ? 1 : 0);
    for (int i = 0; i < X.len; ++i) {
      const float* c = &X.prof5[(size_t)i * 5];
      O.pos_prof.push_back(make_float4(c[0], c[1], c[2], c[3]));
      O.pos_w.push_back(X.has_bp ? X.pos_weight[i] : 1.0f);
      O.pos_chr.push_back((uint8_t)X.rows[0][i]);
    }
    bpla_weights(X, O.pos_lru);
    {
      bool dy = true;  // the device's dyadic_sum test (bpla.hip), in host float
      for (int i = 0; i < X.len; ++i)
        for (int k = 0; k < 4; ++k) {
          const float v = X.prof5[(size_t)i * 5 + k] * 256.0f;
          dy = dy && v == std::rint(v);
        }
      O.ex_dyadic.push_back(dy ? 1 : 0);
      bool full = true;
      for (int i = 0; i < X.len; ++i) {
        const float* c = &X.prof5[(size_t)i * 5];
        full = full && (c[0] + c[1] + c[2] + c[3]) > 0.0f;
      }
      O.ex_str_fast.push_back(dy && full ? 1 : 0);
      bool oh = true;  // the device's onehot_code test (profile_string.hip)
      for (int i = 0; i < X.len && oh; ++i) {
        const float* c = &X.prof5[(size_t)i * 5];
        int ones = 0, zeros = 0;
        for (int k = 0; k < 4; ++k) {
          ones += c[k] == 1.0f;
          zeros += c[k] == 0.0f;
        }
        oh = ones == 1 && zeros == 3;
      }
      O.ex_onehot.push_back(oh ? 1 : 0);
    }
  };
  const double tp1 = tnow();
  double tpx = tp1;
  {
    std::vector<XOut> xo(n);
    std::atomic<int> next{0};
    auto work = [&]() {
      for (int e = next.fetch_add(1); e < n; e = next.fetch_add(1)) pack_x(e, xo[e]);
    };
    run_pool(nthr, work);
    tpx = tnow();
    P.ex_node_base.push_back(0);
    P.ex_edge_base.push_back(0);
    P.ex_bpf_base.push_back(0);
    P.ex_lvl_base.push_back(0);
    P.ex_pos_base.push_back(0);
    // per-example arrays at their prefix-sum offsets, copied on the threads
#define SK_BIG(X) X(nd_a) X(nd_b) X(nd_c) X(nd_w) X(nd_nbp) X(nd_P) X(ed) X(bpf_code) X(bpf_p) X(lvl) \
  X(xr_ch) X(xrow) X(xr_node) X(gr_info) X(gr_pf) X(gr_P) X(xg_ch) X(xg_clg) X(xg_cpf) X(xg_cty)    \
  X(phk_idx) X(gra_gidx) X(gra_row) X(xgrow) X(xg_node) X(pos_prof) X(pos_w) X(pos_chr) X(pos_lru)  \
  X(ex_phi_bits)
#define SK_OFF(f) std::vector<size_t> off_##f(n + 1, 0);
    SK_BIG(SK_OFF)
#undef SK_OFF
    auto app = [](auto& dst, const auto& src) { dst.insert(dst.end(), src.begin(), src.end()); };
    std::vector<long> st_nodes(n), st_nost(n), st_slots(n);  // (SK_PACK_STATS)
    for (int e = 0; e < n; ++e) {
      XOut& O = xo[e];
      st_nodes[e] = O.n_nodes;
      st_nost[e] = O.n_nostore;
      st_slots[e] = O.gslots;
      if (O.rc) {  // the first failing example, as the serial pass would report it
        err = O.err;
        return O.rc;
      }
#define SK_ACC(f) off_##f[e + 1] = off_##f[e] + O.f.size();
      SK_BIG(SK_ACC)
#undef SK_ACC
      yjobs.push_back(YJob{(int)off_nd_a[e], (int)off_ed[e], (int)off_bpf_code[e], O.nl, O.big});
      P.ex_xch_base.push_back((int32_t)off_xr_ch[e]);
      P.ex_xg_base.push_back((int32_t)off_xgrow[e]);
      P.ex_xgch_base.push_back((int32_t)off_xg_ch[e]);
      P.ex_gr_base.push_back((int32_t)off_gr_info[e]);
      P.ex_gra_base.push_back((int32_t)off_gra_gidx[e]);
      P.ex_phk_base.push_back((int32_t)off_phk_idx[e]);
      app(P.ex_big, O.ex_big); app(P.ex_nslots, O.ex_nslots); app(P.ex_nlxg, O.ex_nlxg);
      app(P.ex_gapless, O.ex_gapless); app(P.ex_nl, O.ex_nl); app(P.ex_nlev, O.ex_nlev);
      app(P.ex_nseqs, O.ex_nseqs); app(P.ex_len, O.ex_len); app(P.ex_has_w, O.ex_has_w);
      app(P.ex_dyadic, O.ex_dyadic); app(P.ex_str_fast, O.ex_str_fast); app(P.ex_onehot, O.ex_onehot);
      P.max_slots = std::max(P.max_slots, O.max_slots);
      P.ex_node_base.push_back((int32_t)off_nd_a[e + 1]);
      P.ex_edge_base.push_back((int32_t)off_ed[e + 1]);
      P.ex_bpf_base.push_back((int32_t)off_bpf_code[e + 1]);
      P.ex_lvl_base.push_back((int32_t)off_lvl[e + 1]);
      P.ex_pos_base.push_back((int32_t)off_pos_prof[e + 1]);
      P.max_nl = std::max(P.max_nl, O.nl);
      P.max_edges = std::max(P.max_edges, (int)O.ed.size());
      P.max_bpf = std::max(P.max_bpf, (int)O.bpf_code.size());
      P.max_nlev = std::max(P.max_nlev, O.nlev);
      P.max_len = std::max(P.max_len, ds->ex[e].len);
    }
    const double tq1 = tnow();
#define SK_SIZE(f) P.f.resize(off_##f[n]);
    SK_BIG(SK_SIZE)
#undef SK_SIZE
    const double tq2 = tnow();
    {
      std::atomic<int> nx{0};
      auto copy = [&]() {
        for (int e = nx.fetch_add(1); e < n; e = nx.fetch_add(1)) {
          XOut& O = xo[e];
          for (uint32_t& r : O.gra_row) r += (uint32_t)off_xgrow[e];  // example-local -> dataset row
#define SK_CPY(f) std::copy(O.f.begin(), O.f.end(), P.f.begin() + off_##f[e]);
          SK_BIG(SK_CPY)
#undef SK_CPY
          O = XOut();  // free as we go
        }
      };
      run_pool(nthr, copy);
    }
    if (tstats) fprintf(stderr, "[sk pack] offsets %.1f ms, resize %.1f ms, copy %.1f ms\n", tq1 - tpx, tq2 - tq1, tnow() - tq2);
#undef SK_BIG
    if (tstats) fprintf(stderr, "[sk pack] keys %.1f ms, x-role %.1f ms (%d threads) + append %.1f ms\n",
                        tp1 - tp0, tpx - tp1, nthr, tnow() - tpx);
    if (std::getenv("SK_PACK_STATS")) {  // diagnostic: rows, unstored rows, slots
      long s_rows = 0, s_nost = 0, s_slots = 0, s_nodes = 0, s_st = 0, s_slab = 0, s_gam = 0, s_phi = 0,
           s_reg = 0;
      for (int e = 0; e < n; ++e) {
        s_rows += P.ex_nlxg[e];
        s_nodes += st_nodes[e];
        s_nost += st_nost[e];
        s_slots += st_slots[e];
        // row reads the kernel issues: slab / Gamma / Phi child records, minus
        // the previous row (taken from registers); stored rows
        uint32_t prev = 0xffffu;
        size_t k = (size_t)P.ex_xgch_base[e];
        for (size_t r = (size_t)P.ex_xg_base[e]; r < (size_t)P.ex_xg_base[e] + P.ex_nlxg[e]; ++r) {
          const int ne = P.xgrow[r].a & 0xff;
          for (int t = 0; t < ne; ++t, ++k) {
            const uint32_t c = P.xg_ch[k] & 0xffffu;
            if (c == prev) ++s_reg;
            else if (c & 0x8000u) ++s_gam;
            else if (c & 0x4000u) ++s_phi;
            else ++s_slab;
          }
          prev = P.xgrow[r].b >> 16;
          s_st += prev < 0x4000u;
        }
      }
      fprintf(stderr,
              "[sk pack] gamma schedule: %ld nodes, %ld rows, %ld unstored, %ld slots; stored %ld, reads: "
              "slab %ld gamma %ld phi %ld, from registers %ld\n",
              s_nodes, s_rows, s_nost, s_slots, s_st, s_slab, s_gam, s_phi, s_reg);
    }
  }
  // the x-role arrays are final: the caller may start uploading them while
  // the y-role records are formed (sk_dataset_upload)
  if (after_x) (*after_x)();
  const double tp2 = tnow();
  {
    std::vector<YOut> yo(yjobs.size());
    const int nthr = (int)std::max<size_t>(1, std::min<size_t>({yjobs.size() / 8 + 1, pcap,
                                                                (size_t)std::max(1u, std::thread::hardware_concurrency())}));
    std::atomic<size_t> next{0};
    auto work = [&]() {
      for (size_t e = next.fetch_add(1); e < yjobs.size(); e = next.fetch_add(1)) pack_y(yjobs[e], yo[e]);
    };
    run_pool(nthr, work);
    const double ty1 = tnow();
    // appended at prefix-sum offsets, copied on the threads (as the x role)
    const size_t ny = yo.size();
#define SK_YBIG(X) X(ysc) X(ycs) X(ye2) X(yn_a) X(yn_b) X(yn_c) X(yn_p0) X(yrec) X(yn_w) X(yn_nbp) X(yn_P)
#define SK_OFF(f) std::vector<size_t> off_##f(ny + 1, 0);
    SK_YBIG(SK_OFF)
#undef SK_OFF
    for (size_t e = 0; e < ny; ++e) {
      YOut& Y = yo[e];
      if (!Y.err.empty()) {
        err = Y.err;
        return SK_ERR_INVALID;
      }
#define SK_ACC(f) off_##f[e + 1] = off_##f[e] + Y.f.size();
      SK_YBIG(SK_ACC)
#undef SK_ACC
      P.ex_ysc_base.push_back((int32_t)(off_ysc[e] / 64));
      P.ex_ycs_base.push_back((int32_t)off_ycs[e]);
      P.ex_nch.push_back(Y.nch);
      P.max_nch = std::max(P.max_nch, Y.nch);
    }
#define SK_SIZE(f) P.f.resize(off_##f[ny]);
    SK_YBIG(SK_SIZE)
#undef SK_SIZE
    next = 0;
    auto copy = [&]() {
      for (size_t e = next.fetch_add(1); e < ny; e = next.fetch_add(1)) {
        YOut& Y = yo[e];
#define SK_CPY(f) std::copy(Y.f.begin(), Y.f.end(), P.f.begin() + off_##f[e]);
        SK_YBIG(SK_CPY)
#undef SK_CPY
        Y = YOut();  // free as we go
      }
    };
    run_pool(nthr, copy);
#undef SK_YBIG
    if (tstats) {
      long tch = 0;
      for (int32_t c : P.ex_nch) tch += c;
      fprintf(stderr, "[sk pack] y-role %.1f ms (%d threads) + append %.1f ms; sweep chunks %ld (%.2f per y)\n",
              ty1 - tp2, nthr, tnow() - ty1, tch, P.ex_nch.empty() ? 0.0 : (double)tch / P.ex_nch.size());
    }
  }
  return SK_OK;
}

// ------------------------------------------------------------ parameters
bool kind_is_bpla(int k) { return k >= SK_BPLA && k <= SK_LA_SW; }
bool kind_has_stem(int k) {
  return k != SK_SU_STR && k != SK_SI_STR && k != SK_NAIVE_STR && !kind_is_bpla(k) &&
         k != SK_STEM4D;
}
bool kind_has_str(int k) {
  return k == SK_SU_STR || k == SK_SI_STR || k == SK_SU_STEM_STR || k == SK_SI_STEM_STR ||
         k == SK_LSU_STEM_STR || k == SK_NAIVE_STR;
}
bool kind_subst(int k) {  // RIBOSUM (Su*) vs match/mismatch (Si*)
  return k == SK_SU_STEM || k == SK_SU_STR || k == SK_SU_STEM_STR || k == SK_LSU_STEM ||
         k == SK_LSU_STEM_STR;
}
int32_t combine_mode(int k) {
  switch (k) {
    case SK_SU_STEM:
    case SK_SI_STEM: return sk::kCombineStem;
    case SK_SU_STR:
    case SK_SI_STR:
    case SK_NAIVE_STR: return sk::kCombineStr;
    case SK_SU_STEM_STR:
    case SK_SI_STEM_STR: return sk::kCombineAdd;
    case SK_LSU_STEM: return sk::kCombineLogStem;
    default: return sk::kCombineLogAdd;
  }
}

std::vector<double> gap_powers(double g, int n) {
  // SimpleEdgeScore::initialize (score_table.cpp:60-77): g[k] = g[k-1]*gap
  std::vector<double> v(std::max(n, 1));
  v[0] = 1.0;
  for (int k = 1; k < n; ++k) v[k] = v[k - 1] * g;
  return v;
}

// ------------------------------------------------------------ work buffers
struct Arena {
  char* base;
  size_t off = 0, cap;
  template <class T>
  T* take(size_t n) {
    off = (off + 255) & ~size_t(255);
    T* p = reinterpret_cast<T*>(base + off);
    off += n * sizeof(T);
    return p;
  }
};

int ensure_work(sk_context* ctx, size_t bytes) {
  if (ctx->work_bytes >= bytes) return SK_OK;
  if (ctx->work) {
    SK_HIP(ctx, hipStreamSynchronize(ctx->stream));
    (void)hipFree(ctx->work);
    ctx->work = nullptr;
    ctx->work_bytes = 0;
  }
  const size_t b = std::max(bytes, size_t(1) << 20);
  SK_HIP(ctx, hipMalloc(&ctx->work, b));
  ctx->work_bytes = b;
  return SK_OK;
}

int ensure_scratch(sk_context* ctx, size_t bytes) {
  if (ctx->scratch_bytes >= bytes) return SK_OK;
  if (ctx->scratch) {
    SK_HIP(ctx, hipStreamSynchronize(ctx->stream));
    (void)hipFree(ctx->scratch);
    ctx->scratch = nullptr;
    ctx->scratch_bytes = 0;
  }
  void* p = nullptr;
  SK_HIP(ctx, hipMalloc(&p, bytes));
  ctx->scratch = static_cast<double*>(p);
  ctx->scratch_bytes = bytes;
  return SK_OK;
}

int check_set(sk_context* ctx, sk_dataset* ds) {
  if (!ds) return fail(ctx, SK_ERR_INVALID, "null dataset");
  if (!ds->uploaded || ds->device != ctx->device)
    return fail(ctx, SK_ERR_INVALID, "dataset not uploaded to this context's device");
  return SK_OK;
}

// BPLA kinds: one systolic launch (bpla.hip), result straight to out_dev.
int run_bpla(sk_context* ctx, sk_dataset* xs_, sk_dataset* ys_, const sk_kernel_params* kp,
             const int32_t* x, const int32_t* y, int64_t n, double* out_dev) {
  const bool bp = kp->kind == SK_BPLA || kp->kind == SK_BPLA_SW;
  const bool sw = kp->kind == SK_BPLA_SW || kp->kind == SK_LA_SW;
  // SK_HOST_STATS: host time per phase (diagnostic)
  static const bool host_stats = std::getenv("SK_HOST_STATS") != nullptr;
  auto now_ms = [] {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
  };
  const double tb0 = host_stats ? now_ms() : 0.0;
  double tb1 = tb0, tb2 = tb0;
  const HostPack& PX = xs_->pack;
  const HostPack& PY = ys_->pack;
  // per-example lengths and flags once (the pair loops below touch only
  // these small arrays, not the examples)
  const bool general_only = SK_KNOB("SK_BPLA_GENERAL") != nullptr;  // A/B switch
  auto ex_info = [&](const sk_dataset* d, const HostPack& H, std::vector<int32_t>& len,
                     std::vector<uint8_t>& ok, std::vector<uint8_t>& dy) {
    const size_t m = d->ex.size();
    len.resize(m);
    ok.resize(m);
    dy.resize(m);
    for (size_t i = 0; i < m; ++i) {
      len[i] = d->ex[i].len;
      ok[i] = !bp || d->ex[i].has_bp;  // BPLAScore reads p_left/p_right/p_unpair
      dy[i] = !general_only && H.ex_dyadic[i];
    }
  };
  std::vector<int32_t> lx, ly;
  std::vector<uint8_t> okx, oky, dyx, dyy;
  ex_info(xs_, PX, lx, okx, dyx);
  ex_info(ys_, PY, ly, oky, dyy);
  // one pass: cells, validity, fast flags, per-y counts of the fast pairs
  // (fast: both profiles dyadic -- the fast kernel with tabulated LAScore
  // factors; the rest the general one)
  std::vector<uint8_t> fastk((size_t)n);
  std::vector<int32_t> ycnt(ys_->ex.size(), 0);
  double cells = 0.0;
  int64_t n_fast = 0, distinct = 0;
  for (int64_t k = 0; k < n; ++k) {
    const int32_t a = x[k], b = y[k];
    if (!okx[a] || !oky[b])
      return fail(ctx, SK_ERR_INVALID, "BPLA with base pairs needs examples built with use_bp");
    cells += (double)lx[a] * (double)ly[b];
    const uint8_t f = dyx[a] & dyy[b];
    fastk[(size_t)k] = f;
    n_fast += f;
    if (f && ycnt[b]++ == 0) ++distinct;
  }
  ctx->last_cells = cells;
  // Fast pairs first, the permutation undone through oidx; fast pairs
  // grouped by y (a workgroup stages one y for all its waves) when the y's
  // repeat enough, else one pair per wave.  Items: runs of one y of at most
  // SK_BPLA_ITEM pairs (default 16 per wave of a full workgroup).
  std::vector<int32_t> px, py;
  std::vector<int64_t> oidx;
  constexpr int kItemWaves = 8;
  static const int item_max = SK_KNOB("SK_BPLA_ITEM") ? std::max(1, std::atoi(SK_KNOB("SK_BPLA_ITEM")))
                                                          : 16 * sk::kBplaItemsWavesMax;
  std::vector<int2> items;
  {
    const bool group = n_fast >= 4 * kItemWaves * std::max<int64_t>(distinct, 1) &&
                       !SK_KNOB("SK_BPLA_NO_ITEMS");
    const bool permute = n_fast != n || group;
    if (permute && n_fast) {
      px.resize((size_t)n);
      py.resize((size_t)n);
      oidx.resize((size_t)n);
      // fast pairs in y order (stable counting sort) or in call order, then
      // the general ones
      std::vector<int64_t> pos(ys_->ex.size() + 1, 0);
      if (group)
        for (size_t j = 0; j < ys_->ex.size(); ++j) pos[j + 1] = pos[j] + ycnt[j];
      int64_t f = 0, g = n_fast;
      for (int64_t k = 0; k < n; ++k) {
        const int64_t d = fastk[(size_t)k] ? (group ? pos[y[k]]++ : f++) : g++;
        px[(size_t)d] = x[k];
        py[(size_t)d] = y[k];
        oidx[(size_t)d] = k;
      }
      if (group)  // runs of one y
        for (int64_t a = 0; a < n_fast;) {
          int64_t b = a;
          while (b < n_fast && py[(size_t)b] == py[(size_t)a] && b - a < item_max) ++b;
          items.push_back(make_int2((int)a, (int)(b - a)));
          a = b;
        }
      x = px.data();
      y = py.data();
    }
  }
  if (host_stats) tb1 = now_ms();
  const bool permute = !oidx.empty();
  const size_t nb = (size_t)n;
  const size_t npx = PX.pos_prof.size(), npy = ys_ == xs_ ? 0 : PY.pos_prof.size();
  const size_t ntab = n_fast ? 2 * (npx + npy) : 0;
  int rc = ensure_work(ctx, 16 * 8 + nb * 8 + (permute ? nb * 8 : 0) + ntab * sizeof(sk::BplaPos) +
                                items.size() * sizeof(int2) + 8192);
  if (rc) return rc;
  // the call's host inputs and zeroed counters are laid out as on the device
  // and go up in ONE copy (separate small copies and a memset cost the
  // stream ~0.1 ms of gaps per call); asynchronous calls upload them on the
  // copy stream into a buffer of their own (up_reserve), overlapping the
  // previous call's kernels
  double* d_tb;
  unsigned long long* d_ctr;
  int32_t *d_px, *d_py;
  int64_t* d_oidx;
  int2* d_items;
  auto lay = [&](Arena& U) {
    d_tb = U.take<double>(16);
    d_ctr = U.take<unsigned long long>(8);
    d_px = U.take<int32_t>(nb);
    d_py = U.take<int32_t>(nb);
    d_oidx = permute ? U.take<int64_t>(nb) : nullptr;
    d_items = items.empty() ? nullptr : U.take<int2>(items.size());
  };
  Arena A{static_cast<char*>(ctx->work), 0, ctx->work_bytes};
  Arena U{nullptr, 0, 0};
  lay(U);  // (sizes only)
  const size_t up_bytes = U.off;
  if (ctx->async) {
    char* ub = nullptr;
    SK_HIP(ctx, sk::up_reserve(ctx, up_bytes, &ub));
    U = Arena{ub, 0, up_bytes};
    lay(U);
  } else {
    lay(A);
    U.base = A.base;
  }
  sk::BplaPos* d_tab = ntab ? A.take<sk::BplaPos>(ntab) : nullptr;
  hipStream_t S = ctx->stream;
  {
    thread_local std::vector<char> hb;
    hb.assign(up_bytes, 0);
    auto put = [&](const void* dptr, const void* src, size_t bytes) {
      if (bytes) std::memcpy(hb.data() + (static_cast<const char*>(dptr) - U.base), src, bytes);
    };
    put(d_tb, kp->score_table, 16 * 8);
    put(d_px, x, nb * 4);
    put(d_py, y, nb * 4);
    if (permute) put(d_oidx, oidx.data(), nb * 8);
    if (d_items) put(d_items, items.data(), items.size() * sizeof(int2));
    if (ctx->async)
      SK_HIP(ctx, sk::up_copy(ctx, hb.data(), up_bytes, S));
    else
      SK_HIP(ctx, sk::h2d(ctx, U.base, hb.data(), up_bytes, S));
  }
  sk::BplaLaunch T;
  T.xset = xs_->dev;
  T.yset = ys_->dev;
  T.table = d_tb;
  T.alpha = kp->alpha;
  T.beta = kp->beta;
  T.gap = kp->gap;
  T.ext = kp->ext;
  T.beta_gap = std::exp(kp->beta * kp->gap);  // bpla_kernel.cpp:70-71
  T.beta_ext = std::exp(kp->beta * kp->ext);
  T.sw = sw ? 1 : 0;
  T.bp = bp ? 1 : 0;
  T.oidx = d_oidx;
  T.out = out_dev;
  if (host_stats) tb2 = now_ms();
  SK_HIP(ctx, hipEventRecord(ctx->ev0, S));
  if (n_fast) {
    // x-role table of the x set, y-role table of the y set
    sk::BplaPos* tx = d_tab;           // [npx] x role | [npx] y role
    sk::BplaPos* ty = d_tab + npx;
    // the exp path's x operands carry beta (bpla_fast_chunk2)
    const double xscale = sw ? 1.0 : kp->beta;
    SK_HIP(ctx, sk::launch_bpla_tab(xs_->dev.pos_prof, xs_->dev.pos_lru, (int64_t)npx, d_tb, xscale, tx,
                                    d_tab + npx, S));
    if (npy) {
      ty = d_tab + 2 * npx + npy;      // [npy] x role (unused) | [npy] y role
      SK_HIP(ctx, sk::launch_bpla_tab(ys_->dev.pos_prof, ys_->dev.pos_lru, (int64_t)npy, d_tb, xscale,
                                      d_tab + 2 * npx, ty, S));
    }
    sk::BplaLaunch F = T;
    F.xtab = tx;
    F.ytab = ty;
    F.xs = d_px;
    F.ys = d_py;
    F.n_pairs = n_fast;
    F.pair_counter = d_ctr;
    F.lds_max_len = (std::max(PY.max_len, 64) + 1) & ~1;
    int w, per_cu;
    int64_t units;
    if (d_items) {  // y-grouped: workgroups of up to 16 waves sharing the y columns
      F.items = d_items;
      F.n_items = (int32_t)items.size();
      // pairs a wave streams back to back (SK_BPLA_CHUNK: 1..kBplaChunkMax)
      // (0: per item, as many as give each wave one chunk)
      F.chunk = 8;  // C4, items of 192 pairs: 7.99 ms per launch against 8.58 (4) and 8.97 (16)
      if (const char* e = SK_KNOB("SK_BPLA_CHUNK")) F.chunk = std::atoi(e);
      F.chunk = std::min(std::max(F.chunk, 0), sk::kBplaChunkMax);
      // waves per workgroup and workgroups per CU (SK_BPLA_IWAVES /
      // SK_BPLA_IWG: geometry experiments; the VGPR budget caps the waves
      // a SIMD holds, whatever is asked)
      // Default: one 16-wave workgroup per CU (C4: 11.1 against 11.7 ms
      // per launch for two 8-wave ones: the y columns staged once for 16
      // waves), halved while its LDS does not fit, the CU's 16 waves then
      // made up by more workgroups.
      static const int iw =
          SK_KNOB("SK_BPLA_IWAVES") ? std::atoi(SK_KNOB("SK_BPLA_IWAVES")) : sk::kBplaItemsWavesMax;
      static const int iwg = SK_KNOB("SK_BPLA_IWG") ? std::atoi(SK_KNOB("SK_BPLA_IWG")) : 0;
      w = std::min(std::max(iw, 1), sk::kBplaItemsWavesMax);
      while (w > 1 && sk::bpla_items_lds_bytes(F.lds_max_len, w) > 163840) w /= 2;
      const size_t l = sk::bpla_items_lds_bytes(F.lds_max_len, w);
      if (l > 163840) return fail(ctx, SK_ERR_UNSUPPORTED, "sequence too long for BPLA kernel LDS");
      per_cu = std::max(1, std::min<int>((int)(163840 / l), iwg > 0 ? iwg : std::max(1, sk::kBplaItemsWavesMax / w)));
      units = F.n_items;
    } else {
      const size_t wl = sk::bpla_fast_wave_lds_bytes(F.lds_max_len);
      if (wl > 163840) return fail(ctx, SK_ERR_UNSUPPORTED, "sequence too long for BPLA kernel LDS");
      // as many waves per CU as the per-wave LDS allows (<= 16), in
      // workgroups of up to 4
      static const int wcap =
          SK_KNOB("SK_BPLA_WAVES") ? std::atoi(SK_KNOB("SK_BPLA_WAVES")) : 16;
      const int per_cu_w =
          (int)std::max<size_t>(1, std::min<size_t>((size_t)wcap, (163840 - 2 * sk::kBplaExpLds) / wl));
      w = std::min(4, per_cu_w);
      per_cu = std::max(1, per_cu_w / w);
      units = (n_fast + w - 1) / w;
    }
    const int64_t g = std::min<int64_t>((int64_t)ctx->n_cu * per_cu, units);
    SK_HIP(ctx, sk::lev_mark(ctx, S));
    SK_HIP(ctx, sk::launch_bpla_fast(F, (int)g, w, S));
    SK_HIP(ctx, sk::lev_mark(ctx, S));
  }
  if (n_fast < n) {
    sk::BplaLaunch G = T;
    G.xs = d_px + n_fast;
    G.ys = d_py + n_fast;
    G.oidx = d_oidx ? d_oidx + n_fast : nullptr;
    G.n_pairs = n - n_fast;
    G.pair_counter = d_ctr + 1;
    G.lds_max_len = (std::max(PY.max_len, 64) + 1) & ~1;
    const int w = 4;
    const size_t lds = sk::bpla_lds_bytes(G, w);
    if (lds > 163840) return fail(ctx, SK_ERR_UNSUPPORTED, "sequence too long for BPLA kernel LDS");
    const int per_cu = std::max(1, std::min<int>((int)(163840 / lds), 8));
    const int64_t g = std::min<int64_t>((int64_t)ctx->n_cu * per_cu, (G.n_pairs + w - 1) / w);
    SK_HIP(ctx, sk::lev_mark(ctx, S));
    SK_HIP(ctx, sk::launch_bpla(G, (int)g, w, S));
    SK_HIP(ctx, sk::lev_mark(ctx, S));
  }
  SK_HIP(ctx, hipEventRecord(ctx->ev1, S));
  const double tb3 = host_stats ? now_ms() : 0.0;
  ctx->last_launches = (n_fast ? 1 : 0) + (n_fast < n ? 1 : 0);
  SK_HIP(ctx, sk::call_finish(ctx, S, true, false));
  if (host_stats)
    fprintf(stderr, "[sk bpla host] plan %.3f ms, uploads %.3f ms, launches %.3f ms, wait %.3f ms (GPU %.3f ms)\n",
            tb1 - tb0, tb2 - tb1, tb3 - tb2, now_ms() - tb3, ctx->async ? -1.0 : ctx->last_stem_ms);
  return SK_OK;
}

// 4-D stem kernel: per example, the lowercased sequence (the loader's
// ToLower, common/example.cpp:26-34) and BPMat::prob(a, b) for a <= b by
// diagonal e = b - a (prob(a,a) = 0), as float (stem_kernel.cpp:320, 328).
void stem4d_tables(const Example& X, const sk_kernel_params* kp, std::vector<float>& bp,
                   std::vector<uint8_t>& chr) {
  const int L = X.len;
  std::string s = X.rows[0];
  for (char& c : s) c = (char)std::tolower((unsigned char)c);
  chr.assign(s.begin(), s.end());
  chr.push_back(0);
  bp.clear();
  for (int e = 0; e < L; ++e)
    for (int a = 0; a + e < L; ++a) {
      const int b = a + e;
      float v = 0.0f;
      if (kp->bp_model == 0) {
        if (e > 0) v = (float)X.bpp[sk::tri_index(L, a, b)];
      } else {  // NormalBasePair / WobbleBasePair (stem_kernel.cpp:354-396)
        const char p = s[a], q = s[b];
        bool ok = (p == 'a' && q == 'u') || (p == 'u' && q == 'a') || (p == 'g' && q == 'c') ||
                  (p == 'c' && q == 'g');
        if (kp->bp_model == 2) ok = ok || (p == 'g' && q == 'u') || (p == 'u' && q == 'g');
        v = ((unsigned)a + 1 + kp->loop <= (unsigned)b && ok) ? 1.0f : 0.0f;
      }
      bp.push_back(v);
    }
}

static int stem4d_dataset_tables(sk_context* ctx, sk_dataset* ds, const sk_kernel_params* kp,
                                 std::shared_ptr<const Stem4dTables>* out) {
  std::lock_guard<std::mutex> lk(ds->s4_mu);
  auto same = [&](const std::shared_ptr<Stem4dTables>& t) {
    return t->device == ctx->device && t->model == kp->bp_model && t->loop == kp->loop;
  };
  auto it = std::find_if(ds->s4.begin(), ds->s4.end(), same);
  if (it != ds->s4.end() && (*it)->n_ex == ds->ex.size()) {
    *out = *it;
    return SK_OK;
  }
  auto tp = std::make_shared<Stem4dTables>();
  Stem4dTables& T = *tp;
  const size_t n = ds->ex.size();
  std::vector<float> bpall, bp;
  std::vector<uint8_t> chall, chr;
  T.bp_off.assign(n, -1);
  T.ch_off.assign(n, -1);
  T.why.assign(n, 0);
  T.acgu.assign(n, 0);
  for (size_t e = 0; e < n; ++e) {
    const Example& X = ds->ex[e];
    if (X.n_rows != 1) {
      T.why[e] = 1;
      continue;
    }
    if (kp->bp_model == 0 && !X.has_bp) {
      T.why[e] = 2;
      continue;
    }
    stem4d_tables(X, kp, bp, chr);
    T.acgu[e] = 1;
    for (int a = 0; a < X.len; ++a)
      if (!std::strchr("acgu", (char)chr[a]) || !chr[a]) T.acgu[e] = 0;
    T.bp_off[e] = (int64_t)bpall.size();
    T.ch_off[e] = (int64_t)chall.size();
    bpall.insert(bpall.end(), bp.begin(), bp.end());
    chall.insert(chall.end(), chr.begin(), chr.end());
  }
  T.device = ctx->device;
  SK_HIP(ctx, upload(T.buf, bpall, &T.bp));
  SK_HIP(ctx, upload(T.buf, chall, &T.ch));
  T.model = kp->bp_model;
  T.loop = kp->loop;
  T.n_ex = n;
  // the set it replaces is freed once no call holds it (after its device
  // synchronizes, ~Stem4dTables)
  if (it != ds->s4.end()) {
    *it = tp;
  } else {
    if (ds->s4.size() >= kS4Sets) ds->s4.erase(ds->s4.begin());
    ds->s4.push_back(tp);
  }
  *out = tp;
  return SK_OK;
}

int64_t stem4d_plane_doubles(int m) {
  int64_t r = 0;
  for (int d2 = 0; d2 <= m; ++d2) r += ((m + 1 - d2) + 3) & ~3;
  return r;
}

// waves per pair of the column kernel for a batch whose y lengths lie in
// [min_m, max_m] (min_m counts |y| >= 2 only; INT32_MAX for none)
static int col_waves(int cpl, int min_m, int max_m, int max_n) {
  static const int w_env = SK_KNOB("SK4C_W") ? std::max(1, std::atoi(SK_KNOB("SK4C_W"))) : 0;
  int W = std::min(w_env ? w_env : sk::stem4d_col_max_waves(cpl), sk::stem4d_col_max_waves(cpl));
  if (min_m != INT32_MAX) W = std::min(W, sk::stem4d_col_w_max(min_m));
  W = std::max(W, 1);
  while (W > 1 && sk::stem4d_col_lds_bytes(cpl, W, max_m, max_n) > 160 * 1024) --W;
  return W;
}

int run_stem4d(sk_context* ctx, sk_dataset* xs_, sk_dataset* ys_, const sk_kernel_params* kp,
               const int32_t* x, const int32_t* y, int64_t n, double* out_dev) {
  if (kp->bp_model < 0 || kp->bp_model > 2 || !(kp->bp_bound >= 0.0))
    return fail(ctx, SK_ERR_INVALID, "4-D stem kernel: bp_model 0..2 and bp_bound >= 0");
  // StemKernel::operator() (stem_kernel.h:52-55): partial_dp when ali_bound
  // > 0 or band > 0; ali_bound is a float option
  const float ali_bound = (float)kp->ali_bound;
  const bool ali = ali_bound > 0.0f;  // -a: residues must be ACGU
  // Anchors come from the PairHMM only with the intended zerop.  As the
  // reference builds today (ali_zerop_fixed 0) every posterior is NaN, no
  // position is anchored and the constraints are [0, |y|] for every x
  // position whatever the band (checked against the oracle's
  // full NaN-propagating restatement), and partial_dp over the full range is
  // full_dp operation for operation.
  const bool ali_phmm = ali && kp->ali_zerop_fixed;
  // per-example tables, resident per dataset (built on first use)
  std::shared_ptr<const Stem4dTables> tx, ty;
  int rc = stem4d_dataset_tables(ctx, xs_, kp, &tx);
  if (rc) return rc;
  if (ys_ == xs_) ty = tx;
  else if ((rc = stem4d_dataset_tables(ctx, ys_, kp, &ty))) return rc;
  const Stem4dTables& TX = *tx;
  const Stem4dTables& TY = *ty;
  auto usable = [&](const Stem4dTables& T, int e) -> int {
    if (T.why[e] == 1) return fail(ctx, SK_ERR_INVALID, "4-D stem kernel takes single sequences");
    if (T.why[e] == 2) return fail(ctx, SK_ERR_INVALID, "4-D stem kernel with bp_model 0 needs base pairs");
    if (ali && !T.acgu[e])  // PairHMM's char2rna asserts on anything else (phmm.cpp:247-258)
      return fail(ctx, SK_ERR_INVALID, "4-D stem kernel: alignment constraints need A/C/G/U sequences");
    return SK_OK;
  };
  int max_m = 0, max_n = 0;
  double cells = 0.0;
  for (int64_t k = 0; k < n; ++k) {
    if ((rc = usable(TX, x[k])) || (rc = usable(TY, y[k]))) return rc;
    const double a = xs_->ex[x[k]].len, b = ys_->ex[y[k]].len;
    max_m = std::max(max_m, (int)b);
    max_n = std::max(max_n, (int)a);
    cells += (a + 1) * (a + 2) / 2 * (b + 1) * (b + 2) / 2;
  }
  ctx->last_cells = cells;
  // batches bounded by scratch memory
  size_t free_b = 0, total_b = 0;
  SK_HIP(ctx, hipMemGetInfo(&free_b, &total_b));
  const double budget = std::min(128e9, 0.5 * (double)free_b);
  std::vector<int64_t> order(n);
  std::iota(order.begin(), order.end(), 0);
  // g^k for y spans (d1 = 0 planes) and, in the column kernel, x spans (the
  // diagonal cells G0(i, j, l, l) = g^(j-i))
  const std::vector<double> gp = gap_powers(kp->gap, std::max(max_m, max_n) + 2);
  rc = ensure_work(ctx, gp.size() * 8 + 4096);
  if (rc) return rc;
  Arena A{static_cast<char*>(ctx->work), 0, ctx->work_bytes};
  double* d_gp = A.take<double>(gp.size());
  hipStream_t S = ctx->stream;
  SK_HIP(ctx, hipMemcpyAsync(d_gp, gp.data(), gp.size() * 8, hipMemcpyHostToDevice, S));
  const int cpl = sk::stem4d_cpl(max_m);
  // |y| >= 512: the kernel sweeps k tiles of 512 and hands each tile's first
  // K3/G3 column to the next through per-item boundary columns
  const bool ktiles = max_m + 1 > 64 * cpl;
  const int64_t kb_stride = ktiles ? 4 * (int64_t)(max_m + 1) : 0;
  // full_dp: G-only planes with the K chain summed (stem4d.hip); the banded
  // and PairHMM-constrained partial_dp keep the four-state planes (their
  // boundary approximations read K0 / K1 off the band)
  const bool banded = ali_phmm || (!ali && kp->len_band > 0);
  const bool gsum = !banded && !SK_KNOB("SK4_NO_GSUM");
  const size_t nst = gsum ? 2 : 4;
  // full_dp with one k tile: the column-group kernel (one workgroup per pair,
  // B' handed on through LDS, NB columns chained per position;
  // stem4d.hip sk_stem4d_col_kernel); SK4_SPAN=1 (per call, A/B) runs the
  // pre-combined span kernel instead, SK4_NO_PRE=1 the K-sum span kernel
  // (pairs whose y is too short for the column schedule, 2 <= m < 2 PF + 3,
  // go to the span kernel in batches of their own)
  const bool colk_call = gsum && !ktiles && !SK_KNOB("SK4_SPAN") && !SK_KNOB("SK4_NO_PRE");
  const int col_nb = colk_call ? sk::stem4d_col_nb(cpl) : 0;
  // (|x| <= stem4d_col_max_n(): the kernel holds x in LDS and counts its
  // steps in an int; longer x take the span kernel)
  auto col_ok = [&](int64_t q) {
    const int m = ys_->ex[y[q]].len;
    return colk_call && xs_->ex[x[q]].len <= sk::stem4d_col_max_n() &&
           (m <= 1 || sk::stem4d_col_w_max(m) >= 1);
  };
  // batches of one kernel: the column kernel's pairs first, then longest x first
  std::stable_sort(order.begin(), order.end(), [&](int64_t a, int64_t b) {
    const bool ca = col_ok(a), cb = col_ok(b);
    if (ca != cb) return ca;
    return xs_->ex[x[a]].len > xs_->ex[x[b]].len;
  });
  double total_ms = 0.0;
  int launches = 0;
  Stem4dBatch& Bt = ctx->s4d;
  for (int64_t b0 = 0; b0 < n;) {
    // pairs of this batch and their scratch
    std::vector<sk::Stem4dPair> prs;
    double bytes = 0.0;     // rings + boundary columns (the budget)
    size_t ring_bytes = 0;  // rings only: pair p's at scratch_off, boundary columns after all
    int64_t b1 = b0;
    int maxn = 0;
    const bool colk = col_ok(order[b0]);
    while (b1 < n && prs.size() < 4096 && col_ok(order[b1]) == colk) {
      const int64_t q = order[b1];
      sk::Stem4dPair p;
      p.n = xs_->ex[x[q]].len;
      p.m = ys_->ex[y[q]].len;
      p.plane_doubles = stem4d_plane_doubles(p.m);
      // column kernel: n G0 planes (slot i) + the round wrap's NB B' planes;
      // span kernels: a ring of three spans of n + 1 planes (+ acc)
      const size_t rb = colk ? ((size_t)(p.n + col_nb) * (size_t)p.plane_doubles * 8 + 255) & ~(size_t)255
                             : ((size_t)3 * (p.n + 1) * nst * (size_t)p.plane_doubles * 8 +
                                (gsum ? (size_t)(p.n + 1) * 8 : 0) + 255) & ~(size_t)255;
      const double pb = (double)rb + (double)(p.n + 1) * (double)kb_stride * 8.0;
      if (!prs.empty() && bytes + pb > budget) break;
      p.scratch_off = (int64_t)(ring_bytes / 8);
      bytes += pb;
      ring_bytes += rb;
      p.x_bp = TX.bp_off[x[q]];
      p.x_chr = TX.ch_off[x[q]];
      p.y_bp = TY.bp_off[y[q]];
      p.y_chr = TY.ch_off[y[q]];
      p.out_index = q;
      maxn = std::max(maxn, p.n);
      prs.push_back(p);
      ++b1;
    }
    if (colk) {
      // one launch for the batch: W waves per pair, W <= m - 2 PF - 2 for
      // every pair (the round wrap's lag, stem4d.hip kS4cV; |y| <= 1: no
      // stacking source, K = 1 without a step), the class's register budget
      // and 160 KB of LDS (SK4C_W: fewer, A/B)
      int min_m = INT32_MAX;
      for (const auto& p : prs)
        if (p.m >= 2) min_m = std::min(min_m, p.m);
      const int W = col_waves(cpl, min_m, max_m, maxn);
      rc = ensure_scratch(ctx, ring_bytes + 64);
      if (rc) return rc;
      if (Bt.cap_pairs < prs.size()) {
        if (Bt.pairs) {
          SK_HIP(ctx, hipStreamSynchronize(S));
          (void)hipFree(Bt.pairs);
        }
        Bt.cap_pairs = std::max<size_t>(prs.size(), 64);
        SK_HIP(ctx, hipMalloc(&Bt.pairs, Bt.cap_pairs * sizeof(sk::Stem4dPair)));
      }
      SK_HIP(ctx, hipMemcpyAsync(Bt.pairs, prs.data(), prs.size() * sizeof(sk::Stem4dPair),
                                 hipMemcpyHostToDevice, S));
      sk::Stem4dLaunch L;
      L.pairs = Bt.pairs;
      L.scratch = ctx->scratch;
      L.bpdiag = TX.bp;
      L.chars = TX.ch;
      L.bpdiag_y = TY.bp;
      L.chars_y = TY.ch;
      L.gpow = d_gp;
      L.gap = kp->gap;
      L.stack = kp->stack;
      L.subst = kp->subst;
      L.bp_bound = (float)kp->bp_bound;
      L.out = out_dev;
      L.gsum = 3;
      SK_HIP(ctx, hipEventRecord(ctx->ev0, S));
      SK_HIP(ctx, sk::lev_mark(ctx, S));
      SK_HIP(ctx, sk::launch_stem4d_col(L, (int64_t)prs.size(), cpl, W, max_m, maxn, S));
      SK_HIP(ctx, sk::lev_mark(ctx, S));
      ctx->last_s4d_classes |= 1u << ((cpl == 1 ? 0 : cpl == 2 ? 1 : cpl == 4 ? 2 : 3) + 8);
      ++launches;
      SK_HIP(ctx, hipEventRecord(ctx->ev1, S));
      SK_HIP(ctx, hipStreamSynchronize(S));
      SK_HIP(ctx, sk::lev_collect(ctx));
      float ms = 0.f;
      SK_HIP(ctx, hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
      total_ms += ms;
      b0 = b1;
      continue;
    }
    // partial_dp constraints per pair: x position -> [c_low, c_high].  With
    // -a the PairHMM kernel writes them on the device; with -b alone
    // (alignment_constraints with ali_bound 0, stem_kernel.cpp:68-74) they
    // are formed here.
    std::vector<int32_t> blo, bhi;
    size_t n_band = 0;
    int max_n1 = 1, max_m1 = 1;
    if (ali_phmm) {
      for (auto& p : prs) {
        p.band_off = (int64_t)n_band;
        n_band += (size_t)p.n + 1;
        max_n1 = std::max(max_n1, p.n + 1);
        max_m1 = std::max(max_m1, p.m + 1);
      }
    } else if (!ali && kp->len_band > 0) {
      for (auto& p : prs) {
        p.band_off = (int64_t)blo.size();
        for (int i = 0; i <= p.n; ++i) {
          const unsigned jj = p.n ? (unsigned)((double)i / p.n * p.m + 0.5) : 0u;
          blo.push_back((int32_t)(jj < kp->len_band ? 0u : jj - kp->len_band));
          bhi.push_back((int32_t)(jj + kp->len_band > (unsigned)p.m ? (unsigned)p.m : jj + kp->len_band));
        }
      }
    }
    // work items {pair, i} per span d1 and part, concatenated: the pairs are
    // dealt to nh parts whose launches run on their own streams (main, class,
    // side, aux), so each span's tail overlaps the other parts' launches (the
    // boundary columns of k tiles are per launch item: one stream then)
    int nh = SK_KNOB("SK4_STREAMS") ? std::atoi(SK_KNOB("SK4_STREAMS")) : 4;
    if (SK_KNOB("SK_SERIAL_CLASSES") || ktiles) nh = 1;
    nh = std::max(1, std::min({nh, 4, (int)prs.size()}));
    const hipStream_t hs[4] = {S, ctx->cls, ctx->side, ctx->aux};
    std::vector<int2> items;
    std::vector<int64_t> ioff((size_t)(maxn + 1) * nh + 1, 0);
    for (int d1 = 0; d1 <= maxn; ++d1)
      for (int h = 0; h < nh; ++h) {
        ioff[(size_t)d1 * nh + h] = (int64_t)items.size();
        for (size_t p = h; p < prs.size(); p += nh)
          for (int i = 0; i + d1 <= prs[p].n; ++i) items.push_back(make_int2((int)p, i));
      }
    ioff.back() = (int64_t)items.size();
    if (!ali_phmm) n_band = blo.size();
    const size_t phmm_bytes =
        ali_phmm ? prs.size() * sk::phmm_pair_bytes(max_n1, max_m1) : 0;
    // boundary columns after the rings: at most the d1 = 0 launch's items
    const size_t kb_bytes = ktiles ? (size_t)(ioff[nh] - ioff[0]) * (size_t)kb_stride * 8 : 0;
    rc = ensure_scratch(ctx, std::max(ring_bytes + kb_bytes + 64, phmm_bytes));
    if (rc) return rc;
    if (Bt.cap_pairs < prs.size() || Bt.cap_items < items.size()) {
      if (Bt.pairs) (void)hipFree(Bt.pairs);
      if (Bt.items) (void)hipFree(Bt.items);
      Bt.cap_pairs = std::max<size_t>(prs.size(), 64);
      Bt.cap_items = std::max<size_t>(items.size(), 4096);
      SK_HIP(ctx, hipMalloc(&Bt.pairs, Bt.cap_pairs * sizeof(sk::Stem4dPair)));
      SK_HIP(ctx, hipMalloc(&Bt.items, Bt.cap_items * sizeof(int2)));
    }
    SK_HIP(ctx, hipMemcpyAsync(Bt.pairs, prs.data(), prs.size() * sizeof(sk::Stem4dPair),
                               hipMemcpyHostToDevice, S));
    SK_HIP(ctx, hipMemcpyAsync(Bt.items, items.data(), items.size() * sizeof(int2),
                               hipMemcpyHostToDevice, S));
    if (n_band) {
      if (Bt.cap_band < n_band) {
        if (Bt.band) {
          SK_HIP(ctx, hipStreamSynchronize(S));
          (void)hipFree(Bt.band);
        }
        Bt.cap_band = std::max<size_t>(n_band, 4096);
        SK_HIP(ctx, hipMalloc(&Bt.band, 2 * Bt.cap_band * sizeof(int32_t)));
      }
      if (!blo.empty()) {
        SK_HIP(ctx, hipMemcpyAsync(Bt.band, blo.data(), blo.size() * 4, hipMemcpyHostToDevice, S));
        SK_HIP(ctx, hipMemcpyAsync(Bt.band + Bt.cap_band, bhi.data(), bhi.size() * 4,
                                   hipMemcpyHostToDevice, S));
      }
    }
    sk::Stem4dLaunch L;
    L.pairs = Bt.pairs;
    L.scratch = ctx->scratch;
    L.bpdiag = TX.bp;
    L.chars = TX.ch;
    L.bpdiag_y = TY.bp;
    L.chars_y = TY.ch;
    L.gpow = d_gp;
    L.gap = kp->gap;
    L.stack = kp->stack;
    L.subst = kp->subst;
    L.bp_bound = (float)kp->bp_bound;
    L.out = out_dev;
    L.band_lo = n_band ? Bt.band : nullptr;
    L.band_hi = n_band ? Bt.band + Bt.cap_band : nullptr;
    L.kbound = ktiles ? ctx->scratch + ring_bytes / 8 : nullptr;
    L.kbound_stride = kb_stride;
    // one k tile: each plane's stacking chain produced one span early by the
    // plane that streams its G0 rows (stem4d.hip sk_stem4d_pre_kernel)
    const bool no_pre = SK_KNOB("SK4_NO_PRE") != nullptr;  // per call (A/B tests)
    L.gsum = gsum ? (!ktiles && !no_pre ? 2 : 1) : 0;
    SK_HIP(ctx, hipEventRecord(ctx->ev0, S));
    if (ali_phmm) {
      sk::PhmmLaunch H;
      H.pairs = Bt.pairs;
      H.n_pairs = (int64_t)prs.size();
      H.chars = TX.ch;
      H.chars_y = TY.ch;
      H.scratch = reinterpret_cast<char*>(ctx->scratch);
      H.n1 = max_n1;
      H.m1 = max_m1;
      H.pair_bytes = sk::phmm_pair_bytes(max_n1, max_m1);
      H.ali_bound = ali_bound;
      H.band = kp->len_band;
      H.zerop_fixed = kp->ali_zerop_fixed ? 1 : 0;
      H.band_lo = Bt.band;
      H.band_hi = Bt.band + Bt.cap_band;
      SK_HIP(ctx, sk::launch_phmm(H, S));
    }
    if (nh > 1) {
      SK_HIP(ctx, hipEventRecord(ctx->evk, S));
      for (int h = 1; h < nh; ++h) SK_HIP(ctx, hipStreamWaitEvent(hs[h], ctx->evk, 0));
    }
    for (int d1 = 0; d1 <= maxn; ++d1)
      for (int h = 0; h < nh; ++h) {
        const size_t q = (size_t)d1 * nh + h;
        L.d1 = d1;
        L.items = Bt.items + ioff[q];
        L.n_items = ioff[q + 1] - ioff[q];
        if (!L.n_items) continue;
        SK_HIP(ctx, sk::lev_mark(ctx, hs[h]));
        SK_HIP(ctx, sk::launch_stem4d(L, cpl, hs[h]));
        SK_HIP(ctx, sk::lev_mark(ctx, hs[h]));
        ctx->last_s4d_classes |= 1u << ((cpl == 1 ? 0 : cpl == 2 ? 1 : cpl == 4 ? 2 : 3) +
                                        (L.band_lo ? 4 : 0));
        ++launches;
      }
    for (int h = 1; h < nh; ++h) {
      hipEvent_t e = h == 1 ? ctx->evx : h == 2 ? ctx->evj : ctx->eva;
      SK_HIP(ctx, hipEventRecord(e, hs[h]));
      SK_HIP(ctx, hipStreamWaitEvent(S, e, 0));
    }
    SK_HIP(ctx, hipEventRecord(ctx->ev1, S));
    SK_HIP(ctx, hipStreamSynchronize(S));
    SK_HIP(ctx, sk::lev_collect(ctx));
    float ms = 0.f;
    SK_HIP(ctx, hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
    total_ms += ms;
    b0 = b1;
  }
  ctx->last_stem_ms = total_ms;
  ctx->last_launches = launches;
  return SK_OK;
}

// Core: out_dev[k] = K(xset[x[k]], yset[y[k]]) (device buffer), async.
int run_pairs(sk_context* ctx, sk_dataset* xs_, sk_dataset* ys_, const sk_kernel_params* kp,
              const int32_t* x, const int32_t* y, int64_t n, double* out_dev) {
  if (!ctx || !kp) return fail(ctx, SK_ERR_INVALID, "null argument");
  int rc = check_set(ctx, xs_);
  if (rc) return rc;
  rc = check_set(ctx, ys_);
  if (rc) return rc;
  if (n < 0) return fail(ctx, SK_ERR_INVALID, "negative pair count");
  if (kp->kind < SK_SU_STEM || kp->kind > SK_STEM4D)
    return fail(ctx, SK_ERR_UNSUPPORTED, "unknown kernel kind");
  ctx->last_stem_ms = ctx->last_str_ms = ctx->last_cells = 0.0;
  ctx->last_launches = 0;
  sk::lev_reset(ctx);
  ctx->last_stem_classes = ctx->last_s4d_classes = 0;
  if (n == 0) return SK_OK;
  const int nx = (int)xs_->ex.size(), ny = (int)ys_->ex.size();
  for (int64_t k = 0; k < n; ++k)
    if (x[k] < 0 || x[k] >= nx || y[k] < 0 || y[k] >= ny)
      return fail(ctx, SK_ERR_RANGE, "pair index out of range");
  SK_HIP(ctx, sk::call_begin(ctx));
  if (kind_is_bpla(kp->kind)) return run_bpla(ctx, xs_, ys_, kp, x, y, n, out_dev);
  if (kp->kind == SK_STEM4D) {
    // synchronous batches (each waits for its spans): its totals are final
    rc = run_stem4d(ctx, xs_, ys_, kp, x, y, n, out_dev);
    if (rc == SK_OK && ctx->async) {
      ctx->acc_stem_ms += ctx->last_stem_ms;
      ctx->acc_cells += ctx->last_cells;
      ctx->acc_launches += ctx->last_launches;
      ctx->acc_launch_ms += ctx->last_launch_ms_sum;
      ctx->acc_launch_n += ctx->last_launch_n;
    }
    return rc;
  }

  const bool stem = kind_has_stem(kp->kind), str = kind_has_str(kp->kind);
  const HostPack& PX = xs_->pack;
  const HostPack& PY = ys_->pack;
  // SK_HOST_STATS: host planning time per phase (diagnostic)
  const bool host_stats = std::getenv("SK_HOST_STATS") != nullptr;
  auto now_ms = [] {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
  };
  const double th0 = host_stats ? now_ms() : 0.0;
  double th1 = th0, th2 = th0;

  // ---- host-side work lists
  // stem items: pairs grouped by y, chunks, largest first, in classes by the
  // y example's register template (MAXK = 64-node slots per lane): one
  // launch per class, each sized (LDS, waves) for its own largest y
  struct StemClass {
    int maxk = 0;
    int max_nl = 0, max_edges = 0, max_bpf = 0, max_nch = 0;
    int nwaves = 1, grid = 1;
    size_t item_off = 0, n_items = 0;
  };
  std::vector<StemClass> classes;
  std::vector<int4> items;
  std::vector<int32_t> ixs;
  std::vector<int64_t> ioidx;
  std::vector<int32_t> big_x, big_y;  // pairs whose y goes to the big-y kernel
  std::vector<int64_t> big_o;
  int big_max_nl = 0;
  const int max_len = std::max(PX.max_len, PY.max_len);
  if (stem) {
    std::vector<int64_t> cnt(ny + 1, 0);
    for (int64_t k = 0; k < n; ++k) cnt[y[k] + 1]++;
    for (int j = 0; j < ny; ++j) cnt[j + 1] += cnt[j];
    std::vector<int64_t> byy(n);
    {
      std::vector<int64_t> pos(cnt.begin(), cnt.end() - 1);
      for (int64_t k = 0; k < n; ++k) byy[pos[y[k]]++] = k;
    }
    // within one y, costliest x first: the waves of a workgroup take the
    // item's pairs round-robin, so equal-cost rounds and a cheap last round
    // (one packed key per pair, ties by input order: deterministic)
    // (the y's on host threads: each sorts its own range of byy)
    {
      std::atomic<int> nextj{0};
      auto work = [&]() {
        std::vector<uint64_t> key;
        std::vector<int64_t> tmp;
        for (int j = nextj.fetch_add(1); j < ny; j = nextj.fetch_add(1)) {
          const int64_t b = cnt[j], e = cnt[j + 1];
          if (e - b < 2) continue;
          key.resize(e - b);
          for (int64_t t = b; t < e; ++t)
            key[t - b] = ((uint64_t)(0xffffffffu - (uint32_t)PX.ex_nl[x[byy[t]]]) << 32) | (uint32_t)(t - b);
          std::sort(key.begin(), key.end());
          tmp.assign(byy.begin() + b, byy.begin() + e);
          for (int64_t t = b; t < e; ++t) byy[t] = tmp[(uint32_t)key[t - b]];
        }
      };
      run_pool(plan_threads(n / 65536 + 1), work);
    }
    ixs.resize(n);
    ioidx.resize(n);
    for (int64_t t = 0; t < n; ++t) {
      ixs[t] = x[byy[t]];
      ioidx[t] = byy[t];
    }
    // y examples beyond the register classes (or forced there by the
    // diagnostic SK_FORCE_BIG_Y=1) go to sk_dag_stem_big_kernel
    const bool force_big = [] {
      const char* e = SK_KNOB("SK_FORCE_BIG_Y");
      return e && std::atoi(e) != 0;
    }();
    std::vector<uint8_t> ybig(ny, 0);
    for (int j = 0; j < ny; ++j) ybig[j] = force_big || PY.ex_big[j] ? 1 : 0;
    auto in_class = [&](int j, int maxk) {
      return !ybig[j] && sk::stem_maxk(PY.ex_nl[j] + 1) == maxk;  // (one slot free: dag_stem.hip zslot)
    };
    {
      std::vector<int64_t> bk;  // pairs dealt cyclically to the waves: costliest first
      for (int j = 0; j < ny; ++j) {
        if (!ybig[j] || cnt[j + 1] == cnt[j]) continue;
        big_max_nl = std::max(big_max_nl, PY.ex_nl[j]);
        for (int64_t t = cnt[j]; t < cnt[j + 1]; ++t) bk.push_back(byy[t]);
      }
      std::stable_sort(bk.begin(), bk.end(), [&](int64_t a, int64_t b) {
        return (double)PX.ex_nl[x[a]] * PY.ex_nl[y[a]] > (double)PX.ex_nl[x[b]] * PY.ex_nl[y[b]];
      });
      for (int64_t k : bk) {
        big_x.push_back(x[k]);
        big_y.push_back(y[k]);
        big_o.push_back(k);
      }
    }
    for (int maxk : {32, 28, 24, 20, 17, 16, 12, 8, 4}) {
      StemClass C;
      C.maxk = maxk;
      bool any = false;
      for (int j = 0; j < ny; ++j) {
        if (cnt[j + 1] == cnt[j] || !in_class(j, maxk)) continue;
        any = true;
        C.max_nl = std::max(C.max_nl, PY.ex_nl[j]);
        C.max_edges = std::max(C.max_edges, PY.ex_edge_base[j + 1] - PY.ex_edge_base[j]);
        C.max_bpf = std::max(C.max_bpf, PY.ex_bpf_base[j + 1] - PY.ex_bpf_base[j]);
        C.max_nch = std::max(C.max_nch, PY.ex_nch[j]);
      }
      if (!any) continue;
      sk::StemLaunch L;
      L.lds_max_nl = 64 * maxk;
      L.lds_max_edges = (C.max_edges + 3) & ~3;
      L.lds_max_bpf = (C.max_bpf + 1 + 3) & ~3;
      L.lds_max_nch = C.max_nch + 2;  // + 2 dummy chunks read past the end (dag_stem.hip)
      L.lds_max_len_pad = (max_len + 2 + 3) & ~3;
      L.n_gpow = max_len + 2;
      L.n_gpow_pad = (L.n_gpow + 1) & ~1;
      L.xset.n_gam = (int32_t)PX.gam_key.size();
      L.gam_on = L.xset.n_gam > 0;
      int max_dyn = 0, vgprs = 0, max_w = 8;
      SK_HIP(ctx, sk::stem_kernel_attr(L.lds_max_nl, &max_dyn, &vgprs, &max_w));
      const int valloc = ((std::max(vgprs, 1) + 7) / 8) * 8;
      const int waves_cu_vgpr = 4 * std::min(8, 512 / valloc);
      int best = 0, per_cu = 1;
      for (int w = max_w; w >= 1; --w) {  // the template's __launch_bounds__
        const size_t lds = sk::stem_lds_bytes(L, w);
        if (lds > (size_t)max_dyn) continue;
        const int pc = std::min<int>((int)(163840 / lds), std::min(32, waves_cu_vgpr) / w);
        if (pc * w > best) {
          best = pc * w;
          C.nwaves = w;
          per_cu = pc;
        }
      }
      if (best == 0) return fail(ctx, SK_ERR_UNSUPPORTED, "y example too large for LDS");
#ifdef SK_STAMPS
      // diagnostics: SK_FORCE_WAVES=w,p -> w waves per workgroup, p workgroups per CU
      if (const char* fw = SK_KNOB("SK_FORCE_WAVES")) {
        int w = 0, pc = 0;
        if (std::sscanf(fw, "%d,%d", &w, &pc) == 2 && w >= 1 && w <= C.nwaves && pc >= 1) {
          C.nwaves = w;
          per_cu = pc;
        }
      }
#endif
      C.grid = ctx->n_cu * per_cu;
      // Work items = pairs of one y (the workgroup stages one y DAG in LDS
      // and waits for its slowest wave at every item boundary, about half a
      // pair per wave).  Guided self-scheduling: the y's are taken largest
      // column first and each item is 1/(K * grid) of the class's remaining
      // cost (at least one round of W pairs), so the first items are large
      // (few boundaries) and the last ones a round each (short launch tail).
      // Items are pulled in this order (K = 1.5; NS 161k pairs/s at K = 1,
      // 160.8k at 1.5, 160.0k at 2, 157.2k at 8; C2 148k at 1.5, 140k at 1).
      std::vector<int> ysel;
      double class_cost = 0.0;
      for (int j = 0; j < ny; ++j) {
        if (cnt[j + 1] == cnt[j] || !in_class(j, maxk)) continue;
        ysel.push_back(j);
        for (int64_t t = cnt[j]; t < cnt[j + 1]; ++t)
          class_cost += (double)PX.ex_nl[x[byy[t]]] * (double)PY.ex_nl[j];
      }
      std::stable_sort(ysel.begin(), ysel.end(), [&](int a, int b) {
        return cnt[a + 1] - cnt[a] > cnt[b + 1] - cnt[b];
      });
      double gss_k = 1.5;  // tuning knob: SK_GSS_K (items per workgroup at the start)
      if (const char* e = SK_KNOB("SK_GSS_K")) gss_k = std::max(0.25, std::atof(e));
      const double share = 1.0 / (gss_k * (double)C.grid);
      double remaining = class_cost;
      C.item_off = items.size();
      for (int j : ysel) {
        const double yw = (double)PY.ex_nl[j];
        int64_t b = cnt[j];
        while (b < cnt[j + 1]) {
          const double target = remaining * share;
          int64_t e = b;
          double cost = 0.0;
          // whole rounds of W pairs until the target cost is reached
          while (e < cnt[j + 1] && (e - b < C.nwaves || cost < target)) {
            const int64_t re = std::min<int64_t>(cnt[j + 1], e + C.nwaves);
            for (int64_t t = e; t < re; ++t) cost += (double)PX.ex_nl[x[byy[t]]] * yw;
            e = re;
          }
          items.push_back(make_int4(j, (int)b, (int)(e - b), 0));
          remaining -= cost;
          b = e;
        }
      }
      C.n_items = items.size() - C.item_off;
      C.grid = (int)std::min<int64_t>(C.grid, std::max<int64_t>(1, (int64_t)C.n_items));
      classes.push_back(C);
    }
    double cells = 0.0;
    for (int64_t k = 0; k < n; ++k) cells += (double)PX.ex_nl[x[k]] * (double)PY.ex_nl[y[k]];
    ctx->last_cells = cells;
  }

  if (host_stats) th1 = now_ms();
  // the items' phi keys (the union over their x's; gapless y only), for the
  // workgroups' Phi tables (dag_stem.hip)
  std::vector<int32_t> item_phi_off, item_phi;
  const bool phi_on = stem && !PX.phi_al.empty() && !PX.gam_key.empty();
  if (phi_on) {
    // union of the x's key bitsets, keys ordered by gamma key (the kernel
    // forms one H row per gamma key and wave)
    // (contiguous item ranges on host threads, concatenated in item order)
    const size_t W = (PX.phi_al.size() + 63) / 64;
    const size_t ni = items.size();
    const int T = plan_threads((int)(ni / 512 + 1));
    std::vector<std::vector<int32_t>> tkeys(T), tcnt(T);
    run_slices(T, [&](int t) {
      std::vector<uint64_t> acc(W);
      for (size_t i = ni * t / T; i < ni * (t + 1) / T; ++i) {
        const int4 it = items[i];
        const size_t k0 = tkeys[t].size();
        if (PY.ex_gapless[it.x]) {
          std::fill(acc.begin(), acc.end(), 0ull);
          for (int u = it.y; u < it.y + it.z; ++u) {
            const uint64_t* b = PX.ex_phi_bits.data() + (size_t)ixs[u] * W;
            for (size_t w = 0; w < W; ++w) acc[w] |= b[w];
          }
          // (phi keys are numbered in gamma key order: the bits come sorted)
          for (size_t w = 0; w < W; ++w)
            for (uint64_t m = acc[w]; m; m &= m - 1) tkeys[t].push_back((int32_t)(w * 64 + __builtin_ctzll(m)));
        }
        tcnt[t].push_back((int32_t)(tkeys[t].size() - k0));
      }
    });
    item_phi_off.assign(1, 0);
    for (int t = 0; t < T; ++t) {
      item_phi.insert(item_phi.end(), tkeys[t].begin(), tkeys[t].end());
      for (int32_t c : tcnt[t]) item_phi_off.push_back(item_phi_off.back() + c);
    }
    if (std::getenv("SK_PHI_STATS"))
      std::fprintf(stderr, "[phi] keys=%zu items=%zu item keys=%zu pairs=%lld phi components=%zu rows=%zu\n",
                   PX.phi_al.size(), items.size(), item_phi.size(), (long long)n, PX.phk_idx.size(),
                   PX.xgrow.size());
  }

  if (host_stats) th2 = now_ms();
  // string kernel: pairs of dyadic, never-empty profiles (both weighted or
  // neither) take the fast path (profile_string.hip), first; the rest the
  // general kernel, the permutation undone through oidx
  // (one-hot pairs first, then the other fast pairs, then the rest)
  std::vector<int32_t> spx, spy;
  std::vector<int64_t> soidx;
  int64_t n_soh = 0, n_sfast = 0;  // one-hot pairs; fast pairs (one-hot included)
  // (the fast kernels' per-wave LDS rows must fit a CU: else the general one)
  const int str_lds_len = (std::max(PY.max_len, 64) + 1) & ~1;
  if (str && kp->kind != SK_NAIVE_STR && !SK_KNOB("SK_STR_GENERAL") &&
      sk::str_fast_wave_lds_bytes(str_lds_len, false) + sk::kStrFastLds0 <= 163840) {
    auto cat = [&](int64_t k) {
      const int a = x[k], b = y[k];
      if (PX.ex_has_w[a] != PY.ex_has_w[b]) return 2;
      if (PX.ex_onehot[a] && PY.ex_onehot[b]) return 0;
      return PX.ex_str_fast[a] && PY.ex_str_fast[b] ? 1 : 2;
    };
    int64_t cnt3[3] = {0, 0, 0};
    for (int64_t k = 0; k < n; ++k) ++cnt3[cat(k)];
    n_soh = cnt3[0];
    n_sfast = cnt3[0] + cnt3[1];
    if (cnt3[0] != n && cnt3[1] != n && cnt3[2] != n) {
      spx.reserve(n);
      spy.reserve(n);
      soidx.reserve(n);
      for (int c = 0; c < 3; ++c)
        for (int64_t k = 0; k < n; ++k)
          if (cat(k) == c) {
            spx.push_back(x[k]);
            spy.push_back(y[k]);
            soidx.push_back(k);
          }
    }
  }
  const size_t n_str_pos = n_sfast ? PX.pos_prof.size() + (ys_ == xs_ ? 0 : PY.pos_prof.size()) : 0;

  // ---- device work arena
  const size_t nb = (size_t)n;
  size_t need = 0;
  need += soidx.size() * 8 + n_str_pos * (2 * sizeof(sk::StrPos) + sizeof(sk::StrCode)) + 1024;
  need += (item_phi_off.size() + item_phi.size()) * 4 + 512;
  need += 256 * 8 + 16 * 8 + (size_t)(max_len + 4) * 8 * 2;
  need += 1024;
  need += items.size() * sizeof(int4) + nb * (4 + 8) + nb * 8 * 2 + nb * 4 * 2 + 64 + 8 * 256;
  need += big_x.size() * (4 + 4 + 8) + 3 * 256;
  need += 16 * 256;
  rc = ensure_work(ctx, need);
  if (rc) return rc;
  Arena A{static_cast<char*>(ctx->work), 0, ctx->work_bytes};
  double* d_co = A.take<double>(256);
  double* d_gp_loop = A.take<double>(max_len + 4);
  double* d_st = A.take<double>(16);
  double* d_gp_str = A.take<double>(max_len + 4);
  int4* d_items = A.take<int4>(std::max<size_t>(items.size(), 1));
  int32_t* d_ixs = A.take<int32_t>(std::max<size_t>(nb, 1));
  int64_t* d_oidx = A.take<int64_t>(std::max<size_t>(nb, 1));
  double* d_stem = A.take<double>(nb);
  double* d_str = A.take<double>(nb);
  int32_t* d_px = A.take<int32_t>(nb);
  int32_t* d_py = A.take<int32_t>(nb);
  int* d_ctr = A.take<int>(64);
  int32_t* d_bx = A.take<int32_t>(std::max<size_t>(big_x.size(), 1));
  int32_t* d_by = A.take<int32_t>(std::max<size_t>(big_x.size(), 1));
  int64_t* d_bo = A.take<int64_t>(std::max<size_t>(big_x.size(), 1));
  int32_t* d_iphi_off = A.take<int32_t>(std::max<size_t>(item_phi_off.size(), 1));
  int32_t* d_iphi = A.take<int32_t>(std::max<size_t>(item_phi.size(), 1));
  int64_t* d_soidx = soidx.empty() ? nullptr : A.take<int64_t>(soidx.size());
  sk::StrPos* d_stab = (n_sfast > n_soh) ? A.take<sk::StrPos>(2 * n_str_pos) : nullptr;
  sk::StrCode* d_ctab = n_soh ? A.take<sk::StrCode>(n_str_pos) : nullptr;

  // parameter tables
  std::vector<double> co(256), st(16);
  const bool subst = kind_subst(kp->kind);
  for (int k = 0; k < 256; ++k)
    co[k] = subst ? std::exp(SK_RIBOSUM_P[k] * kp->beta)
                  : ((k >> 4) == (k & 15) ? kp->stack : kp->covar);
  for (int k = 0; k < 16; ++k)
    st[k] = subst ? std::exp(SK_RIBOSUM_S[k] * kp->alpha)
                  : ((k >> 2) == (k & 3) ? kp->match : kp->mismatch);
  const std::vector<double> gl = gap_powers(kp->loop_gap, max_len + 4);
  const std::vector<double> gs = gap_powers(kp->gap, max_len + 4);
  hipStream_t S = ctx->stream;
  SK_HIP(ctx, sk::h2d(ctx, d_co, co.data(), 256 * 8, S));
  SK_HIP(ctx, sk::h2d(ctx, d_st, st.data(), 16 * 8, S));
  SK_HIP(ctx, sk::h2d(ctx, d_gp_loop, gl.data(), gl.size() * 8, S));
  SK_HIP(ctx, sk::h2d(ctx, d_gp_str, gs.data(), gs.size() * 8, S));
  SK_HIP(ctx, hipMemsetAsync(d_ctr, 0, 64 * sizeof(int), S));

  double* stem_out = (combine_mode(kp->kind) == sk::kCombineStem) ? out_dev : d_stem;
  double* str_out = (combine_mode(kp->kind) == sk::kCombineStr) ? out_dev : d_str;

  // string kernel inputs first: with a stem part it forks to the side stream
  // here, ahead of the stem launches
  const bool side = stem && str;
  if (str) {
    SK_HIP(ctx, sk::h2d(ctx, d_px, spx.empty() ? x : spx.data(), nb * 4, S));
    SK_HIP(ctx, sk::h2d(ctx, d_py, spy.empty() ? y : spy.data(), nb * 4, S));
    if (d_soidx)
      SK_HIP(ctx, sk::h2d(ctx, d_soidx, soidx.data(), soidx.size() * 8, S));
    if (side) {
      SK_HIP(ctx, hipEventRecord(ctx->evf, S));
      SK_HIP(ctx, hipStreamWaitEvent(ctx->side, ctx->evf, 0));
    }
  }
  if (stem) {
    SK_HIP(ctx, sk::h2d(ctx, d_items, items.data(), items.size() * sizeof(int4), S));
    SK_HIP(ctx, sk::h2d(ctx, d_ixs, ixs.data(), nb * 4, S));
    SK_HIP(ctx, sk::h2d(ctx, d_oidx, ioidx.data(), nb * 8, S));
    if (phi_on) {
      SK_HIP(ctx, sk::h2d(ctx, d_iphi_off, item_phi_off.data(), item_phi_off.size() * 4, S));
      if (!item_phi.empty())
        SK_HIP(ctx, sk::h2d(ctx, d_iphi, item_phi.data(), item_phi.size() * 4, S));
    }
    const double gap2 = kp->loop_gap * kp->loop_gap;
    const size_t nnd = std::max<size_t>(PX.nd_a.size(), 1);
    const size_t nxc = std::max<size_t>(PX.xr_ch.size(), 1), nxg = std::max<size_t>(PX.xgrow.size(), 1),
                 nxgc = std::max<size_t>(PX.xg_ch.size(), 1),
                 ngh = std::max<size_t>(PX.ex_nl.size() * PX.gam_key.size(), 1),
                 nphk = std::max<size_t>(PX.phk_idx.size(), 1);
    if (!xs_->prep) {
      void* p = nullptr;
      SK_HIP(ctx, hipMalloc(&p, (3 * nnd + nxc + nxg + nxgc + ngh + nphk) * sizeof(double)));
      xs_->prep = static_cast<double*>(p);
      xs_->buf.ptrs.push_back(p);
      xs_->prep_loop_gap = -1.0;
    }
    sk::DevParamNodes pn;
    pn.nd_L = xs_->prep;
    pn.nd_SL = xs_->prep + nnd;
    pn.xr_SL = xs_->prep + 2 * nnd;
    pn.xr_chw = xs_->prep + 3 * nnd;
    pn.xg_SL = pn.xr_chw + nxc;
    pn.xg_chw = pn.xg_SL + nxg;
    pn.gam_h = pn.xg_chw + nxgc;
    pn.phk_w = pn.gam_h + ngh;
    if (!(xs_->prep_loop_gap == kp->loop_gap)) {  // once per dataset and loop_gap
      SK_HIP(ctx, sk::launch_prep(xs_->dev, pn, d_gp_loop, gap2, S));
      xs_->prep_loop_gap = kp->loop_gap;
    }
    // class c runs on the main stream (c even) or the class stream (c odd):
    // one scratch region per stream, serving its classes in turn
    const bool two_streams = classes.size() > 1 && !SK_KNOB("SK_SERIAL_CLASSES");
    size_t scratch_need = 0, scratch_x = 0;
    for (size_t c = 0; c < classes.size(); ++c) {
      const StemClass& C = classes[c];
      // + one junk row: root rows are stored there (never read)
      const int64_t slab = (int64_t)(PX.max_slots + 1) * 64 * C.maxk;
      // + the workgroups' Gamma tables
      const int64_t gtab = (int64_t)PX.gam_key.size() * 64 * C.maxk;
      // + their Phi tables and sums
      const int64_t ptab = phi_on ? (int64_t)PX.phi_al.size() * (64 * C.maxk + 1) : 0;
      const size_t b = (size_t)C.grid * (C.nwaves * slab + gtab + ptab) * sizeof(double);
      size_t& r = (two_streams && (c & 1)) ? scratch_x : scratch_need;
      r = std::max(r, b);
    }
    // big-y kernel: per wave S, G1 and the G0 slots, rows of `big_stride`
    // doubles; as many waves as pairs, the grid, and a scratch budget allow
    const int64_t big_stride = ((int64_t)std::max(big_max_nl, 1) + 63) / 64 * 64;
    const int64_t big_wave = (int64_t)(PX.max_slots + 2) * big_stride;
    int big_grid = 0;
    if (!big_x.empty()) {
      size_t free_b = 0, total_b = 0;
      SK_HIP(ctx, hipMemGetInfo(&free_b, &total_b));
      const size_t budget = std::max<size_t>(std::min<size_t>(free_b / 2, (size_t)32 << 30),
                                             (size_t)big_wave * 8 * sk::kStemBigWaves);
      const int64_t by_mem = (int64_t)(budget / ((size_t)big_wave * 8 * sk::kStemBigWaves));
      const int64_t by_pairs = ((int64_t)big_x.size() + sk::kStemBigWaves - 1) / sk::kStemBigWaves;
      big_grid = (int)std::max<int64_t>(1, std::min<int64_t>({by_mem, by_pairs, (int64_t)ctx->n_cu * 8}));
      scratch_need = std::max(scratch_need,
                              (size_t)big_grid * sk::kStemBigWaves * (size_t)big_wave * sizeof(double));
    }
    scratch_need = (scratch_need + 255) / 256 * 256;
    rc = ensure_scratch(ctx, std::max<size_t>(scratch_need + scratch_x, 64));
    if (rc) return rc;
    double* scratch_cls = ctx->scratch + scratch_need / sizeof(double);
#ifdef SK_STAMPS
    unsigned long long* d_stamps = nullptr;
    SK_HIP(ctx, hipMalloc(&d_stamps, 16 * sizeof(unsigned long long)));
    SK_HIP(ctx, hipMemsetAsync(d_stamps, 0, 16 * sizeof(unsigned long long), S));
#endif
    if (host_stats)
      std::fprintf(stderr, "[host] pairs=%lld plan %.2f ms, phi keys %.2f ms, uploads+prep %.2f ms\n",
                   (long long)n, th1 - th0, th2 - th1, now_ms() - th2);
    SK_HIP(ctx, hipEventRecord(ctx->ev0, S));
    if (two_streams) {
      SK_HIP(ctx, hipEventRecord(ctx->evk, S));
      SK_HIP(ctx, hipStreamWaitEvent(ctx->cls, ctx->evk, 0));
    }
    for (size_t c = 0; c < classes.size(); ++c) {
      const StemClass& C = classes[c];
      const bool on_cls = two_streams && (c & 1);
      sk::StemLaunch SL;
      SL.xset = xs_->dev;
      SL.yset = ys_->dev;
      SL.pn = pn;
      SL.co_subst = d_co;
      SL.gpow = d_gp_loop;
      SL.n_gpow = max_len + 2;
      SL.n_gpow_pad = (SL.n_gpow + 1) & ~1;
      SL.gap2 = gap2;
      SL.band = kp->len_band;
      SL.lds_max_nl = 64 * C.maxk;
      SL.lds_max_edges = (C.max_edges + 3) & ~3;
      SL.lds_max_bpf = (C.max_bpf + 1 + 3) & ~3;
      SL.lds_max_nch = C.max_nch + 2;  // + 2 dummy chunks read past the end (dag_stem.hip)
      SL.lds_max_len_pad = (max_len + 2 + 3) & ~3;
      SL.items = d_items + C.item_off;
      SL.n_items = (int32_t)C.n_items;
      SL.xs = d_ixs;
      SL.oidx = d_oidx;
      SL.out = stem_out;
      SL.item_counter = d_ctr + 16 + (int)c;
      SL.slab_doubles = (int64_t)(PX.max_slots + 1) * SL.lds_max_nl;
      SL.scratch = on_cls ? scratch_cls : ctx->scratch;
      SL.gam_on = !PX.gam_key.empty();
      SL.gam_doubles = (int64_t)PX.gam_key.size() * SL.lds_max_nl;
      SL.gam = SL.scratch + (size_t)C.grid * C.nwaves * SL.slab_doubles;
      SL.phi_on = phi_on ? 1 : 0;
      SL.phi_doubles = phi_on ? (int64_t)PX.phi_al.size() * (SL.lds_max_nl + 1) : 0;
      SL.phi = SL.gam + (size_t)C.grid * SL.gam_doubles;
      SL.item_phi_off = d_iphi_off + C.item_off;
      SL.item_phi = d_iphi;
#ifdef SK_STAMPS
      SL.stamps = d_stamps;
#endif
      SK_HIP(ctx, sk::lev_mark(ctx, on_cls ? ctx->cls : S));
      SK_HIP(ctx, sk::launch_stem(SL, C.grid, C.nwaves, on_cls ? ctx->cls : S));
      SK_HIP(ctx, sk::lev_mark(ctx, on_cls ? ctx->cls : S));
      ctx->last_stem_classes |= 1u << (C.maxk % 4 ? C.maxk : C.maxk / 4);  // (MAXK 17: bit 17)
    }
    if (two_streams) {
      SK_HIP(ctx, hipEventRecord(ctx->evx, ctx->cls));
      SK_HIP(ctx, hipStreamWaitEvent(S, ctx->evx, 0));
    }
    if (!big_x.empty()) {
      const size_t nbig = big_x.size();
      SK_HIP(ctx, sk::h2d(ctx, d_bx, big_x.data(), nbig * 4, S));
      SK_HIP(ctx, sk::h2d(ctx, d_by, big_y.data(), nbig * 4, S));
      SK_HIP(ctx, sk::h2d(ctx, d_bo, big_o.data(), nbig * 8, S));
      sk::StemBigLaunch BL;
      BL.xset = xs_->dev;
      BL.yset = ys_->dev;
      BL.pn = pn;
      BL.co_subst = d_co;
      BL.gpow = d_gp_loop;
      BL.n_gpow = max_len + 2;
      BL.gap2 = gap2;
      BL.band = kp->len_band;
      BL.xs = d_bx;
      BL.ys = d_by;
      BL.oidx = d_bo;
      BL.n_pairs = (int64_t)nbig;
      BL.out = stem_out;
      BL.scratch = ctx->scratch;
      BL.stride = big_stride;
      BL.wave_doubles = big_wave;
      SK_HIP(ctx, sk::lev_mark(ctx, S));
      SK_HIP(ctx, sk::launch_stem_big(BL, big_grid, S));
      SK_HIP(ctx, sk::lev_mark(ctx, S));
      ctx->last_stem_classes |= 1u;
    }
    SK_HIP(ctx, hipEventRecord(ctx->ev1, S));
#ifdef SK_STAMPS
    {
      unsigned long long h[16];
      SK_HIP(ctx, hipMemcpyAsync(h, d_stamps, sizeof(h), hipMemcpyDeviceToHost, S));
      SK_HIP(ctx, hipStreamSynchronize(S));
      (void)hipFree(d_stamps);
      const double rows = (double)h[8];
      std::fprintf(stderr, "[stamps] classes=%zu pairs=%llu rows=%.0f cycles/row:", classes.size(),
                   h[9], rows);
      const char* nm[7] = {"hdr", "A", "Rfill", "passes", "zero", "sweep", "store"};
      for (int i = 0; i < 7; ++i) std::fprintf(stderr, " %s=%.0f", nm[i], h[i] / rows);
      std::fprintf(stderr, "\n[stamps] per row: A-loaded rows=%.3f swept chunks=%.2f match passes=%.2f band nodes=%.1f\n",
                   h[10] / rows, h[11] / rows, h[12] / rows, h[13] / rows);
      for (const StemClass& C : classes)
        std::fprintf(stderr, "[stamps] class maxk=%d max_nl=%d max_edges=%d max_nch=%d waves/wg=%d grid=%d items=%zu\n",
                     C.maxk, C.max_nl, C.max_edges, C.max_nch, C.nwaves, C.grid, C.n_items);
    }
#endif
    ctx->last_launches = (int32_t)classes.size() + (big_x.empty() ? 0 : 1);
  }
  if (str) {
    const hipStream_t SS = side ? ctx->side : S;
    sk::StrLaunch T;
    T.xset = xs_->dev;
    T.yset = ys_->dev;
    T.st = d_st;
    T.gpow = d_gp_str;
    T.gap = kp->gap;
    T.naive = kp->kind == SK_NAIVE_STR ? 1 : 0;
    T.xs = d_px + n_sfast;
    T.ys = d_py + n_sfast;
    T.oidx = d_soidx ? d_soidx + n_sfast : nullptr;
    T.n_pairs = n - n_sfast;
    T.out = str_out;
    T.pair_counter = reinterpret_cast<unsigned long long*>(d_ctr + 8);
    T.lds_max_len = (std::max(PY.max_len, 1) + 1) & ~1;
    // 4 waves per workgroup while their rows fit 64 KB of LDS, fewer for
    // longer y (one wave's rows fit the CU's 160 KB up to L ~ 4,000)
    int w = 4;
    while (w > 1 && sk::str_lds_bytes(T, w) > 65536) w /= 2;
    const size_t lds = sk::str_lds_bytes(T, w);
    if (lds > 163840) return fail(ctx, SK_ERR_UNSUPPORTED, "sequence too long for string kernel LDS");
    const int per_cu = std::max(1, std::min<int>((int)(163840 / lds), 8));
    const int64_t g = std::max<int64_t>(1, std::min<int64_t>((int64_t)ctx->n_cu * per_cu, (n - n_sfast + w - 1) / w));
    SK_HIP(ctx, hipEventRecord(ctx->ev2, SS));
    for (int oh = 1; oh >= 0; --oh) {
      const int64_t b = oh ? 0 : n_soh, e = oh ? n_soh : n_sfast;
      if (e <= b) continue;
      const size_t npx = PX.pos_prof.size(), npy = PY.pos_prof.size();
      const void *tx, *ty;
      if (oh) {  // [npx] x set | [npy] y set
        SK_HIP(ctx, sk::launch_str_code_tab(xs_->dev.pos_prof, xs_->dev.pos_w, (int64_t)npx, d_ctab, SS));
        if (ys_ != xs_)
          SK_HIP(ctx, sk::launch_str_code_tab(ys_->dev.pos_prof, ys_->dev.pos_w, (int64_t)npy, d_ctab + npx, SS));
        tx = d_ctab;
        ty = ys_ != xs_ ? d_ctab + npx : d_ctab;
      } else {   // [npx] x role | [npx] y role (| [npy] x role, unused | [npy] y role)
        SK_HIP(ctx, sk::launch_str_tab(xs_->dev.pos_prof, xs_->dev.pos_w, (int64_t)npx, d_st, d_stab,
                                       d_stab + npx, SS));
        tx = d_stab;
        ty = d_stab + npx;
        if (ys_ != xs_) {
          SK_HIP(ctx, sk::launch_str_tab(ys_->dev.pos_prof, ys_->dev.pos_w, (int64_t)npy, d_st, d_stab + 2 * npx,
                                         d_stab + 2 * npx + npy, SS));
          ty = d_stab + 2 * npx + npy;
        }
      }
      sk::StrFastLaunch F;
      F.xset = xs_->dev;
      F.yset = ys_->dev;
      F.xtab = static_cast<const sk::StrPos*>(tx);
      F.ytab = static_cast<const sk::StrPos*>(ty);
      F.st = d_st;
      F.onehot = oh;
      F.gpow = d_gp_str;
      F.gap = kp->gap;
      F.xs = d_px + b;
      F.ys = d_py + b;
      F.oidx = d_soidx ? d_soidx + b : nullptr;
      F.n_pairs = e - b;
      F.out = str_out;
      F.lds_max_len = (std::max(PY.max_len, 64) + 1) & ~1;
      const size_t wl = sk::str_fast_wave_lds_bytes(F.lds_max_len, oh != 0);
      if (wl + sk::kStrFastLds0 > 163840) return fail(ctx, SK_ERR_UNSUPPORTED, "sequence too long for string kernel LDS");
      const int per_cu_w = (int)std::max<size_t>(1, std::min<size_t>(16, (163840 - sk::kStrFastLds0) / wl));
      const int fw = std::min(4, per_cu_w);
      const int64_t fg = std::min<int64_t>((int64_t)ctx->n_cu * std::max(1, per_cu_w / fw), (e - b + fw - 1) / fw);
      SK_HIP(ctx, sk::launch_str_fast(F, (int)fg, fw, SS));
    }
    if (n_sfast < n) SK_HIP(ctx, sk::launch_str(T, (int)g, w, SS));
    SK_HIP(ctx, hipEventRecord(ctx->ev3, SS));
    if (side) {  // join before the combine
      SK_HIP(ctx, hipEventRecord(ctx->evj, ctx->side));
      SK_HIP(ctx, hipStreamWaitEvent(S, ctx->evj, 0));
    }
  }
  const int32_t mode = combine_mode(kp->kind);
  if (mode != sk::kCombineStem && mode != sk::kCombineStr)
    SK_HIP(ctx, sk::launch_combine(d_stem, d_str, out_dev, n, mode, kp->alpha, kp->beta, S));
  // timings: now (synchronous calls), or when sk_sync_timing asks (async)
  SK_HIP(ctx, sk::call_finish(ctx, S, stem, str));
  return SK_OK;
}

// BPLAKernel::compute_gradients over pairs (the bpla_optimizer's per-pair
// step, bpla_kernel.cpp:385-401, bpla_optimizer.cpp:52-255): batches bounded
// by scratch memory, one thread per pair.
int bpla_gradients(sk_context* ctx, sk_dataset* xs_, sk_dataset* ys_, const sk_kernel_params* kp,
                   const int32_t* x, const int32_t* y, int64_t n, double* value, double* grad) {
  if (!ctx || !xs_ || !ys_ || !kp || (n > 0 && (!x || !y || !value || !grad)))
    return fail(ctx, SK_ERR_INVALID, "null argument");
  int rc = check_set(ctx, xs_);
  if (rc) return rc;
  rc = check_set(ctx, ys_);
  if (rc) return rc;
  if (n <= 0) return n < 0 ? fail(ctx, SK_ERR_INVALID, "negative pair count") : SK_OK;
  SK_HIP(ctx, sk::call_begin(ctx));  // (synchronous: a fresh timing set, not a pending one)
  for (int64_t k = 0; k < n; ++k) {
    if (x[k] < 0 || x[k] >= (int)xs_->ex.size() || y[k] < 0 || y[k] >= (int)ys_->ex.size())
      return fail(ctx, SK_ERR_INVALID, "pair index out of range");
    if (!xs_->ex[x[k]].has_bp || !ys_->ex[y[k]].has_bp)
      return fail(ctx, SK_ERR_INVALID, "BPLA gradients need examples built with use_bp");
  }
  size_t free_b = 0, total_b = 0;
  SK_HIP(ctx, hipMemGetInfo(&free_b, &total_b));
  // one thread per pair, latency-bound: throughput grows with the pairs in
  // flight, so batches take most of the HBM
  const double budget = std::min(96e9, 0.6 * (double)free_b);
  rc = ensure_work(ctx, 16 * 8 + 4096);
  if (rc) return rc;
  double* d_tb = static_cast<double*>(ctx->work);
  hipStream_t S = ctx->stream;
  SK_HIP(ctx, hipMemcpyAsync(d_tb, kp->score_table, 16 * 8, hipMemcpyHostToDevice, S));
  // freed on every return path (an early SK_HIP return inside an optimizer
  // loop would otherwise leak both on each failing call)
  struct DevBuf {
    void* p = nullptr;
    ~DevBuf() {
      if (p) (void)hipFree(p);
    }
  } xy_buf, out_buf;
  SK_HIP(ctx, hipMalloc(&xy_buf.p, (size_t)2 * n * sizeof(int32_t)));
  SK_HIP(ctx, hipMalloc(&out_buf.p, (size_t)10 * n * sizeof(double)));
  int32_t* d_xy = static_cast<int32_t*>(xy_buf.p);
  double* d_out = static_cast<double*>(out_buf.p);
  SK_HIP(ctx, hipMemcpyAsync(d_xy, x, (size_t)n * 4, hipMemcpyHostToDevice, S));
  SK_HIP(ctx, hipMemcpyAsync(d_xy + n, y, (size_t)n * 4, hipMemcpyHostToDevice, S));
  double total_ms = 0.0;
  // pairs whose profiles are all dyadic take the wave-per-pair kernel (the
  // BPLA fast path's operand tables); the rest the thread-per-pair one
  const HostPack& PX = xs_->pack;
  const HostPack& PY = ys_->pack;
  std::vector<int32_t> wx, wy, gx, gy;
  std::vector<int64_t> wo, go;
  const bool general_only = SK_KNOB("SK_BPLA_GENERAL") != nullptr;  // A/B switch
  for (int64_t k = 0; k < n; ++k) {
    if (!general_only && PX.ex_dyadic[x[k]] && PY.ex_dyadic[y[k]]) {
      wx.push_back(x[k]);
      wy.push_back(y[k]);
      wo.push_back(k);
    } else {
      gx.push_back(x[k]);
      gy.push_back(y[k]);
      go.push_back(k);
    }
  }
  if (!wx.empty()) {
    const size_t nw = wx.size();
    const size_t npx = PX.pos_prof.size(), npy = ys_ == xs_ ? 0 : PY.pos_prof.size();
    const size_t ntab = 2 * (npx + npy);
    int tmax = 1, maxlen = 64;
    for (size_t k = 0; k < nw; ++k) {
      tmax = std::max(tmax, sk::bpla_steps(xs_->ex[wx[k]].len, ys_->ex[wy[k]].len));
      maxlen = std::max(maxlen, ys_->ex[wy[k]].len);
    }
    maxlen = (maxlen + 1) & ~1;
    const size_t wl = sk::bpla_grad_wave_lds_bytes(maxlen);
    if (wl + sk::kBplaExpLds > 163840)
      return fail(ctx, SK_ERR_UNSUPPORTED, "sequence too long for the BPLA gradient kernel LDS");
    const int per_cu_w = (int)std::max<size_t>(1, std::min<size_t>(16, (163840 - 2 * sk::kBplaExpLds) / wl));
    const int wpb = std::min(4, per_cu_w);
    const int64_t bt = (int64_t)3 * 64 * tmax;
    int64_t grid = (int64_t)ctx->n_cu * std::max(1, per_cu_w / wpb);
    grid = std::min<int64_t>(grid, std::max<int64_t>(1, ((int64_t)nw + wpb - 1) / wpb));
    grid = std::min<int64_t>(grid, std::max<int64_t>(1, (int64_t)(budget / (8.0 * bt * wpb))));
    DevBuf tab_buf, idx_buf;
    SK_HIP(ctx, hipMalloc(&tab_buf.p, ntab * sizeof(sk::BplaPos) + 64));
    SK_HIP(ctx, hipMalloc(&idx_buf.p, nw * (4 + 4 + 8) + 64));
    int32_t* d_wx = static_cast<int32_t*>(idx_buf.p);
    int32_t* d_wy = d_wx + nw;
    int64_t* d_wo = reinterpret_cast<int64_t*>(static_cast<char*>(idx_buf.p) + ((nw * 8 + 15) & ~size_t(15)));
    unsigned long long* d_cnt = reinterpret_cast<unsigned long long*>(d_tb + 16);  // after the table (work arena)
    SK_HIP(ctx, hipMemcpyAsync(d_wx, wx.data(), nw * 4, hipMemcpyHostToDevice, S));
    SK_HIP(ctx, hipMemcpyAsync(d_wy, wy.data(), nw * 4, hipMemcpyHostToDevice, S));
    SK_HIP(ctx, hipMemcpyAsync(d_wo, wo.data(), nw * 8, hipMemcpyHostToDevice, S));
    SK_HIP(ctx, hipMemsetAsync(d_cnt, 0, 8, S));
    sk::BplaPos* tabs = static_cast<sk::BplaPos*>(tab_buf.p);
    sk::BplaPos* tx = tabs;  // [npx] x role | [npx] y role (| [npy] x role | [npy] y role)
    sk::BplaPos* ty = tabs + npx;
    SK_HIP(ctx, sk::launch_bpla_tab(xs_->dev.pos_prof, xs_->dev.pos_lru, (int64_t)npx, d_tb, 1.0, tx,
                                    tabs + npx, S));
    if (npy) {
      ty = tabs + 2 * npx + npy;
      SK_HIP(ctx, sk::launch_bpla_tab(ys_->dev.pos_prof, ys_->dev.pos_lru, (int64_t)npy, d_tb, 1.0,
                                      tabs + 2 * npx, ty, S));
    }
    rc = ensure_scratch(ctx, (size_t)grid * wpb * (size_t)bt * 8 + 64);
    if (rc) return rc;
    sk::BplaGradLaunch W;
    W.xset = xs_->dev;
    W.yset = ys_->dev;
    W.table = d_tb;
    W.alpha = kp->alpha;
    W.beta = kp->beta;
    W.gap = kp->gap;
    W.ext = kp->ext;
    W.beta_gap = std::exp(kp->beta * kp->gap);  // bpla_kernel.cpp:188-189
    W.beta_ext = std::exp(kp->beta * kp->ext);
    W.xs = d_wx;
    W.ys = d_wy;
    W.n_pairs = (int64_t)nw;
    W.scratch = ctx->scratch;
    W.value = d_out;
    W.grad = d_out + n;
    W.xtab = tx;
    W.ytab = ty;
    W.pair_counter = d_cnt;
    W.oidx = d_wo;
    W.lds_max_len = maxlen;
    W.bt_doubles = bt;
    SK_HIP(ctx, hipEventRecord(ctx->ev0, S));
    SK_HIP(ctx, sk::launch_bpla_grad_wave(W, (int)grid, wpb, S));
    SK_HIP(ctx, hipEventRecord(ctx->ev1, S));
    SK_HIP(ctx, hipStreamSynchronize(S));
    float ms = 0.f;
    SK_HIP(ctx, hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
    total_ms += ms;
  }
  // the thread-per-pair kernel over the remaining pairs, in place of (x, y)
  if (!wx.empty() && !gx.empty()) {
    SK_HIP(ctx, hipMemcpyAsync(d_xy, gx.data(), gx.size() * 4, hipMemcpyHostToDevice, S));
    SK_HIP(ctx, hipMemcpyAsync(d_xy + n, gy.data(), gy.size() * 4, hipMemcpyHostToDevice, S));
  }
  const int64_t ng = wx.empty() ? n : (int64_t)gx.size();
  const int32_t* hx = wx.empty() ? x : gx.data();
  const int32_t* hy = wx.empty() ? y : gy.data();
  // general results: in place when every pair is general, else in their own
  // region (values | grads of the general list), scattered on the host
  double* g_out = wx.empty() ? d_out : d_out + 5 * n;
  for (int64_t b0 = 0; b0 < ng && rc == SK_OK;) {
    int n1 = 1, m1 = 1;
    int64_t b1 = b0;
    while (b1 < ng) {
      const int a1 = std::max(n1, xs_->ex[hx[b1]].len + 1), c1 = std::max(m1, ys_->ex[hy[b1]].len + 1);
      if (b1 > b0 && (double)(b1 - b0 + 1) * sk::bpla_grad_pair_bytes(a1, c1) > budget) break;
      n1 = a1, m1 = c1, ++b1;
    }
    const int64_t cnt = b1 - b0;
    rc = ensure_scratch(ctx, (size_t)cnt * sk::bpla_grad_pair_bytes(n1, m1) + 64);
    if (rc) break;
    sk::BplaGradLaunch G;
    G.xset = xs_->dev;
    G.yset = ys_->dev;
    G.table = d_tb;
    G.alpha = kp->alpha;
    G.beta = kp->beta;
    G.gap = kp->gap;
    G.ext = kp->ext;
    G.beta_gap = std::exp(kp->beta * kp->gap);  // bpla_kernel.cpp:188-189
    G.beta_ext = std::exp(kp->beta * kp->ext);
    G.xs = d_xy + b0;
    G.ys = d_xy + n + b0;
    G.n_pairs = cnt;
    G.n1 = n1;
    G.m1 = m1;
    G.scratch = ctx->scratch;
    G.value = g_out + b0;
    G.grad = g_out + ng + 4 * b0;
    SK_HIP(ctx, hipEventRecord(ctx->ev0, S));
    SK_HIP(ctx, sk::launch_bpla_grad(G, S));
    SK_HIP(ctx, hipEventRecord(ctx->ev1, S));
    SK_HIP(ctx, hipStreamSynchronize(S));
    float ms = 0.f;
    SK_HIP(ctx, hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
    total_ms += ms;
    b0 = b1;
  }
  if (rc == SK_OK) {
    hipError_t e = hipSuccess;
    if (!wx.empty()) {  // wave kernel: by original index
      std::vector<double> v(n), g(4 * (size_t)n);
      e = hipMemcpy(v.data(), d_out, (size_t)n * 8, hipMemcpyDeviceToHost);
      if (e == hipSuccess) e = hipMemcpy(g.data(), d_out + n, (size_t)4 * n * 8, hipMemcpyDeviceToHost);
      for (int64_t k : wo) {
        value[k] = v[k];
        for (int q = 0; q < 4; ++q) grad[4 * k + q] = g[4 * k + q];
      }
    }
    if (e == hipSuccess && ng) {
      std::vector<double> v(ng), g(4 * (size_t)ng);
      e = hipMemcpy(v.data(), g_out, (size_t)ng * 8, hipMemcpyDeviceToHost);
      if (e == hipSuccess) e = hipMemcpy(g.data(), g_out + ng, (size_t)4 * ng * 8, hipMemcpyDeviceToHost);
      for (int64_t t = 0; t < ng; ++t) {
        const int64_t k = wx.empty() ? t : go[t];
        value[k] = v[t];
        for (int q = 0; q < 4; ++q) grad[4 * k + q] = g[4 * t + q];
      }
    }
    if (e != hipSuccess) rc = fail(ctx, SK_ERR_HIP, hipGetErrorString(e));
  }
  ctx->last_stem_ms = total_ms;
  return rc;
}

int pairs_host(sk_context* ctx, sk_dataset* xs_, sk_dataset* ys_, const sk_kernel_params* kp,
               const int32_t* x, const int32_t* y, int64_t n, double* out) {
  if (n == 0) return SK_OK;
  double* d = nullptr;
  SK_HIP(ctx, hipMalloc(&d, (size_t)n * sizeof(double)));
  int rc = run_pairs(ctx, xs_, ys_, kp, x, y, n, d);
  if (rc == SK_OK) {
    // the results are on the context's stream (an asynchronous call has not
    // waited for them): read them in its order
    hipError_t e = hipMemcpyAsync(out, d, (size_t)n * sizeof(double), hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) rc = fail(ctx, SK_ERR_HIP, hipGetErrorString(e));
  }
  (void)hipFree(d);
  return rc;
}

}  // namespace

namespace sk {
int ctx_fail(sk_context* ctx, int code, const std::string& msg) { return fail(ctx, code, msg); }
}  // namespace sk

// =================================================================== ABI
// ---- examples as bytes (a dataset built in rank shares, gathered) --------
// Layout: "SKEX", version 1, count; per example its label and every Example
// field in declaration order (PODs raw, vectors as u64 count + elements,
// strings as u32 length + bytes), little-endian as the host.
namespace {
struct ExWriter {
  uint8_t* buf;
  size_t cap, n = 0;
  void raw(const void* p, size_t b) {
    if (buf && n + b <= cap) std::memcpy(buf + n, p, b);
    n += b;
  }
  template <class T>
  void pod(const T& v) { raw(&v, sizeof(T)); }
  void str(const std::string& s) {
    pod((uint32_t)s.size());
    raw(s.data(), s.size());
  }
  template <class T>
  void vec(const std::vector<T>& v) {
    pod((uint64_t)v.size());
    raw(v.data(), v.size() * sizeof(T));
  }
};
struct ExReader {
  const uint8_t* buf;
  size_t size, n = 0;
  bool ok = true;
  void raw(void* p, size_t b) {
    if (!ok || b > size - n) {
      ok = false;
      return;
    }
    std::memcpy(p, buf + n, b);
    n += b;
  }
  template <class T>
  void pod(T& v) { raw(&v, sizeof(T)); }
  void str(std::string& s) {
    uint32_t l = 0;
    pod(l);
    if (!ok || l > size - n) {
      ok = false;
      return;
    }
    s.assign(reinterpret_cast<const char*>(buf + n), l);
    n += l;
  }
  template <class T>
  void vec(std::vector<T>& v) {
    uint64_t c = 0;
    pod(c);
    if (!ok || c > (size - n) / sizeof(T)) {
      ok = false;
      return;
    }
    v.resize((size_t)c);
    raw(v.data(), (size_t)c * sizeof(T));
  }
};
template <class IO, class E>
void example_fields(IO& io, E& X) {
  io.pod(X.len);
  io.pod(X.n_rows);
  uint8_t hb = X.has_bp ? 1 : 0;  // (a byte on the wire, not a bool's object representation)
  io.pod(hb);
  if constexpr (std::is_same_v<IO, ExReader>) X.has_bp = hb != 0;
  uint32_t nr = (uint32_t)X.rows.size();
  io.pod(nr);
  if constexpr (std::is_same_v<IO, ExReader>) {
    if (!io.ok || nr > io.size - io.n) {
      io.ok = false;
      return;
    }
    X.rows.resize(nr);
  }
  for (auto& r : X.rows) io.str(r);
  io.vec(X.prof5);
  io.pod(X.n_seqs);
  io.vec(X.pos_weight);
  io.vec(X.bpp);
  io.vec(X.first);
  io.vec(X.last);
  io.vec(X.weight);
  io.vec(X.edge_off);
  io.vec(X.edge_to);
  io.vec(X.edge_gaps);
  io.vec(X.bpf_off);
  io.vec(X.bpf_code);
  io.vec(X.bpf_p);
  io.vec(X.roots);
  io.vec(X.max_pa);
}
constexpr uint32_t kExMagic = 0x58454b53u;  // "SKEX"

// The invariants example_build.cpp establishes and the packer and kernels
// rely on (sizes, offsets, children numbered before parents, positions and
// bp-frequency codes in range): an imported example must hold them all.
bool example_valid(const Example& X) {
  const size_t L = X.len >= 0 ? (size_t)X.len : 0;
  if (X.len < 0 || X.n_rows < 1 || X.rows.size() != (size_t)X.n_rows) return false;
  for (const auto& r : X.rows)
    if (r.size() != L) return false;
  if (X.prof5.size() != L * 5) return false;
  const size_t nn = X.first.size();
  if (X.last.size() != nn || X.weight.size() != nn) return false;
  if (X.edge_off.size() != nn + 1 || X.bpf_off.size() != nn + 1 || X.edge_off[0] != 0 || X.bpf_off[0] != 0)
    return false;
  for (size_t v = 0; v < nn; ++v) {
    if (X.edge_off[v + 1] < X.edge_off[v] || X.bpf_off[v + 1] < X.bpf_off[v]) return false;
    if (X.first[v] > X.last[v] || X.last[v] >= L) return false;
  }
  if (X.edge_to.size() != X.edge_off[nn] || X.edge_gaps.size() != X.edge_off[nn]) return false;
  if (X.bpf_code.size() != X.bpf_off[nn] || X.bpf_p.size() != X.bpf_off[nn]) return false;
  for (size_t v = 0; v < nn; ++v)
    for (uint32_t k = X.edge_off[v]; k < X.edge_off[v + 1]; ++k)
      if (X.edge_to[k] >= v) return false;  // children before parents
  for (uint8_t c : X.bpf_code)
    if (c >= 16) return false;
  for (uint32_t r : X.roots)
    if (r >= nn) return false;
  if (X.has_bp) {
    if (X.bpp.size() != (L > 1 ? L * (L - 1) / 2 : 0) || X.pos_weight.size() != L || X.max_pa.size() != nn)
      return false;
  } else if (nn != 0) {
    return false;
  }
  return true;
}
}  // namespace

extern "C" {

void sk_kernel_params_default(sk_kernel_params* p, int32_t kind) {
  if (!p) return;
  p->kind = kind;
  p->len_band = 10;
  p->beta = 0.3;
  p->loop_gap = 0.2;
  p->stack = 1.3;
  p->covar = 0.8;
  p->alpha = 0.2;
  p->gap = 0.8;
  p->match = 1.0;
  p->mismatch = 0.8;
  // bpla_kernel/main.cpp:20-26 (float table), 68-76 (float options)
  static const float kBplaTable[16] = {5.846613f,  -1.860000f, -1.460000f, -1.390000f,
                                       -1.860000f, 4.786613f,  -2.480000f, -1.050000f,
                                       -1.460000f, -2.480000f, 4.656613f,  -1.740000f,
                                       -1.390000f, -1.050000f, -1.740000f, 5.276613f};
  for (int k = 0; k < 16; ++k) p->score_table[k] = (double)kBplaTable[k];
  p->ext = (double)-0.75f;
  // stem_kernel/main.cpp:40-60 (float options; bp_bound default of -p)
  p->subst = (double)0.5f;
  p->bp_bound = 0.0;
  p->bp_model = 0;
  p->loop = 3;
  p->ali_bound = 0.0;
  p->ali_zerop_fixed = 0;
  if (kind == SK_STEM4D) {
    p->gap = (double)0.8f;
    p->stack = (double)1.0f;
    p->len_band = 0;
  }
  if (kind >= SK_BPLA && kind <= SK_LA_SW) {
    p->gap = (double)-8.0f;
    p->alpha = (double)4.5f;
    p->beta = (double)0.11f;
  }
}

const char* sk_strerror(int s) {
  switch (s) {
    case SK_OK: return "ok";
    case SK_ERR_INVALID: return "invalid argument";
    case SK_ERR_HIP: return "HIP runtime error";
    case SK_ERR_NO_DEVICE: return "no usable gfx950 device";
    case SK_ERR_ALLOC: return "allocation failed";
    case SK_ERR_RANGE: return "index out of range";
    case SK_ERR_UNSUPPORTED: return "unsupported";
    default: return "unknown status";
  }
}

const char* sk_last_error(const sk_context* ctx) { return ctx ? ctx->err.c_str() : ""; }

int sk_open(int device, void* hip_stream, sk_context** out) {
  if (!out) return SK_ERR_INVALID;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return SK_ERR_NO_DEVICE;
  if (device < 0 || device >= n) return SK_ERR_RANGE;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return SK_ERR_NO_DEVICE;
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return SK_ERR_NO_DEVICE;
  std::unique_ptr<sk_context> c(new (std::nothrow) sk_context());
  if (!c) return SK_ERR_ALLOC;
  c->device = device;
  c->n_cu = prop.multiProcessorCount;
  if (hipSetDevice(device) != hipSuccess) return SK_ERR_HIP;
  if (hip_stream) {
    c->stream = static_cast<hipStream_t>(hip_stream);
  } else {
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) return SK_ERR_HIP;
    c->own_stream = true;
  }
  // a failure part-way releases what was created (sk_close skips nulls)
  if (hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&c->cls, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&c->eva, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->evf, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->evj, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->evk, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->evx, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->stage[0].ev, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->stage[1].ev, hipEventDisableTiming) != hipSuccess ||
      sk::call_begin(c.get()) != hipSuccess) {  // (creates timing set 0: ev0..ev3)
    sk_close(c.release());
    return SK_ERR_HIP;
  }
  *out = c.release();
  return SK_OK;
}

int sk_close(sk_context* ctx) {
  if (!ctx) return SK_OK;
  (void)hipSetDevice(ctx->device);
  // work may still be queued on any of the context's streams (e.g. after an
  // error part-way through a multi-stream call): drain them all before the
  // buffers they read are freed
  for (hipStream_t st : {ctx->stream, ctx->side, ctx->cls, ctx->aux, ctx->cps})
    if (st) (void)hipStreamSynchronize(st);
  sk::comm_destroy(ctx->comm);
  ctx->comm = nullptr;
  if (ctx->scratch) (void)hipFree(ctx->scratch);
  if (ctx->work) (void)hipFree(ctx->work);
  if (ctx->s4d.pairs) (void)hipFree(ctx->s4d.pairs);
  if (ctx->s4d.items) (void)hipFree(ctx->s4d.items);
  if (ctx->s4d.band) (void)hipFree(ctx->s4d.band);
  if (ctx->side) (void)hipStreamDestroy(ctx->side);
  if (ctx->cls) (void)hipStreamDestroy(ctx->cls);
  if (ctx->aux) (void)hipStreamDestroy(ctx->aux);
  for (hipEvent_t e : {ctx->evf, ctx->evj, ctx->evk, ctx->evx, ctx->eva})
    if (e) (void)hipEventDestroy(e);
  for (auto& T : ctx->tset) {  // (ev0..ev3 are the current set's)
    for (hipEvent_t e : T.ev)
      if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : T.lev) (void)hipEventDestroy(e);
  }
  for (auto& G : ctx->stage) {
    if (G.ev) (void)hipEventDestroy(G.ev);
    if (G.uev) (void)hipEventDestroy(G.uev);
    if (G.dbuf) (void)hipFree(G.dbuf);
    for (auto& b : G.blocks) (void)hipHostFree(b.first);
  }
  if (ctx->cps) (void)hipStreamDestroy(ctx->cps);
  if (ctx->own_stream && ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
  return SK_OK;
}

int sk_dataset_create(sk_dataset** ds) {
  if (!ds) return SK_ERR_INVALID;
  *ds = new (std::nothrow) sk_dataset();
  return *ds ? SK_OK : SK_ERR_ALLOC;
}

int sk_dataset_free(sk_dataset* ds) {
  delete ds;
  return SK_OK;
}

int sk_dataset_add(sk_dataset* ds, const char* label, int n_rows, const char* const* rows,
                   const double* const* bpp_rows, float th, int use_bp) {
  if (!ds || n_rows <= 0 || !rows) return SK_ERR_INVALID;
  if (use_bp && !bpp_rows) return SK_ERR_INVALID;
  if (ds->uploaded) return SK_ERR_INVALID;
  try {
    Example ex;
    sk::build_example(ex, n_rows, rows, bpp_rows, th, use_bp != 0);
    ds->ex.push_back(std::move(ex));
    ds->labels.emplace_back(label ? label : "");
  } catch (const std::bad_alloc&) {
    return SK_ERR_ALLOC;
  } catch (const std::exception& e) {
    ds->err = e.what();
    return SK_ERR_INVALID;
  }
  return SK_OK;
}

int sk_dataset_add_copy(sk_dataset* dst, const sk_dataset* src, int32_t i) {
  if (!dst || !src || i < 0 || (size_t)i >= src->ex.size()) return SK_ERR_INVALID;
  if (dst->uploaded) return SK_ERR_INVALID;
  try {
    dst->ex.push_back(src->ex[(size_t)i]);
    dst->labels.push_back(src->labels[(size_t)i]);
  } catch (const std::bad_alloc&) {
    return SK_ERR_ALLOC;
  }
  return SK_OK;
}

// ---- examples as bytes: see the helpers above extern "C"
int sk_dataset_export(const sk_dataset* ds, int32_t first, int32_t count, uint8_t* buf, size_t cap,
                      size_t* size) {
  if (!ds || !size || first < 0 || count < 0 || (size_t)first + (size_t)count > ds->ex.size())
    return SK_ERR_INVALID;
  ExWriter w{buf, buf ? cap : 0};
  w.pod(kExMagic);
  w.pod((uint32_t)1);
  w.pod((uint32_t)count);
  for (int32_t i = first; i < first + count; ++i) {
    w.str(ds->labels[(size_t)i]);
    example_fields(w, const_cast<Example&>(ds->ex[(size_t)i]));
  }
  *size = w.n;
  return buf && w.n > cap ? SK_ERR_RANGE : SK_OK;
}

int sk_dataset_import(sk_dataset* ds, const uint8_t* buf, size_t size) {
  if (!ds || (!buf && size)) return SK_ERR_INVALID;
  if (ds->uploaded) return SK_ERR_INVALID;
  ExReader r{buf, size};
  uint32_t magic = 0, ver = 0, count = 0;
  r.pod(magic);
  r.pod(ver);
  r.pod(count);
  if (!r.ok || magic != kExMagic || ver != 1) return SK_ERR_INVALID;
  std::vector<Example> ex;
  std::vector<std::string> lab;
  try {
    for (uint32_t i = 0; i < count && r.ok; ++i) {
      lab.emplace_back();
      r.str(lab.back());
      ex.emplace_back();
      example_fields(r, ex.back());
    }
  } catch (const std::bad_alloc&) {
    return SK_ERR_ALLOC;
  }
  if (!r.ok || r.n != size) return SK_ERR_INVALID;  // nothing appended from a malformed buffer
  for (const Example& X : ex)
    if (!example_valid(X)) return SK_ERR_INVALID;
  try {
    ds->ex.insert(ds->ex.end(), std::make_move_iterator(ex.begin()), std::make_move_iterator(ex.end()));
    ds->labels.insert(ds->labels.end(), lab.begin(), lab.end());
  } catch (const std::bad_alloc&) {
    return SK_ERR_ALLOC;
  }
  return SK_OK;
}

int sk_dataset_pack_digest(sk_dataset* ds, uint64_t* y_hash, uint64_t* x_hash) {
  if (!ds || !y_hash || !x_hash) return SK_ERR_INVALID;
  if (ds->uploaded) return SK_ERR_INVALID;
  std::string err;
  const int rc = pack_dataset(ds, err);
  if (rc) return rc;
  const HostPack& P = ds->pack;
  auto hv = [](const auto& v, uint64_t h) {
    typedef typename std::decay_t<decltype(v)>::value_type T;
    const unsigned char* p = reinterpret_cast<const unsigned char*>(v.data());
    for (size_t i = 0; i < v.size() * sizeof(T); ++i) h = (h ^ p[i]) * 1099511628211ull;
    return h ^ v.size();
  };
  uint64_t hy = 1469598103934665603ull, hx = hy;
#define SK_DG_Y(f) hy = hv(P.f, hy);
#define SK_DG_X(f) hx = hv(P.f, hx);
  SK_PACK_Y_ARRAYS(SK_DG_Y)
  SK_PACK_X_ARRAYS(SK_DG_X)
#undef SK_DG_Y
#undef SK_DG_X
  *y_hash = hy;
  *x_hash = hx;
  ds->pack = HostPack();  // (the upload packs again: do not hold the arrays until then)
  return SK_OK;
}

int sk_dataset_add_synthetic_rows(sk_dataset* ds, int32_t n, int32_t n_rows,
                                  const char* const* rows, const char* const* labels, float th,
                                  int32_t n_threads) {
  if (!ds || n < 0 || n_rows < 1 || (n > 0 && !rows)) return SK_ERR_INVALID;
  if (ds->uploaded) return SK_ERR_INVALID;
  const size_t base = ds->ex.size();
  try {
    ds->ex.resize(base + n);
    for (int32_t i = 0; i < n; ++i) ds->labels.emplace_back(labels && labels[i] ? labels[i] : "+1");
  } catch (const std::bad_alloc&) {
    return SK_ERR_ALLOC;
  }
  int nt = n_threads > 0 ? n_threads : (int)std::thread::hardware_concurrency();
  nt = std::max(1, std::min(nt, std::max<int32_t>(n, 1)));
  std::atomic<int32_t> next(0), status(SK_OK);
  static const bool stats = std::getenv("SK_HOST_STATS") != nullptr;
  std::atomic<int64_t> ns_fold(0), ns_build(0);
  auto work = [&]() {
    std::vector<std::vector<double>> bpp(n_rows);
    std::vector<const double*> bptr(n_rows);
    for (;;) {
      const int32_t i = next.fetch_add(1);
      if (i >= n || status.load() != SK_OK) return;
      try {
        const auto t0 = std::chrono::steady_clock::now();
        const char* const* ex_rows = rows + (size_t)i * n_rows;
        for (int32_t r = 0; r < n_rows; ++r) {
          const char* s = ex_rows[r];
          const int L = (int)std::strlen(s);
          // fold the gap-erased, lower-cased row (common/bpmatrix.cpp:404-414)
          std::string row;
          for (int k = 0; k < L; ++k)
            if (s[k] != '-') row.push_back((char)std::tolower((unsigned char)s[k]));
          bpp[r].assign(row.size() > 1 ? row.size() * (row.size() - 1) / 2 : 1, 0.0);
          sk::fold_nussinov(row.c_str(), (int)row.size(), false, bpp[r].data());
          bptr[r] = bpp[r].data();
        }
        const auto t1 = std::chrono::steady_clock::now();
        sk::build_example(ds->ex[base + i], n_rows, ex_rows, bptr.data(), th, true);
        if (stats) {
          const auto t2 = std::chrono::steady_clock::now();
          ns_fold += std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count();
          ns_build += std::chrono::duration_cast<std::chrono::nanoseconds>(t2 - t1).count();
        }
      } catch (...) {
        status.store(SK_ERR_INVALID);
      }
    }
  };
  run_pool(nt, work);
  if (stats)
    std::fprintf(stderr, "[sk] synthetic examples: %d on %d threads, fold %.3f s, build %.3f s (thread-seconds)\n", n,
                 nt, ns_fold.load() * 1e-9, ns_build.load() * 1e-9);
  if (status.load() != SK_OK) {
    ds->ex.resize(base);
    ds->labels.resize(base);
  }
  return status.load();
}

int sk_dataset_add_synthetic(sk_dataset* ds, int32_t n, const char* const* seqs,
                             const char* const* labels, float th, int32_t n_threads) {
  return sk_dataset_add_synthetic_rows(ds, n, 1, seqs, labels, th, n_threads);
}

int sk_dataset_size(const sk_dataset* ds) { return ds ? (int)ds->ex.size() : 0; }

const char* sk_dataset_label(const sk_dataset* ds, int i) {
  if (!ds || i < 0 || i >= (int)ds->labels.size()) return nullptr;
  return ds->labels[i].c_str();
}

int sk_dataset_shape(const sk_dataset* ds, int i, int32_t* n_nodes, int32_t* n_edges,
                     int32_t* n_bpfreq, int32_t* n_roots, int32_t* seq_len) {
  if (!ds) return SK_ERR_INVALID;
  if (i < 0 || i >= (int)ds->ex.size()) return SK_ERR_RANGE;
  const Example& X = ds->ex[i];
  if (n_nodes) *n_nodes = X.n_nodes();
  if (n_edges) *n_edges = X.n_edges();
  if (n_bpfreq) *n_bpfreq = (int32_t)X.bpf_code.size();
  if (n_roots) *n_roots = (int32_t)X.roots.size();
  if (seq_len) *seq_len = X.len;
  return SK_OK;
}

int sk_dataset_row_traffic(const sk_dataset* ds, int i, int32_t* rows, int32_t* stored,
                           int32_t* slab_reads, int32_t* gamma_reads, int32_t* phi_reads,
                           int32_t* reg_reads, int32_t* y_slots) {
  if (!ds) return SK_ERR_INVALID;
  if (i < 0 || i >= (int)ds->ex.size()) return SK_ERR_RANGE;
  const HostPack& P = ds->pack;
  if ((int)P.ex_nlxg.size() != (int)ds->ex.size()) return SK_ERR_INVALID;  // not packed yet
  // the kernel's row reads: slab / Gamma / Phi child records, minus the
  // previous row's (taken from registers); stored rows (slot < 0x4000)
  int32_t st = 0, sl = 0, ga = 0, ph = 0, rg = 0;
  uint32_t prev = 0xffffu;
  size_t k = (size_t)P.ex_xgch_base[i];
  for (size_t r = (size_t)P.ex_xg_base[i]; r < (size_t)P.ex_xg_base[i] + P.ex_nlxg[i]; ++r) {
    const int ne = P.xgrow[r].a & 0xff;
    for (int t = 0; t < ne; ++t, ++k) {
      const uint32_t c = P.xg_ch[k] & 0xffffu;
      if (c == prev) ++rg;
      else if (c & 0x8000u) ++ga;
      else if (c & 0x4000u) ++ph;
      else ++sl;
    }
    prev = P.xgrow[r].b >> 16;
    st += prev < 0x4000u;
  }
  if (rows) *rows = P.ex_nlxg[i];
  if (stored) *stored = st;
  if (slab_reads) *slab_reads = sl;
  if (gamma_reads) *gamma_reads = ga;
  if (phi_reads) *phi_reads = ph;
  if (reg_reads) *reg_reads = rg;
  if (y_slots) *y_slots = P.ex_nl[i];
  return SK_OK;
}

int sk_dataset_dag(const sk_dataset* ds, int i, uint32_t* first, uint32_t* last,
                   uint32_t* n_edges, uint32_t* n_bpfreq, float* weight, uint32_t* max_pa,
                   uint32_t* edge_to, uint32_t* edge_gaps, uint32_t* bp_code, float* bp_p,
                   uint32_t* roots, float* pos_weight) {
  if (!ds) return SK_ERR_INVALID;
  if (i < 0 || i >= (int)ds->ex.size()) return SK_ERR_RANGE;
  const Example& X = ds->ex[i];
  const int n = X.n_nodes();
  for (int v = 0; v < n; ++v) {
    if (first) first[v] = X.first[v];
    if (last) last[v] = X.last[v];
    if (n_edges) n_edges[v] = X.edge_off[v + 1] - X.edge_off[v];
    if (n_bpfreq) n_bpfreq[v] = X.bpf_off[v + 1] - X.bpf_off[v];
    if (weight) weight[v] = X.weight[v];
    if (max_pa) max_pa[v] = X.max_pa[v];
  }
  if (edge_to) std::copy(X.edge_to.begin(), X.edge_to.end(), edge_to);
  if (edge_gaps) std::copy(X.edge_gaps.begin(), X.edge_gaps.end(), edge_gaps);
  if (bp_code) std::copy(X.bpf_code.begin(), X.bpf_code.end(), bp_code);
  if (bp_p) std::copy(X.bpf_p.begin(), X.bpf_p.end(), bp_p);
  if (roots) std::copy(X.roots.begin(), X.roots.end(), roots);
  if (pos_weight && X.has_bp) std::copy(X.pos_weight.begin(), X.pos_weight.end(), pos_weight);
  return SK_OK;
}

int sk_dataset_profile(const sk_dataset* ds, int i, float* prof5, float* n_seqs) {
  if (!ds) return SK_ERR_INVALID;
  if (i < 0 || i >= (int)ds->ex.size()) return SK_ERR_RANGE;
  const Example& X = ds->ex[i];
  if (prof5) std::copy(X.prof5.begin(), X.prof5.end(), prof5);
  if (n_seqs) *n_seqs = X.n_seqs;
  return SK_OK;
}

int sk_dataset_bpla_weights(const sk_dataset* ds, int i, float* p_left, float* p_right,
                            float* p_unpair) {
  if (!ds) return SK_ERR_INVALID;
  if (i < 0 || i >= (int)ds->ex.size()) return SK_ERR_RANGE;
  const Example& X = ds->ex[i];
  for (int k = 0; k < X.len; ++k) {
    const float4 w = bpla_weight(X, k);
    if (p_left) p_left[k] = w.x;
    if (p_right) p_right[k] = w.y;
    if (p_unpair) p_unpair[k] = w.z;
  }
  return SK_OK;
}

int sk_dataset_upload(sk_context* ctx, sk_dataset* ds) {
  if (!ctx || !ds) return SK_ERR_INVALID;
  if (ds->uploaded) return ds->device == ctx->device ? SK_OK : fail(ctx, SK_ERR_INVALID, "dataset bound to another device");
  SK_HIP(ctx, hipSetDevice(ctx->device));
  std::string err;
  HostPack& P = ds->pack;
  DevSet& D = ds->dev;
  DeviceBuffers& B = ds->buf;
  const bool stats = std::getenv("SK_HOST_STATS") != nullptr;
  const auto tu0 = std::chrono::steady_clock::now();
  // the x-role arrays go to the device on a second host thread while the
  // y-role records are formed (pack_dataset calls after_x between the two)
  std::thread xt;
  hipError_t xe = hipSuccess;
  double x_ms = 0.0;
  auto up_x = [&]() -> hipError_t {
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return e;
#define SK_UPX(f, d) \
  if ((e = upload(B, P.f, &D.d)) != hipSuccess) return e;
    SK_UPX(ex_nl, ex_nl)
    SK_UPX(ex_node_base, ex_node_base)
    SK_UPX(ex_edge_base, ex_edge_base)
    SK_UPX(ex_bpf_base, ex_bpf_base)
    SK_UPX(ex_lvl_base, ex_lvl_base)
    SK_UPX(ex_nlev, ex_nlev)
    SK_UPX(ex_nseqs, ex_nseqs)
    SK_UPX(ex_len, ex_len)
    SK_UPX(ex_pos_base, ex_pos_base)
    SK_UPX(ex_has_w, ex_has_w)
    SK_UPX(nd_a, nd_a)
    SK_UPX(nd_b, nd_b)
    SK_UPX(nd_c, nd_c)
    SK_UPX(nd_w, nd_w)
    SK_UPX(nd_nbp, nd_nbp)
    SK_UPX(nd_P, nd_P)
    SK_UPX(ed, ed)
    SK_UPX(bpf_code, bpf_code)
    SK_UPX(bpf_p, bpf_p)
    SK_UPX(lvl, lvl)
    SK_UPX(pos_prof, pos_prof)
    SK_UPX(pos_w, pos_w)
    SK_UPX(pos_chr, pos_chr)
    SK_UPX(pos_lru, pos_lru)
    SK_UPX(ex_nslots, ex_nslots)
    SK_UPX(ex_xch_base, ex_xch_base)
    SK_UPX(xrow, xrow)
    SK_UPX(xr_node, xr_node)
    SK_UPX(xr_ch, xr_ch)
    SK_UPX(xgrow, xgrow)
    SK_UPX(xg_node, xg_node)
    SK_UPX(xg_ch, xg_ch)
    SK_UPX(xg_clg, xg_clg)
    SK_UPX(xg_cpf, xg_cpf)
    SK_UPX(ex_xg_base, ex_xg_base)
    SK_UPX(ex_nlxg, ex_nlxg)
    SK_UPX(ex_xgch_base, ex_xgch_base)
    SK_UPX(gr_info, gr_info)
    SK_UPX(gr_pf, gr_pf)
    SK_UPX(gr_P, gr_P)
    SK_UPX(ex_gapless, ex_gapless)
    SK_UPX(gam_key, gam_key)
    SK_UPX(xg_cty, xg_cty)
    SK_UPX(gra_gidx, gra_gidx)
    SK_UPX(gra_row, gra_row)
    SK_UPX(phk_idx, phk_idx)
    SK_UPX(phi_al, phi_al)
    SK_UPX(phi_g, phi_g)
    {
      std::vector<int32_t> grb = P.ex_gr_base;
      grb.push_back((int32_t)P.gr_info.size());
      if ((e = upload(B, grb, &D.ex_gr_base)) != hipSuccess) return e;
      std::vector<int32_t> b1 = P.ex_gra_base, b2 = P.ex_phk_base;
      b1.push_back((int32_t)P.gra_gidx.size());
      b2.push_back((int32_t)P.phk_idx.size());
      if ((e = upload(B, b1, &D.ex_gra_base)) != hipSuccess) return e;
      if ((e = upload(B, b2, &D.ex_phk_base)) != hipSuccess) return e;
    }
#undef SK_UPX
    return hipSuccess;
  };
  const std::function<void()> after_x = [&]() {
    P.xr_ch.insert(P.xr_ch.end(), 8, 0u);  // the kernel prefetches 4 records past a row
    P.xg_ch.insert(P.xg_ch.end(), 8, 0u);
    auto job = [&]() {
      const auto t0 = std::chrono::steady_clock::now();
      xe = up_x();
      x_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    };
    try {
      xt = std::thread(job);
    } catch (const std::system_error&) {
      job();  // no second thread: upload them here, before the y-role pack
    }
  };
  int rc = pack_dataset(ds, err, &after_x);
  if (xt.joinable()) xt.join();
  if (rc) return fail(ctx, rc, err);
  SK_HIP(ctx, xe);
  const auto tu1 = std::chrono::steady_clock::now();
  D.n_examples = (int32_t)ds->ex.size();
  SK_HIP(ctx, upload(B, P.yn_a, &D.yn_a));
  SK_HIP(ctx, upload(B, P.yn_b, &D.yn_b));
  SK_HIP(ctx, upload(B, P.yn_w, &D.yn_w));
  SK_HIP(ctx, upload(B, P.yn_nbp, &D.yn_nbp));
  SK_HIP(ctx, upload(B, P.yn_P, &D.yn_P));
  SK_HIP(ctx, upload(B, P.ysc, &D.ysc));
  SK_HIP(ctx, upload(B, P.ye2, &D.ye2));
  SK_HIP(ctx, upload(B, P.yn_c, &D.yn_c));
  SK_HIP(ctx, upload(B, P.yn_p0, &D.yn_p0));
  SK_HIP(ctx, upload(B, P.ycs, &D.ycs));
  SK_HIP(ctx, upload(B, P.yrec, &D.yrec));
  SK_HIP(ctx, upload(B, P.ex_ysc_base, &D.ex_ysc_base));
  SK_HIP(ctx, upload(B, P.ex_nch, &D.ex_nch));
  SK_HIP(ctx, upload(B, P.ex_ycs_base, &D.ex_ycs_base));
  D.n_gam = (int32_t)P.gam_key.size();
  D.n_phi = (int32_t)P.phi_al.size();
  D.max_nl = P.max_nl;
  D.max_edges = P.max_edges;
  D.max_bpf = P.max_bpf;
  D.max_nlev = P.max_nlev;
  D.max_nch = P.max_nch;
  D.max_len = P.max_len;
  D.max_slots = P.max_slots;
  D.total_nodes = (int64_t)P.nd_a.size();
  ds->device = ctx->device;
  ds->uploaded = true;
  if (stats) {
    const auto tu2 = std::chrono::steady_clock::now();
    std::fprintf(stderr,
                 "[sk upload] pack + x-role arrays %.1f ms (x-role transfer %.1f ms beside the y-role pack), %zu arrays "
                 "%.1f MB in all, y-role transfer %.1f ms\n",
                 std::chrono::duration<double, std::milli>(tu1 - tu0).count(), x_ms, B.ptrs.size(), B.bytes / 1e6,
                 std::chrono::duration<double, std::milli>(tu2 - tu1).count());
  }
  return SK_OK;
}

int sk_pairs_device(sk_context* ctx, sk_dataset* ds, const sk_kernel_params* kp, const int32_t* x,
                    const int32_t* y, int64_t n_pairs, double* out_dev) {
  return run_pairs(ctx, ds, ds, kp, x, y, n_pairs, out_dev);
}

int sk_bpla_gradients(sk_context* ctx, sk_dataset* xs, sk_dataset* ys, const sk_kernel_params* kp,
                      const int32_t* x, const int32_t* y, int64_t n_pairs, double* value,
                      double* grad) {
  return bpla_gradients(ctx, xs, ys, kp, x, y, n_pairs, value, grad);
}

int sk_pairs(sk_context* ctx, sk_dataset* ds, const sk_kernel_params* kp, const int32_t* x,
             const int32_t* y, int64_t n_pairs, double* out) {
  return pairs_host(ctx, ds, ds, kp, x, y, n_pairs, out);
}

int sk_gram(sk_context* ctx, sk_dataset* ds, const sk_kernel_params* kp, int normalize,
            double* out) {
  if (!ctx || !ds || !kp || !out) return fail(ctx, SK_ERR_INVALID, "null argument");
  const int n = (int)ds->ex.size();
  std::vector<int32_t> xi, yi;
  xi.reserve((size_t)n * (n + 1) / 2);
  yi.reserve((size_t)n * (n + 1) / 2);
  // the reference's cell order (kernel_matrix.cpp:44-55): i outer, j >= i
  for (int i = 0; i < n; ++i)
    for (int j = i; j < n; ++j) {
      xi.push_back(i);
      yi.push_back(j);
    }
  std::vector<double> v(std::max<size_t>(xi.size(), 1));
  int rc = pairs_host(ctx, ds, ds, kp, xi.data(), yi.data(), (int64_t)xi.size(), v.data());
  if (rc) return rc;
  // mirror + normalise (kernel_matrix.cpp:560-571): the one-rank case of the
  // sharded assembly (csrc/host/shard.cpp), so both give the same bits
  return sk_shard_assemble(n, 1, v.data(), (int64_t)v.size(), normalize, out);
}

int sk_test_row(sk_context* ctx, sk_dataset* test, int t, sk_dataset* train,
                const int32_t* sv_index, int32_t n_sv, const sk_kernel_params* kp, double* out,
                double* self) {
  if (!ctx || !test || !train || !kp || !out) return fail(ctx, SK_ERR_INVALID, "null argument");
  if (t < 0 || t >= (int)test->ex.size()) return fail(ctx, SK_ERR_RANGE, "test index");
  const int ntr = (int)train->ex.size();
  std::vector<int32_t> xi, yi;
  if (sv_index) {
    for (int32_t k = 0; k < n_sv; ++k) {
      if (sv_index[k] < 0 || sv_index[k] >= ntr) return fail(ctx, SK_ERR_RANGE, "sv index");
      xi.push_back(sv_index[k]);
    }
  } else {
    for (int i = 0; i < ntr; ++i) xi.push_back(i);
  }
  yi.assign(xi.size(), t);
  std::vector<double> v(xi.size());
  // kernel_(train_[i].second, data_.second): x = train, y = test
  int rc = pairs_host(ctx, train, test, kp, xi.data(), yi.data(), (int64_t)xi.size(), v.data());
  if (rc) return rc;
  for (size_t k = 0; k < xi.size(); ++k) out[xi[k]] = v[k];
  if (self) {
    const int32_t a = t;
    rc = pairs_host(ctx, test, test, kp, &a, &a, 1, self);
    if (rc) return rc;
  }
  return SK_OK;
}

int sk_diagonal(sk_context* ctx, sk_dataset* ds, const int32_t* sv_index, int32_t n_sv,
                const sk_kernel_params* kp, double* out) {
  if (!ctx || !ds || !kp || !out) return fail(ctx, SK_ERR_INVALID, "null argument");
  const int n = (int)ds->ex.size();
  std::vector<int32_t> xi;
  if (sv_index) {
    for (int32_t k = 0; k < n_sv; ++k) {
      if (sv_index[k] < 0 || sv_index[k] >= n) return fail(ctx, SK_ERR_RANGE, "sv index");
      xi.push_back(sv_index[k]);
    }
  } else {
    for (int i = 0; i < n; ++i) xi.push_back(i);
  }
  std::vector<double> v(xi.size());
  int rc = pairs_host(ctx, ds, ds, kp, xi.data(), xi.data(), (int64_t)xi.size(), v.data());
  if (rc) return rc;
  for (size_t k = 0; k < xi.size(); ++k) out[xi[k]] = v[k];
  return SK_OK;
}

int sk_test_matrix(sk_context* ctx, sk_dataset* test, sk_dataset* train,
                   const sk_kernel_params* kp, int norm_test, int normalize, double* out,
                   double* self_out) {
  if (!ctx || !test || !train || !kp || !out) return fail(ctx, SK_ERR_INVALID, "null argument");
  const int nt = (int)test->ex.size(), ntr = (int)train->ex.size();
  std::vector<int32_t> xi, yi;
  for (int i = 0; i < nt; ++i)
    for (int j = 0; j < ntr; ++j) {
      xi.push_back(j);
      yi.push_back(i);
    }
  int rc = pairs_host(ctx, train, test, kp, xi.data(), yi.data(), (int64_t)xi.size(), out);
  if (rc) return rc;
  std::vector<double> self(nt, 0.0);
  if (norm_test || normalize) {
    std::vector<int32_t> ti(nt);
    std::iota(ti.begin(), ti.end(), 0);
    rc = pairs_host(ctx, test, test, kp, ti.data(), ti.data(), nt, self.data());
    if (rc) return rc;
    if (self_out) std::copy(self.begin(), self.end(), self_out);
  }
  if (normalize) {
    std::vector<double> diag(ntr);
    rc = sk_diagonal(ctx, train, nullptr, 0, kp, diag.data());
    if (rc) return rc;
    for (int i = 0; i < nt; ++i)
      for (int j = 0; j < ntr; ++j) out[(size_t)i * ntr + j] /= std::sqrt(self[i] * diag[j]);
  }
  return SK_OK;
}

int sk_format_libsvm(const double* m, int32_t rows, int32_t cols, const char* const* labels,
                     char* buf, size_t buf_size, size_t* needed) {
  if ((!m && rows * cols) || rows < 0 || cols < 0) return SK_ERR_INVALID;
  // KernelMatrix::print (kernel_matrix.cpp:756-770): ostream defaults
  std::ostringstream os;
  for (int32_t i = 0; i < rows; ++i) {
    os << (labels && labels[i] ? labels[i] : "") << " 0:" << (i + 1) << " ";
    for (int32_t j = 0; j < cols; ++j) os << (j + 1) << ":" << m[(size_t)i * cols + j] << " ";
    os << "\n";
  }
  const std::string s = os.str();
  if (needed) *needed = s.size() + 1;
  if (buf) {
    if (buf_size < s.size() + 1) return SK_ERR_RANGE;
    std::memcpy(buf, s.c_str(), s.size() + 1);
  }
  return SK_OK;
}

int sk_fold_synthetic(const char* seq, int32_t n, int32_t no_gu, double* out) {
  if (!seq || n < 0 || (!out && n > 1)) return SK_ERR_INVALID;
  try {
    sk::fold_nussinov(seq, n, no_gu != 0, out);
  } catch (const std::bad_alloc&) {
    return SK_ERR_ALLOC;
  }
  return SK_OK;
}

// ---------------------------------------------------------------- McCaskill fold (f1)
namespace {

// Boltzmann factor tables of fold.hip (host/fold_params.h), laid out in one
// buffer: the fixed-size tables first (o_st .. o_ml, n_small doubles), then
// the two whose length follows the batch's longest sequence max_len (hairpin,
// scale powers), so a launch whose tables outgrow the LDS keeps the first
// part in LDS and reads the tail from HBM (fold.hip GTAB).  Entry k of every
// table is the same double whatever max_len is.
void fold_tables(int max_len, sk::FoldLaunch& L, std::vector<double>& t) {
  using namespace sk::foldp;
  t.clear();
  auto bz = [](double e) { return std::exp(-e / kT); };
  L.o_st = (int32_t)t.size();
  for (int a = 0; a < 7; ++a)
    for (int b = 0; b < 7; ++b) t.push_back(a && b ? bz(stack37[a][b]) : 0.0);
  L.o_bu = (int32_t)t.size();
  for (int k = 0; k <= max_loop; ++k) t.push_back(k ? bz(bulge37[k]) : 0.0);
  L.o_in = (int32_t)t.size();
  for (int k = 0; k <= max_loop; ++k) t.push_back(k >= 2 ? bz(interior37[k]) : 0.0);
  L.o_ni = (int32_t)t.size();
  for (int k = 0; k <= max_loop; ++k) t.push_back(bz(std::min(max_ninio, ninio * k)));
  L.o_au = (int32_t)t.size();
  for (int k = 0; k < 7; ++k) t.push_back(k > 2 ? bz(terminal_au) : 1.0);
  L.o_ml = (int32_t)t.size();
  t.push_back(bz(ml_closing + ml_intern));
  t.push_back(bz(ml_intern));
  L.n_small = (int32_t)t.size();
  L.o_hp = (int32_t)t.size();
  for (int k = 0; k <= max_len + 1; ++k) {
    if (k < 3) {
      t.push_back(0.0);
      continue;
    }
    double e = hairpin37[k <= 30 ? k : 30];
    if (k > 30) e += lxc * std::log((double)k / 30.0);
    t.push_back(bz(e));
  }
  L.o_scp = (int32_t)t.size();
  for (int k = 0; k <= max_len + 2; ++k) t.push_back(std::exp(log_sc * k));
  L.log_sc = log_sc;
  L.n_tab = (int32_t)t.size();
  L.n_tab_pad = (L.n_tab + 1) & ~1;
}

int8_t fold_code(char ch) {
  switch (ch) {
    case 'A': case 'a': return 0;
    case 'C': case 'c': return 1;
    case 'G': case 'g': return 2;
    case 'U': case 'u': case 'T': case 't': return 3;
    default: return -1;
  }
}

}  // namespace

// --noLonelyPairs (common/bpmatrix.cpp:56-58, 149, Vienna::noLonelyPairs):
// the legacy ViennaRNA partition function applies it through its pair-type
// table only (1.8 part_func.c make_ptypes; not vendored).  Walking each chain
// (i, j), (i-1, j+1), ... outward from its innermost pair (j - i = 4 or 5),
// a pair is dropped when its inner neighbour was dropped or cannot pair and
// its outer neighbour cannot pair; the outer type is re-read only inside the
// sequence, so a chain's outermost pair compares against its own type.
// lp[i*n + j] = 1 where the pair survives (codes: fold_code, -1 never pairs).
void lonely_pair_table(const int8_t* c, int n, bool no_gu, uint8_t* lp) {
  static const int8_t pt[16] = {0, 0, 0, 5, 0, 0, 1, 0, 0, 2, 0, 4, 6, 0, 3, 0};
  auto raw = [&](int i, int j) {
    const int t = (c[i] < 0 || c[j] < 0) ? 0 : pt[c[i] * 4 + c[j]];
    return (no_gu && (t == 3 || t == 4)) ? 0 : t;
  };
  std::fill(lp, lp + (size_t)n * n, (uint8_t)0);
  for (int k = 0; k < n; ++k)
    for (int l = 1; l <= 2; ++l) {
      int i = k, j = k + 3 + l, otype = 0, ntype = 0;
      if (j >= n) continue;
      int type = raw(i, j);
      for (; i >= 0 && j < n; --i, ++j) {
        if (i > 0 && j < n - 1) ntype = raw(i - 1, j + 1);
        if (!otype && !ntype) type = 0;
        lp[(size_t)i * n + j] = type != 0;
        otype = type;
        type = ntype;
      }
    }
}

int sk_fold_mccaskill(sk_context* ctx, int32_t n, const char* const* seqs, int32_t flags,
                      double* out, double* log_z) {
  if (!ctx || n < 0 || (n > 0 && (!seqs || !out))) return fail(ctx, SK_ERR_INVALID, "null argument");
  if (flags & ~(SK_FOLD_NO_GU | SK_FOLD_NO_CLOSING_GU | SK_FOLD_NO_LONELY_PAIRS))
    return fail(ctx, SK_ERR_UNSUPPORTED, "fold: unknown flag");
  const bool no_lp = (flags & SK_FOLD_NO_LONELY_PAIRS) != 0;
  if (n == 0) return SK_OK;
  std::vector<int> len(n);
  int max_len = 0;
  for (int32_t k = 0; k < n; ++k) {
    if (!seqs[k]) return fail(ctx, SK_ERR_INVALID, "null sequence");
    len[k] = (int)std::strlen(seqs[k]);
    max_len = std::max(max_len, len[k]);
  }
  sk::FoldLaunch L;
  std::vector<double> tab;
  L.no_gu = (flags & SK_FOLD_NO_GU) ? 1 : 0;
  L.no_closing_gu = (flags & SK_FOLD_NO_CLOSING_GU) ? 1 : 0;
  size_t free_b = 0, total_b = 0;
  SK_HIP(ctx, hipMemGetInfo(&free_b, &total_b));
  const double budget = std::min(16e9, 0.4 * (double)free_b);
  hipStream_t S = ctx->stream;
  size_t out_host = 0;  // packed output offset of sequence k (host)
  for (int32_t b0 = 0; b0 < n;) {
    // batch: sequences whose tables fit the budget (at least one)
    std::vector<sk::FoldSeq> sq;
    std::vector<int8_t> codes;
    std::vector<uint8_t> lp;  // --noLonelyPairs tables
    size_t work = 0, outn = 0;
    int32_t b1 = b0;
    int bmax = 0;
    for (; b1 < n; ++b1) {
      const size_t nn = (size_t)len[b1];
      const size_t w = sk::fold_work_doubles(nn);
      if (!sq.empty() && (double)(work + w) * 8.0 > budget) break;
      sk::FoldSeq f;
      f.seq_off = (int64_t)codes.size();
      f.work_off = (int64_t)work;
      f.out_off = (int64_t)outn;
      f.n = (int32_t)nn;
      for (size_t a = 0; a < nn; ++a) codes.push_back(fold_code(seqs[b1][a]));
      if (no_lp) {
        f.lp_off = (int64_t)lp.size();
        lp.resize(lp.size() + nn * nn);
        lonely_pair_table(codes.data() + f.seq_off, (int)nn, L.no_gu != 0, lp.data() + f.lp_off);
      }
      work += w;
      outn += nn > 1 ? nn * (nn - 1) / 2 : 0;
      bmax = std::max(bmax, (int)nn);
      sq.push_back(f);
    }
    const int nb = b1 - b0;
    fold_tables(bmax, L, tab);  // sized by this batch's longest sequence
    if (sk::fold_lds_bytes(L, bmax) > sk::kFoldLdsMax)
      return fail(ctx, SK_ERR_UNSUPPORTED, "fold: sequence too long for the fold kernel's LDS");
    size_t need = sq.size() * sizeof(sk::FoldSeq) + codes.size() + lp.size() + tab.size() * 8 +
                  (outn + nb) * 8 + 7 * 256;
    int rc = ensure_work(ctx, need);
    if (rc) return rc;
    rc = ensure_scratch(ctx, std::max<size_t>(work * 8, 64));
    if (rc) return rc;
    Arena A{static_cast<char*>(ctx->work), 0, ctx->work_bytes};
    sk::FoldSeq* d_sq = A.take<sk::FoldSeq>(sq.size());
    int8_t* d_codes = A.take<int8_t>(std::max<size_t>(codes.size(), 1));
    double* d_tab = A.take<double>(tab.size());
    double* d_out = A.take<double>(std::max<size_t>(outn, 1));
    double* d_lz = A.take<double>(nb);
    uint8_t* d_lp = no_lp ? A.take<uint8_t>(std::max<size_t>(lp.size(), 1)) : nullptr;
    if (no_lp && !lp.empty())
      SK_HIP(ctx, hipMemcpyAsync(d_lp, lp.data(), lp.size(), hipMemcpyHostToDevice, S));
    L.lp = d_lp;
    SK_HIP(ctx, hipMemcpyAsync(d_sq, sq.data(), sq.size() * sizeof(sk::FoldSeq), hipMemcpyHostToDevice, S));
    if (!codes.empty())
      SK_HIP(ctx, hipMemcpyAsync(d_codes, codes.data(), codes.size(), hipMemcpyHostToDevice, S));
    SK_HIP(ctx, hipMemcpyAsync(d_tab, tab.data(), tab.size() * 8, hipMemcpyHostToDevice, S));
    SK_HIP(ctx, hipMemsetAsync(ctx->scratch, 0, work * 8, S));
    SK_HIP(ctx, hipMemsetAsync(d_out, 0, std::max<size_t>(outn, 1) * 8, S));
    L.seqs = d_sq;
    L.codes = d_codes;
    L.tab = d_tab;
    L.work = ctx->scratch;
    L.out = d_out;
    L.log_z = d_lz;
    SK_HIP(ctx, sk::launch_fold(L, nb, bmax, S));
    std::vector<double> lz(nb);
    if (outn) SK_HIP(ctx, hipMemcpyAsync(out + out_host, d_out, outn * 8, hipMemcpyDeviceToHost, S));
    SK_HIP(ctx, hipMemcpyAsync(lz.data(), d_lz, nb * 8, hipMemcpyDeviceToHost, S));
    SK_HIP(ctx, hipStreamSynchronize(S));
    for (int k = 0; k < nb; ++k) {
      if (!std::isfinite(lz[k]))
        return fail(ctx, SK_ERR_UNSUPPORTED, "fold: partition function out of double range (sequence too long)");
      if (log_z) log_z[b0 + k] = lz[k];
    }
    out_host += outn;
    b0 = b1;
  }
  return SK_OK;
}

namespace {
// Threaded DAG builds of n examples of n_rows rows from per-row bpp (caller's
// or folded), appended to ds; the parallel form of the reference's load loop
// (common/framework.h:308-353 + DataLoader<MData>::get, data.cpp:548-586).
int add_examples_threaded(sk_dataset* ds, int32_t n, int32_t n_rows, const char* const* rows,
                          const double* const* bpp_rows, const char* const* labels, float th,
                          int use_bp, int32_t n_threads) {
  const size_t base = ds->ex.size();
  try {
    ds->ex.resize(base + n);
    for (int32_t i = 0; i < n; ++i) ds->labels.emplace_back(labels && labels[i] ? labels[i] : "+1");
  } catch (const std::bad_alloc&) {
    return SK_ERR_ALLOC;
  }
  int nt = n_threads > 0 ? n_threads : (int)std::thread::hardware_concurrency();
  nt = std::max(1, std::min(nt, std::max<int32_t>(n, 1)));
  std::atomic<int32_t> next(0), status(SK_OK);
  auto work = [&]() {
    for (;;) {
      const int32_t i = next.fetch_add(1);
      if (i >= n || status.load() != SK_OK) return;
      try {
        sk::build_example(ds->ex[base + i], n_rows, rows + (size_t)i * n_rows,
                          use_bp ? bpp_rows + (size_t)i * n_rows : nullptr, th, use_bp != 0);
      } catch (...) {
        status.store(SK_ERR_INVALID);
      }
    }
  };
  run_pool(nt, work);
  if (status.load() != SK_OK) {
    ds->ex.resize(base);
    ds->labels.resize(base);
  }
  return status.load();
}
}  // namespace

int sk_dataset_add_batch(sk_dataset* ds, int32_t n, int32_t n_rows, const char* const* rows,
                         const double* const* bpp_rows, const char* const* labels, float th,
                         int32_t use_bp, int32_t n_threads) {
  if (!ds || n < 0 || n_rows < 1 || (n > 0 && (!rows || (use_bp && !bpp_rows)))) return SK_ERR_INVALID;
  if (ds->uploaded) return SK_ERR_INVALID;
  return add_examples_threaded(ds, n, n_rows, rows, bpp_rows, labels, th, use_bp, n_threads);
}

int sk_dataset_add_folded(sk_context* ctx, sk_dataset* ds, int32_t n, int32_t n_rows,
                          const char* const* rows, const char* const* labels, float th,
                          int32_t fold_flags, int32_t n_threads) {
  if (!ctx || !ds || n < 0 || n_rows < 1 || (n > 0 && !rows)) return fail(ctx, SK_ERR_INVALID, "null argument");
  if (ds->uploaded) return fail(ctx, SK_ERR_INVALID, "dataset already uploaded");
  const size_t nr = (size_t)n * n_rows;
  // fold the gap-erased, lower-cased rows (common/bpmatrix.cpp:404-414)
  std::vector<std::string> erased(nr);
  std::vector<const char*> eptr(nr);
  std::vector<size_t> off(nr + 1, 0);
  for (size_t r = 0; r < nr; ++r) {
    if (!rows[r]) return fail(ctx, SK_ERR_INVALID, "null row");
    for (const char* p = rows[r]; *p; ++p)
      if (*p != '-') erased[r].push_back((char)std::tolower((unsigned char)*p));
    eptr[r] = erased[r].c_str();
    const size_t m = erased[r].size();
    off[r + 1] = off[r] + (m > 1 ? m * (m - 1) / 2 : 0);
  }
  std::vector<double> bpp(std::max<size_t>(off[nr], 1));
  int rc = sk_fold_mccaskill(ctx, (int32_t)nr, eptr.data(), fold_flags, bpp.data(), nullptr);
  if (rc) return rc;
  std::vector<const double*> bptr(nr);
  for (size_t r = 0; r < nr; ++r) bptr[r] = bpp.data() + off[r];
  rc = add_examples_threaded(ds, n, n_rows, rows, bptr.data(), labels, th, 1, n_threads);
  return rc ? fail(ctx, rc, "example build failed") : SK_OK;
}

int sk_random_sequences(uint64_t* state, int32_t n_seqs, int32_t len, char* out) {
  if (!state || !out || n_seqs < 0 || len < 0) return SK_ERR_INVALID;
  for (int32_t s = 0; s < n_seqs; ++s) sk::random_sequence(*state, len, out + (size_t)s * (len + 1));
  return SK_OK;
}

int sk_last_timing(const sk_context* ctx, double* stem_ms, double* string_ms, double* cells,
                   int32_t* launches) {
  if (!ctx) return SK_ERR_INVALID;
  if (stem_ms) *stem_ms = ctx->last_stem_ms;
  if (string_ms) *string_ms = ctx->last_str_ms;
  if (cells) *cells = ctx->last_cells;
  if (launches) *launches = ctx->last_launches;
  return SK_OK;
}

int sk_set_async(sk_context* ctx, int32_t on) {
  if (!ctx) return SK_ERR_INVALID;
  if (ctx->async && !on) {  // resolve what is pending first
    const int rc = sk_sync_timing(ctx);
    if (rc) return rc;
  }
  ctx->async = on != 0;
  return SK_OK;
}

int sk_sync_timing(sk_context* ctx) {
  if (!ctx) return SK_ERR_INVALID;
  if (!ctx->async) return SK_OK;
  for (int k = 0; k < sk_context::kTSets; ++k)
    if (sk::tset_resolve(ctx, k) != hipSuccess) return fail(ctx, SK_ERR_HIP, "sk_sync_timing: event");
  ctx->last_stem_ms = ctx->acc_stem_ms;
  ctx->last_str_ms = ctx->acc_str_ms;
  ctx->last_cells = ctx->acc_cells;
  ctx->last_launches = ctx->acc_launches;
  ctx->last_launch_ms_sum = ctx->acc_launch_ms;
  ctx->last_launch_n = ctx->acc_launch_n;
  ctx->acc_stem_ms = ctx->acc_str_ms = ctx->acc_cells = ctx->acc_launch_ms = 0.0;
  ctx->acc_launch_n = ctx->acc_launches = 0;
  return SK_OK;
}

int sk_last_launch_ms(const sk_context* ctx, double* ms_sum, int32_t* n_launches) {
  if (!ctx) return SK_ERR_INVALID;
  if (ms_sum) *ms_sum = ctx->last_launch_ms_sum;
  if (n_launches) *n_launches = ctx->last_launch_n;
  return SK_OK;
}

int sk_stem4d_col_shape(int32_t min_len, int32_t max_len, int32_t* nb, int32_t* waves, int32_t* pf) {
  if (max_len < 0 || min_len > max_len) return SK_ERR_INVALID;
  const int cpl = sk::stem4d_cpl(max_len);
  // the shape of the launch that actually runs (a Gram: x and y lengths in
  // [min_len, max_len]); waves = 0 where the column kernel does not run --
  // |y| >= 512 (k tiles), |x| past its LDS / step-count limit, or a y too
  // short for the column schedule (those pairs take the span kernel)
  const bool runs = max_len + 1 <= 64 * cpl && max_len <= sk::stem4d_col_max_n() &&
                    (min_len <= 1 || sk::stem4d_col_w_max(min_len) >= 1);
  if (nb) *nb = sk::stem4d_col_nb(cpl);
  if (waves) *waves = runs ? col_waves(cpl, min_len >= 2 ? min_len : INT32_MAX, max_len, max_len) : 0;
  if (pf) *pf = sk::stem4d_col_pf();
  return SK_OK;
}

int sk_last_classes(const sk_context* ctx, uint32_t* stem_maxk_mask, uint32_t* stem4d_mask) {
  if (!ctx) return SK_ERR_INVALID;
  if (stem_maxk_mask) *stem_maxk_mask = ctx->last_stem_classes;
  if (stem4d_mask) *stem4d_mask = ctx->last_s4d_classes;
  return SK_OK;
}

void sk_ribosum_tables(float* s16, float* p256) {
  if (s16) std::memcpy(s16, SK_RIBOSUM_S, sizeof(SK_RIBOSUM_S));
  if (p256) std::memcpy(p256, SK_RIBOSUM_P, sizeof(SK_RIBOSUM_P));
}

int sk_char2rna(int c) { return sk::char2rna(c); }

int sk_experiments(void) {
#ifdef SK_EXPERIMENTS
  return 1;
#else
  return 0;
#endif
}

}  // extern "C"
