// Multi-GPU Gram: the cell plan, the assembly and the RCCL all-gather behind
// the C ABI, so a C++ host (the reference's App::train) shards the Gram over
// the GPUs of a node without torch.
//
// Plan: the reference's MPI Gram deals the upper-triangle cells (i <= j,
// row-major) cyclically, cell k to rank k % P (CalcTrainMatrix::operator(),
// common/kernel_matrix.cpp:210-224), and rank 0 receives every rank's values
// point-to-point and scatters them back by replaying the same order
// (:225-261, 495-527).  Here the same cyclic plan is kept -- it gives every
// rank the same cost mix of short and long examples, so no cost model is
// needed -- each rank's values land in a device buffer of ceil(T / P)
// doubles, ONE ncclAllGather over xGMI concatenates the P buffers on every
// rank, and every rank unscatters (cell k = buffer k % P, slot k / P),
// mirrors and normalises exactly as KernelMatrix::calculate
// (common/kernel_matrix.cpp:560-571).  Values depend only on the pair, so
// the P-GPU Gram is bit-identical to the 1-GPU Gram.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "host/sk_internal.h"
#include "stem_kernel.h"

namespace {

int64_t tri_cells(int64_t n) { return n * (n + 1) / 2; }

// Upper triangle rows [r0, r1) from the gathered buffers (row i's cells
// (i, j >= i) are the consecutive cell indices from c0(i) = i*n - i*(i-1)/2),
// normalised as kernel_matrix.cpp:560-571 when diag != nullptr: K_ij /=
// sqrt(K_ii * K_jj) with the raw diagonal, then diag := 1.
void upper_rows(int64_t n, int64_t world, const double* g, int64_t per, const double* diag,
                double* out, int64_t r0, int64_t r1) {
  for (int64_t i = r0; i < r1; ++i) {
    const int64_t c0 = i * n - i * (i - 1) / 2;
    double* row = out + i * n;
    for (int64_t j = i; j < n; ++j) {
      const int64_t k = c0 + (j - i);
      row[j] = g[(k % world) * per + k / world];
    }
    if (diag) {
      for (int64_t j = i + 1; j < n; ++j) row[j] /= std::sqrt(diag[i] * diag[j]);
      row[i] = 1;
    }
  }
}

// Lower triangle = mirror of the upper, in 64 x 64 tiles (row blocks
// [b0, b1) of the lower triangle).
void mirror_blocks(int64_t n, double* out, int64_t b0, int64_t b1) {
  constexpr int64_t T = 64;
  for (int64_t bi = b0; bi < b1; ++bi)
    for (int64_t bj = 0; bj <= bi; ++bj)
      for (int64_t i = bi * T; i < std::min(n, bi * T + T); ++i)
        for (int64_t j = bj * T; j < std::min(i, bj * T + T); ++j) out[i * n + j] = out[j * n + i];
}

// Split rows into chunks of about equal cell count for the host threads.
// Lower = the blocks' share grows with the index (mirror of a triangle).
template <class F>
void parallel_rows(int64_t n, F f, bool lower = false) {
  const int nt = (int)std::max<int64_t>(
      1, std::min<int64_t>(std::thread::hardware_concurrency(), std::max<int64_t>(1, lower ? n / 4 : n / 256)));
  if (nt == 1) {
    f(0, n);
    return;
  }
  std::vector<int64_t> cut(nt + 1, n);
  cut[0] = 0;
  const double tot = (double)tri_cells(n);
  int64_t i = 0;
  double acc = 0;
  for (int t = 1; t < nt; ++t) {
    while (i < n && acc < tot * t / nt) acc += (double)(lower ? i++ + 1 : n - i++);
    cut[t] = i;
  }
  std::vector<std::thread> th;
  for (int t = 0; t < nt; ++t)
    if (cut[t + 1] > cut[t]) th.emplace_back(f, cut[t], cut[t + 1]);
  for (auto& x : th) x.join();
}

}  // namespace

namespace sk {
// accessors into the context (sk_api.cpp)
hipStream_t ctx_stream(sk_context* ctx);
int ctx_device(sk_context* ctx);
void*& ctx_comm(sk_context* ctx);
int ctx_fail(sk_context* ctx, int code, const std::string& msg);

// What sk_comm_init leaves in the context: the communicator and the device
// status word of sk_gram_sharded's agreement, allocated together so that a
// sharded Gram has no failure point before its first collective.
struct CommState {
  ncclComm_t nc = nullptr;
  int32_t* d_st = nullptr;  // 2 words: this rank's -status, the all-reduced max
};

void comm_destroy(void* comm) {
  CommState* c = static_cast<CommState*>(comm);
  if (!c) return;
  if (c->nc) (void)ncclCommDestroy(c->nc);
  if (c->d_st) (void)hipFree(c->d_st);
  delete c;
}
}  // namespace sk

namespace {
sk::CommState* comm_of(sk_context* ctx) { return static_cast<sk::CommState*>(sk::ctx_comm(ctx)); }
}  // namespace

extern "C" {

int64_t sk_shard_count(int32_t n, int32_t rank, int32_t world) {
  if (n < 0 || world <= 0 || rank < 0 || rank >= world) return -1;
  const int64_t T = tri_cells(n);
  return T > rank ? (T - rank + world - 1) / world : 0;
}

int sk_shard_cells(int32_t n, int32_t rank, int32_t world, int32_t* x, int32_t* y) {
  if (n < 0 || world <= 0 || rank < 0 || rank >= world || !x || !y) return SK_ERR_INVALID;
  int64_t k = 0, m = 0;
  for (int32_t i = 0; i < n; ++i) {
    // first j >= i with (cell index) % world == rank
    const int64_t c0 = k;
    int64_t j0 = i + ((rank - c0 % world) % world + world) % world;
    for (int64_t j = j0; j < n; j += world) {
      x[m] = i;
      y[m] = (int32_t)j;
      ++m;
    }
    k += n - i;
  }
  return SK_OK;
}

int sk_shard_assemble(int32_t n, int32_t world, const double* gathered, int64_t per_rank,
                      int normalize, double* out) {
  if (n < 0 || world <= 0 || !out || (n > 0 && !gathered)) return SK_ERR_INVALID;
  if (per_rank < sk_shard_count(n, 0, world)) return SK_ERR_INVALID;
  if (n == 0) return SK_OK;
  std::vector<double> diag;
  if (normalize) {
    diag.resize(n);
    for (int64_t i = 0; i < n; ++i) {
      const int64_t k = i * (int64_t)n - i * (i - 1) / 2;
      diag[i] = gathered[(k % world) * per_rank + k / world];
    }
  }
  parallel_rows(n, [&](int64_t r0, int64_t r1) {
    upper_rows(n, world, gathered, per_rank, normalize ? diag.data() : nullptr, out, r0, r1);
  });
  const int64_t nb = (n + 63) / 64;
  parallel_rows(nb, [&](int64_t b0, int64_t b1) { mirror_blocks(n, out, b0, b1); }, true);
  return SK_OK;
}

int sk_comm_unique_id(uint8_t* id, size_t id_bytes) {
  if (!id || id_bytes < sizeof(ncclUniqueId)) return SK_ERR_INVALID;
  ncclUniqueId u;
  if (ncclGetUniqueId(&u) != ncclSuccess) return SK_ERR_HIP;
  std::memcpy(id, &u, sizeof(u));
  return SK_OK;
}

int sk_comm_init(sk_context* ctx, const uint8_t* id, size_t id_bytes, int32_t rank, int32_t world) {
  if (!ctx || !id || id_bytes < sizeof(ncclUniqueId) || world <= 0 || rank < 0 || rank >= world)
    return sk::ctx_fail(ctx, SK_ERR_INVALID, "sk_comm_init: bad argument");
  void*& c = sk::ctx_comm(ctx);
  sk::comm_destroy(c);
  c = nullptr;
  if (hipSetDevice(sk::ctx_device(ctx)) != hipSuccess)
    return sk::ctx_fail(ctx, SK_ERR_HIP, "sk_comm_init: hipSetDevice");
  // the status word first: a rank that fails here never joins the
  // communicator (its peers then wait in ncclCommInitRank, as for any rank
  // that never calls sk_comm_init); once joined, sk_gram_sharded allocates
  // nothing before its first collective
  sk::CommState* st = new sk::CommState;
  if (hipMalloc(&st->d_st, 2 * sizeof(int32_t)) != hipSuccess) {
    st->d_st = nullptr;
    sk::comm_destroy(st);
    return sk::ctx_fail(ctx, SK_ERR_ALLOC, "sk_comm_init: status word");
  }
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  const ncclResult_t r = ncclCommInitRank(&st->nc, world, u, rank);
  if (r != ncclSuccess) {
    st->nc = nullptr;
    sk::comm_destroy(st);
    return sk::ctx_fail(ctx, SK_ERR_HIP, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
  }
  c = st;
  return SK_OK;
}

int sk_comm_allgather(sk_context* ctx, const double* send_dev, int64_t count, double* recv_dev) {
  if (!ctx || count < 0 || (count > 0 && (!send_dev || !recv_dev)))
    return sk::ctx_fail(ctx, SK_ERR_INVALID, "sk_comm_allgather: bad argument");
  sk::CommState* c = comm_of(ctx);
  if (!c) return sk::ctx_fail(ctx, SK_ERR_INVALID, "sk_comm_allgather: no communicator (sk_comm_init)");
  const ncclResult_t r = ncclAllGather(send_dev, recv_dev, (size_t)count, ncclDouble, c->nc,
                                       sk::ctx_stream(ctx));
  if (r != ncclSuccess)
    return sk::ctx_fail(ctx, SK_ERR_HIP, std::string("ncclAllGather: ") + ncclGetErrorString(r));
  return SK_OK;
}

// Every rank enters every collective whatever its own status: a local
// failure (allocation, an unsupported example, a HIP error) is carried into
// the all-gather as a zero buffer and then agreed on by a max all-reduce of
// the ranks' status codes, so every rank returns an error instead of its
// peers waiting in ncclAllGather forever.
namespace {
int agree_status(sk_context* ctx, int rc) {
  hipStream_t S = sk::ctx_stream(ctx);
  int32_t h[2] = {-rc, 0};
  ncclComm_t c = comm_of(ctx)->nc;
  int32_t* d_st = comm_of(ctx)->d_st;
  if (hipMemcpyAsync(d_st, h, sizeof(int32_t), hipMemcpyHostToDevice, S) != hipSuccess ||
      ncclAllReduce(d_st, d_st + 1, 1, ncclInt32, ncclMax, c, S) != ncclSuccess ||
      hipMemcpyAsync(h + 1, d_st + 1, sizeof(int32_t), hipMemcpyDeviceToHost, S) != hipSuccess ||
      hipStreamSynchronize(S) != hipSuccess)
    return rc ? rc : sk::ctx_fail(ctx, SK_ERR_HIP, "sk_gram_sharded: status all-reduce");
  if (rc) return rc;
  if (h[1]) return sk::ctx_fail(ctx, -h[1], "sk_gram_sharded: another rank failed (status " +
                                              std::to_string(-h[1]) + ")");
  return SK_OK;
}
}  // namespace

int sk_gram_sharded(sk_context* ctx, sk_dataset* ds, const sk_kernel_params* kp, int normalize,
                    double* out) {
  if (!ctx || !ds || !kp || !out) return sk::ctx_fail(ctx, SK_ERR_INVALID, "null argument");
  sk::CommState* c = comm_of(ctx);
  if (!c) return sk::ctx_fail(ctx, SK_ERR_INVALID, "sk_gram_sharded: no communicator (sk_comm_init)");
  int world = 0, rank = 0;
  if (ncclCommCount(c->nc, &world) != ncclSuccess || ncclCommUserRank(c->nc, &rank) != ncclSuccess)
    return sk::ctx_fail(ctx, SK_ERR_HIP, "sk_gram_sharded: communicator query");
  const int32_t n = sk_dataset_size(ds);
  if (n < 0) return sk::ctx_fail(ctx, SK_ERR_INVALID, "sk_gram_sharded: dataset");
  const int64_t per = std::max<int64_t>(sk_shard_count(n, 0, world), 1);
  const int64_t mine = sk_shard_count(n, rank, world);
  std::vector<int32_t> x((size_t)mine), y((size_t)mine);
  int rc = sk_shard_cells(n, rank, world, x.data(), y.data());
  if (rc) return sk::ctx_fail(ctx, rc, "sk_gram_sharded: plan");
  hipStream_t S = sk::ctx_stream(ctx);
  double* d = nullptr;
  if (hipMalloc(&d, (size_t)per * (world + 1) * sizeof(double)) != hipSuccess) {
    d = nullptr;
    rc = sk::ctx_fail(ctx, SK_ERR_ALLOC, "sk_gram_sharded: device buffers");
  }
  rc = agree_status(ctx, rc);  // all ranks have their buffers (or all stop)
  std::vector<double> g;
  if (rc == SK_OK) {
    double* d_mine = d;
    double* d_all = d + per;
    int lrc = hipMemsetAsync(d_mine, 0, (size_t)per * sizeof(double), S) == hipSuccess
                  ? SK_OK
                  : sk::ctx_fail(ctx, SK_ERR_HIP, "sk_gram_sharded: memset");
    if (lrc == SK_OK && mine > 0) lrc = sk_pairs_device(ctx, ds, kp, x.data(), y.data(), mine, d_mine);
    if (lrc != SK_OK) (void)hipMemsetAsync(d_mine, 0, (size_t)per * sizeof(double), S);
    // the all-gather runs on every rank, failed or not
    const int grc = sk_comm_allgather(ctx, d_mine, per, d_all);
    rc = agree_status(ctx, lrc != SK_OK ? lrc : grc);
    if (rc == SK_OK) {
      g.resize((size_t)per * world);
      if (hipMemcpyAsync(g.data(), d_all, g.size() * sizeof(double), hipMemcpyDeviceToHost, S) !=
              hipSuccess ||
          hipStreamSynchronize(S) != hipSuccess)
        rc = sk::ctx_fail(ctx, SK_ERR_HIP, "sk_gram_sharded: gather copy");
    }
  }
  (void)hipStreamSynchronize(S);
  if (d) (void)hipFree(d);
  if (rc) return rc;
  return sk_shard_assemble(n, world, g.data(), per, normalize, out);
}

}  // extern "C"
