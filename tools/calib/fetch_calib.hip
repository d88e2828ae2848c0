// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE for the access widths
// the engine's kernels use (MI355X_MICROARCH.md: FETCH_SIZE counts half the
// bytes of a 16-B-per-lane streaming read; other widths uncalibrated).
// Reads (or writes) a 1 GiB buffer -- four times the 256 MiB Infinity Cache --
// once, coalesced, with 8 or 16 bytes per lane; the counters of each launch
// are compared with the 1 GiB it moves (tools/calib/run.sh).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

__global__ void read8(const double* __restrict__ a, size_t n, double* out) {
  double s = 0.0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    s += a[i];
  if (s == 12345.678) out[0] = s;  // keeps the loads
}

__global__ void read16(const double2* __restrict__ a, size_t n, double* out) {
  double s = 0.0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const double2 v = a[i];
    s += v.x + v.y;
  }
  if (s == 12345.678) out[0] = s;
}

__global__ void write8(double* __restrict__ a, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    a[i] = (double)i;
}

// scattered 8-B reads (the DAG kernel's node / edge record accesses): one
// double per `stride`-element line of the buffer, the lines visited in a
// permuted order (odd multiplier mod a power of two: every line once), so
// each load is a separate request to a line no other load touches
__global__ void read8_scatter(const double* __restrict__ a, size_t lines, size_t stride, double* out) {
  double s = 0.0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < lines; i += (size_t)gridDim.x * blockDim.x)
    s += a[((i * 0x9E3779B1ull) & (lines - 1)) * stride];
  if (s == 12345.678) out[0] = s;
}

// the same coalesced 8-B read under two names, so the two passes of the
// re-read case are told apart in the per-dispatch counter file
__global__ void reread_1(const double* __restrict__ a, size_t n, double* out) {
  double s = 0.0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    s += a[i];
  if (s == 12345.678) out[0] = s;
}
__global__ void reread_2(const double* __restrict__ a, size_t n, double* out) {
  double s = 0.0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    s += a[i];
  if (s == 12345.678) out[0] = s;
}

int main() {
  const size_t bytes = (size_t)1 << 30;
  double* a = nullptr;
  double* out = nullptr;
  if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
  const size_t n8 = bytes / 8;
  hipLaunchKernelGGL(write8, dim3(4096), dim3(256), 0, 0, a, n8);
  hipLaunchKernelGGL(read8, dim3(4096), dim3(256), 0, 0, a, n8, out);
  hipLaunchKernelGGL(read16, dim3(4096), dim3(256), 0, 0, reinterpret_cast<const double2*>(a), n8 / 2, out);
  // one 8-B load per 128-B line and per 64-B line: 8 MiB / 16 MiB of loaded
  // bytes touching every line of the 1 GiB once
  hipLaunchKernelGGL(read8_scatter, dim3(4096), dim3(256), 0, 0, a, n8 / 16, (size_t)16, out);
  hipLaunchKernelGGL(read8_scatter, dim3(4096), dim3(256), 0, 0, a, n8 / 8, (size_t)8, out);
  // re-read of a table that fits the 256 MiB Infinity Cache but not the L2
  // (4 MiB per XCD): a 64 MiB table written, a 1 GiB stream read to evict it,
  // then the table read twice back to back (reread_1: from HBM; reread_2:
  // the Infinity Cache holds it) -- the DAG kernel's child rows are read
  // 2.8 times on average.  Equal FETCH_SIZE for the two passes means the
  // counter counts Infinity-Cache hits as fetched bytes.
  const size_t tb = (size_t)64 << 20;
  double* t = nullptr;
  if (hipMalloc(&t, tb) != hipSuccess) return 1;
  hipLaunchKernelGGL(write8, dim3(4096), dim3(256), 0, 0, t, tb / 8);
  hipLaunchKernelGGL(read8, dim3(4096), dim3(256), 0, 0, a, n8, out);
  hipLaunchKernelGGL(reread_1, dim3(4096), dim3(256), 0, 0, t, tb / 8, out);
  hipLaunchKernelGGL(reread_2, dim3(4096), dim3(256), 0, 0, t, tb / 8, out);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  std::printf("moved %zu bytes per launch (write8, read8, read16); read8_scatter: one 8-B load per 128-B "
              "line (%zu loads), then per 64-B line (%zu loads); reread_1 / reread_2: a %zu-byte table "
              "read twice after a 1 GiB eviction stream\n", bytes, n8 / 16, n8 / 8, tb);
  (void)hipFree(t);
  (void)hipFree(a);
  (void)hipFree(out);
  return 0;
}
