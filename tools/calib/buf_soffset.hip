// Does the raw-buffer range check on gfx950 include the SGPR offset?
// Loads lane * 8 + soffset from a descriptor of `bytes` records over a
// buffer of 1..512 doubles (value = index + 1), and stores likewise; prints
// which lanes returned data / wrote.  A calibration probe for the 4-D column
// kernel's row descriptors, not part of the library.
//   hipcc --offload-arch=gfx950 -O2 tools/calib/buf_soffset.hip -o tools/calib/buf_soffset
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void probe(const double* src, double* out, double* dst, int bytes, int soff) {
  const int lane = threadIdx.x;
  const auto r = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, bytes, 0x00020000);
  out[lane] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, lane * 8, soff, 0));
  const auto w = __builtin_amdgcn_make_buffer_rsrc((void*)dst, (short)0, bytes, 0x00020000);
  typedef unsigned int u2 __attribute__((__vector_size__(2 * sizeof(unsigned int))));
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, 1000.0 + lane), w, lane * 8, soff, 0);
}

int main() {
  double *src, *out, *dst;
  if (hipMalloc(&src, 512 * 8) || hipMalloc(&out, 64 * 8) || hipMalloc(&dst, 512 * 8)) return 1;
  double h[512];
  for (int k = 0; k < 512; ++k) h[k] = k + 1;
  if (hipMemcpy(src, h, sizeof h, hipMemcpyHostToDevice)) return 1;
  const int cases[][2] = {{80, 0}, {80, 64}, {80, 256}, {800, 256}};
  for (auto& cs : cases) {
    if (hipMemset(dst, 0, 512 * 8)) return 1;
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, src, out, dst, cs[0], cs[1]);
    if (hipDeviceSynchronize()) return 2;
    double o[64], d[512];
    if (hipMemcpy(o, out, sizeof o, hipMemcpyDeviceToHost) || hipMemcpy(d, dst, sizeof d, hipMemcpyDeviceToHost)) return 3;
    int nl = 0, nw = 0, first = -1;
    for (int l = 0; l < 64; ++l) nl += o[l] != 0.0;
    for (int k = 0; k < 512; ++k)
      if (d[k] != 0.0) {
        ++nw;
        if (first < 0) first = k;
      }
    printf("bytes %d soffset %d: loads returning data %d (lane0 %.0f), stores landed %d (first at %d)\n", cs[0], cs[1],
           nl, o[0], nw, first);
  }
  return 0;
}
