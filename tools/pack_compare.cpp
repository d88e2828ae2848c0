// Host packing check (CPU only): build with two versions of sk_api.cpp and
// compare the hashes of the packed arrays and the pack time, e.g.
//   git show HEAD~1:stem_kernel_amd/csrc/sk_api.cpp > /tmp/old.cpp
//   hipcc -O3 -std=c++17 -Iinclude -Istem_kernel_amd/csrc -D__HIP_PLATFORM_AMD__ '-DSRC="/tmp/old.cpp"' \
//     tools/pack_compare.cpp -o /tmp/pc_old -Lstem_kernel_amd -lstem_kernel_amd -Wl,-rpath,$PWD/stem_kernel_amd -L/opt/rocm/lib -lrccl
//   /tmp/pc_old 2048 200   (likewise with -DSRC=... the tree's sk_api.cpp)
#include SRC
#include <chrono>
template <class V> static uint64_t hv(const V& v, uint64_t h) {
  typedef typename V::value_type T;
  const unsigned char* p = reinterpret_cast<const unsigned char*>(v.data());
  for (size_t i = 0; i < v.size() * sizeof(T); ++i) h = (h ^ p[i]) * 1099511628211ull;
  return h ^ v.size();
}
int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 512;
  const int L = argc > 2 ? atoi(argv[2]) : 200;
  sk_dataset* ds = nullptr;
  sk_dataset_create(&ds);
  uint64_t st = 0x5EED0001ull;
  std::vector<char> buf((size_t)n * (L + 1));
  sk_random_sequences(&st, n, L, buf.data());
  std::vector<std::string> ss(n);
  std::vector<const char*> sp(n);
  for (int i = 0; i < n; ++i) { ss[i].assign(&buf[(size_t)i * (L + 1)], L); sp[i] = ss[i].c_str(); }
  int rc = sk_dataset_add_synthetic(ds, n, sp.data(), nullptr, 0.01f, 8);
  std::string err;
  auto t1 = std::chrono::steady_clock::now();
  rc |= pack_dataset(ds, err);
  auto t2 = std::chrono::steady_clock::now();
  const HostPack& P = ds->pack;
  uint64_t h = 1469598103934665603ull, hx = h;
  const bool each = std::getenv("PC_EACH") != nullptr;  // one line per array (bisecting a mismatch)
#define PC_HY(f) h = hv(P.f, h); if (each) printf("  %s %016llx\n", #f, (unsigned long long)hv(P.f, 1469598103934665603ull));
#define PC_HX(f) hx = hv(P.f, hx); if (each) printf("  %s %016llx\n", #f, (unsigned long long)hv(P.f, 1469598103934665603ull));
  SK_PACK_Y_ARRAYS(PC_HY)
  SK_PACK_X_ARRAYS(PC_HX)
  printf("rc=%d n=%d L=%d pack %.3f s  y-hash %016llx  x-hash %016llx max_nch %d\n", rc, n, L,
         std::chrono::duration<double>(t2 - t1).count(), (unsigned long long)h, (unsigned long long)hx, P.max_nch);
}
