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
  // every packed array: the y-role records (SK_YBIG and their bases) and the
  // x-role / per-example arrays (SK_BIG, the ex_* vectors, the key tables)
#define PC_Y(X) X(yn_a) X(yn_b) X(yn_c) X(ye2) X(ysc) X(yrec) X(yn_w) X(yn_nbp) X(yn_p0) X(yn_P) X(ycs) \
  X(ex_ysc_base) X(ex_nch) X(ex_ycs_base)
#define PC_X(X) X(nd_a) X(nd_b) X(nd_c) X(nd_w) X(nd_nbp) X(nd_P) X(ed) X(bpf_code) X(bpf_p) X(lvl)      \
  X(xr_ch) X(xrow) X(xr_node) X(gr_info) X(gr_pf) X(gr_P) X(xg_ch) X(xg_clg) X(xg_cpf) X(xg_cty)          \
  X(phk_idx) X(gra_gidx) X(gra_row) X(xgrow) X(xg_node) X(pos_prof) X(pos_w) X(pos_chr) X(pos_lru)        \
  X(ex_phi_bits) X(ex_nl) X(ex_node_base) X(ex_edge_base) X(ex_bpf_base) X(ex_lvl_base) X(ex_nlev)        \
  X(ex_len) X(ex_pos_base) X(ex_has_w) X(ex_dyadic) X(ex_str_fast) X(ex_onehot) X(ex_big) X(ex_nseqs)     \
  X(ex_nslots) X(ex_xch_base) X(gam_key) X(ex_xg_base) X(ex_nlxg) X(ex_xgch_base) X(ex_gr_base)           \
  X(ex_gapless) X(phi_al) X(phi_g) X(ex_gra_base) X(ex_phk_base)
  uint64_t h = 1469598103934665603ull, hx = h;
  const bool each = std::getenv("PC_EACH") != nullptr;  // one line per array (bisecting a mismatch)
#define PC_HY(f) h = hv(P.f, h); if (each) printf("  %s %016llx\n", #f, (unsigned long long)hv(P.f, 1469598103934665603ull));
#define PC_HX(f) hx = hv(P.f, hx); if (each) printf("  %s %016llx\n", #f, (unsigned long long)hv(P.f, 1469598103934665603ull));
  PC_Y(PC_HY)
  PC_X(PC_HX)
  printf("rc=%d n=%d L=%d pack %.3f s  y-hash %016llx  x-hash %016llx max_nch %d\n", rc, n, L,
         std::chrono::duration<double>(t2 - t1).count(), (unsigned long long)h, (unsigned long long)hx, P.max_nch);
}
