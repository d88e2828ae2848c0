// Host preprocessing for one example: profile, averaged bp matrix, per-row
// unpaired probabilities and the stem DAG.  Restates the reference's
//   MData(ma, th, pf_scale, opts)   stem_kernel_lite/data.cpp:324-345
//   Profiler                        stem_kernel_lite/data.cpp:33-132
//   DAGBuilder                      stem_kernel_lite/data.cpp:141-307
//   find_root / find_max_parent     stem_kernel_lite/data.cpp:396-435
//   fill_weight                     stem_kernel_lite/data.cpp:437-453
//   average_matrix                  common/bpmatrix.cpp:306-342
// with the same float/double intermediates, so node order, edge order,
// node weights and bp frequencies come out bit-identical.  Unlike the
// reference, candidate lists are kept for two CYK columns only (the
// recurrence reads column j and j-1) and the DAG is emitted straight into CSR.
#include <algorithm>
#include <cctype>
#include <cstring>
#include <stdexcept>

#include "sk_internal.h"

namespace sk {

namespace {
constexpr uint32_t kNone = 0xffffffffu;
constexpr int kGap = 4;

const char kSym[17] = {'a', 'c', 'g', 'u', 't', '-', 'r', 'y', 'm',
                       'k', 's', 'w', 'b', 'd', 'h', 'v', 'n'};
const unsigned char kCode[17] = {0, 1, 2, 3, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15};
}  // namespace

const float kIupac[16][4] = {
    {1.0f, 0.0f, 0.0f, 0.0f},       {0.0f, 1.0f, 0.0f, 0.0f},       {0.0f, 0.0f, 1.0f, 0.0f},
    {0.0f, 0.0f, 0.0f, 1.0f},       {0.0f, 0.0f, 0.0f, 0.0f},       {0.5f, 0.0f, 0.5f, 0.0f},
    {0.0f, 0.5f, 0.0f, 0.5f},       {0.5f, 0.5f, 0.0f, 0.0f},       {0.0f, 0.0f, 0.5f, 0.5f},
    {0.0f, 0.5f, 0.5f, 0.0f},       {0.5f, 0.0f, 0.0f, 0.5f},       {0.0f, float(1.0 / 3), float(1.0 / 3), float(1.0 / 3)},
    {float(1.0 / 3), 0.0f, float(1.0 / 3), float(1.0 / 3)},        {float(1.0 / 3), float(1.0 / 3), 0.0f, float(1.0 / 3)},
    {float(1.0 / 3), float(1.0 / 3), float(1.0 / 3), 0.0f},        {0.25f, 0.25f, 0.25f, 0.25f},
};

int char2rna(int c) {
  const char r = (char)std::tolower(c);
  for (int k = 0; k < 17; ++k)
    if (kSym[k] == r) return kCode[k];
  return kGap;
}

namespace {

// A read-only view of a packed strict-upper-triangle bp matrix, 1-based access.
struct BpView {
  const double* p = nullptr;
  int n = 0;
  double operator()(int i1, int j1) const { return p[tri_index(n, i1 - 1, j1 - 1)]; }
};

// Per-row profile helper (the reference's Profiler).
struct RowProfile {
  const std::string* seq = nullptr;
  BpView bpm;
  float w = 1.0f;
  std::vector<float> col;       // [len][5]
  std::vector<uint32_t> idx;    // aligned pos -> row pos
  std::vector<float> nbp;       // unpaired probability (float arithmetic)

  void init(const std::string& s, BpView m) {
    seq = &s;
    bpm = m;
    const int len = (int)s.size();
    col.assign((size_t)len * 5, 0.0f);
    for (int i = 0; i < len; ++i) {
      const int r = char2rna((unsigned char)s[i]);
      if (r != kGap) {
        for (int a = 0; a < 4; ++a) col[i * 5 + a] += kIupac[r][a] * 1.0f;
      } else {
        col[i * 5 + kGap] += 1.0f;
      }
    }
    idx.assign(len, kNone);
    uint32_t k = 0;
    for (int i = 0; i < len; ++i)
      if (s[i] != '-') idx[i] = k++;
    nbp.assign(len, 1.0f);
    const bool mapped = bpm.n != len;
    for (int i = 0; i < len; ++i) {
      if (idx[i] == kNone) continue;
      for (int j = 0; j < len; ++j) {
        if (j == i || idx[j] == kNone) continue;
        const int a = j < i ? j : i, b = j < i ? i : j;
        nbp[i] -= mapped ? bpm(idx[a] + 1, idx[b] + 1) : bpm(a + 1, b + 1);
      }
      if (nbp[i] < 0.0) nbp[i] = 0.0f;
    }
  }
  float loop(int i) const { return w * nbp[i]; }
};

struct Pos {
  uint32_t a, b;
};
using PosList = std::vector<Pos>;

class DagBuilder {
 public:
  DagBuilder(const std::vector<RowProfile>& prof, BpView bpm, float th, Example& ex)
      : prof_(prof), bpm_(bpm), th_(th), n_(bpm.n), ex_(ex) {}

  void run() {
    scan();
    visit_.assign((size_t)n_ * (n_ + 1) / 2, kNone);
    ex_.edge_off.assign(1, 0);
    ex_.bpf_off.assign(1, 0);
    for (int i = 0; i < n_; ++i)
      for (auto it = head_[i].rbegin(); it != head_[i].rend(); ++it) visit(it->a, it->b);
  }

 private:
  static size_t cell(int i, int j) { return (size_t)j * (j + 1) / 2 + (size_t)i; }

  // Bottom-up scan of the bp matrix (DAGBuilder::initialize, data.cpp:165-191).
  // cand[i] holds ch(i, j) for the current column j, prev[i] ch(i, j-1).
  void scan() {
    head_.assign(n_, PosList());
    kids_.assign((size_t)n_ * (n_ + 1) / 2, PosList());
    std::vector<PosList> cur(n_ + 1), prev(n_ + 1);
    for (int j = 1; j < n_; ++j) {
      for (int i = 0; i <= n_; ++i) cur[i].clear();
      for (int i = j - 1; i >= 0; --i) {
        if (bpm_(i + 1, j + 1) >= (double)th_) {
          // the pair's children are the candidates of (i+1, j-1)
          if (i + 1 <= j - 1) kids_[cell(i, j)].swap(prev[i + 1]);
          cur[i].push_back(Pos{(uint32_t)i, (uint32_t)j});
          head_[i].push_back(Pos{(uint32_t)i, (uint32_t)j});
        } else {
          const uint32_t hb = head_[i].empty() ? 0u : head_[i].back().b;
          const PosList& below = cur[i + 1];  // ch(i+1, j); empty on the diagonal
          PosList& out = cur[i];
          out.reserve(below.size() + head_[i].size());
          for (const Pos& c : below)
            if (!(hb > c.b)) out.push_back(c);
          out.insert(out.end(), head_[i].begin(), head_[i].end());
        }
      }
      std::swap(cur, prev);
    }
  }

  float loop_profile(int i) const {
    float v = 0.0f, t = 0.0f;
    for (const RowProfile& p : prof_) {
      if (p.idx[i] != kNone) v += p.loop(i);
      t += p.w;
    }
    return v / t;
  }

  void bp_freq(int i, int j) {
    bool have[16] = {false};
    float acc[16] = {0.0f};
    float t = 0.0f;
    for (const RowProfile& p : prof_) {
      if (p.idx[i] != kNone && p.idx[j] != kNone) {
        const bool mapped = p.bpm.n != (int)p.seq->size();
        const float pr = (float)(mapped ? p.bpm(p.idx[i] + 1, p.idx[j] + 1) : p.bpm(i + 1, j + 1));
        for (int a = 0; a < 4; ++a) {
          if (p.col[i * 5 + a] == 0.0) continue;
          for (int b = 0; b < 4; ++b) {
            if (p.col[j * 5 + b] == 0.0) continue;
            const float add = p.w * pr * p.col[i * 5 + a] * p.col[j * 5 + b];
            const int k = a * 4 + b;
            acc[k] = have[k] ? acc[k] + add : add;
            have[k] = true;
          }
        }
      }
      t += p.w;
    }
    for (int k = 0; k < 16; ++k)
      if (have[k]) {
        ex_.bpf_code.push_back((uint8_t)k);
        ex_.bpf_p.push_back(acc[k] / t);
      }
  }

  uint32_t emit(uint32_t a, uint32_t b, float w) {
    ex_.first.push_back(a);
    ex_.last.push_back(b);
    ex_.weight.push_back(w);
    ex_.edge_off.push_back((uint32_t)ex_.edge_to.size());
    ex_.bpf_off.push_back((uint32_t)ex_.bpf_code.size());
    return (uint32_t)ex_.first.size() - 1;
  }

  // post-order construction (build_helper / make_leaf / make_loop / make_stem,
  // data.cpp:193-244); returns the node id of (a, b).
  uint32_t visit(uint32_t a, uint32_t b) {
    uint32_t& slot = visit_[cell((int)a, (int)b)];
    if (slot != kNone) return slot;
    if (a == b) {
      slot = emit(a, b, 1.0f);
      return slot;
    }
    const PosList& kids = kids_[cell((int)a, (int)b)];
    // children first: their subtrees precede this node in the numbering
    std::vector<uint32_t> to, gaps;
    if (kids.empty()) {
      to.push_back(visit(a, a));
      gaps.push_back(b - a - 1);
    } else {
      for (const Pos& c : kids) {
        to.push_back(visit(c.a, c.b));
        gaps.push_back((c.a - a - 1) + (b - c.b - 1));
      }
    }
    const float w = loop_profile((int)a) * loop_profile((int)b);
    ex_.edge_to.insert(ex_.edge_to.end(), to.begin(), to.end());
    ex_.edge_gaps.insert(ex_.edge_gaps.end(), gaps.begin(), gaps.end());
    bp_freq((int)a, (int)b);
    // emit() records the CSR end offsets after the pushes above
    slot = emit(a, b, w);
    return slot;
  }

  const std::vector<RowProfile>& prof_;
  BpView bpm_;
  float th_;
  int n_;
  Example& ex_;
  std::vector<PosList> head_;
  std::vector<PosList> kids_;
  std::vector<uint32_t> visit_;
};

}  // namespace

void build_example(Example& ex, int n_rows, const char* const* rows,
                   const double* const* bpp_rows, float th, bool use_bp) {
  if (n_rows <= 0) throw std::invalid_argument("example without rows");
  ex = Example();
  ex.n_rows = n_rows;
  ex.len = (int)std::strlen(rows[0]);
  for (int r = 0; r < n_rows; ++r) {
    ex.rows.emplace_back(rows[r]);
    if ((int)ex.rows.back().size() != ex.len) throw std::invalid_argument("wrong alignment");
  }
  const int L = ex.len;
  ex.prof5.assign((size_t)L * 5, 0.0f);
  for (int r = 0; r < n_rows; ++r) {
    for (int i = 0; i < L; ++i) {
      const int c = char2rna((unsigned char)rows[r][i]);
      if (c != kGap) {
        for (int a = 0; a < 4; ++a) ex.prof5[i * 5 + a] += kIupac[c][a] * 1.0f;
      } else {
        ex.prof5[i * 5 + kGap] += 1.0f;
      }
    }
    ex.n_seqs += 1.0f;
  }
  ex.has_bp = use_bp;
  ex.edge_off.assign(1, 0);
  ex.bpf_off.assign(1, 0);
  if (!use_bp) return;

  // averaged matrix over the aligned columns (rows summed in order, then /n)
  ex.bpp.assign(L > 1 ? (size_t)L * (L - 1) / 2 : 0, 0.0);
  std::vector<BpView> row_views(n_rows);
  for (int r = 0; r < n_rows; ++r) {
    std::vector<int> map(L, -1);
    int nr = 0;
    for (int i = 0; i < L; ++i)
      if (rows[r][i] != '-') map[i] = nr++;
    row_views[r] = BpView{bpp_rows[r], nr};
    for (int j = 1; j < L; ++j) {
      if (map[j] < 0) continue;
      for (int i = j - 1; i >= 0; --i)
        if (map[i] >= 0) ex.bpp[tri_index(L, i, j)] += row_views[r](map[i] + 1, map[j] + 1);
    }
  }
  for (double& v : ex.bpp) v = v / n_rows;
  const BpView avg{ex.bpp.data(), L};

  std::vector<RowProfile> prof(n_rows);
  for (int r = 0; r < n_rows; ++r) prof[r].init(ex.rows[r], n_rows > 1 ? row_views[r] : avg);

  DagBuilder(prof, avg, th, ex).run();

  const int n = ex.n_nodes();
  std::vector<char> has_parent(n, 0);
  ex.max_pa.assign(n, kNone);
  for (int v = 0; v < n; ++v)
    for (uint32_t e = ex.edge_off[v]; e < ex.edge_off[v + 1]; ++e) {
      const uint32_t c = ex.edge_to[e];
      has_parent[c] = 1;
      if (ex.max_pa[c] == kNone || ex.max_pa[c] < (uint32_t)v) ex.max_pa[c] = (uint32_t)v;
    }
  for (int v = 0; v < n; ++v)
    if (!has_parent[v]) ex.roots.push_back((uint32_t)v);

  ex.pos_weight.assign(L, 0.0f);
  for (int i = 0; i < L; ++i) {
    float v = 0.0f, t = 0.0f;
    for (const RowProfile& p : prof) {
      if (p.idx[i] != kNone) v += p.loop(i);
      t += p.w;
    }
    ex.pos_weight[i] = v / t;
  }
}

}  // namespace sk
