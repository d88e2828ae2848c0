// Portions (multiclass_probability below keeps libsvm's operation order, and
// so its structure and names, for bit-compatible probabilities) derive from
// LIBSVM:
//   Copyright (c) 2000-2007 Chih-Chung Chang and Chih-Jen Lin.
//   All rights reserved.
//   Redistribution and use in source and binary forms, with or without
//   modification, are permitted provided that the following conditions are
//   met: 1. Redistributions of source code must retain the above copyright
//   notice, this list of conditions and the following disclaimer.
//   2. Redistributions in binary form must reproduce the above copyright
//   notice, this list of conditions and the following disclaimer in the
//   documentation and/or other materials provided with the distribution.
//   3. Neither name of copyright holders nor the names of its contributors
//   may be used to endorse or promote products derived from this software
//   without specific prior written permission.
//   THIS SOFTWARE IS PROVIDED BY THE COPYRIGHT HOLDERS AND CONTRIBUTORS "AS
//   IS" AND ANY EXPRESS OR IMPLIED WARRANTIES, INCLUDING, BUT NOT LIMITED TO,
//   THE IMPLIED WARRANTIES OF MERCHANTABILITY AND FITNESS FOR A PARTICULAR
//   PURPOSE ARE DISCLAIMED.  IN NO EVENT SHALL THE REGENTS OR CONTRIBUTORS BE
//   LIABLE FOR ANY DIRECT, INDIRECT, INCIDENTAL, SPECIAL, EXEMPLARY, OR
//   CONSEQUENTIAL DAMAGES (INCLUDING, BUT NOT LIMITED TO, PROCUREMENT OF
//   SUBSTITUTE GOODS OR SERVICES; LOSS OF USE, DATA, OR PROFITS; OR BUSINESS
//   INTERRUPTION) HOWEVER CAUSED AND ON ANY THEORY OF LIABILITY, WHETHER IN
//   CONTRACT, STRICT LIABILITY, OR TORT (INCLUDING NEGLIGENCE OR OTHERWISE)
//   ARISING IN ANY WAY OUT OF THE USE OF THIS SOFTWARE, EVEN IF ADVISED OF
//   THE POSSIBILITY OF SUCH DAMAGE.
//
// libsvm prediction for predict mode's Output (f3): the reference's
// SVMPredict (libsvm/svm_util.{h,cpp}) over its vendored libsvm 2.8x
// (libsvm/svm.cpp, libsvm/qmatrix.cpp), restated from the published
// algorithm:
//   svm_load_model        svm.cpp:1288-1475  (text model: header keywords, then
//                                             "coef.. idx:value .." SV lines)
//   svm_predict_values    svm.cpp:1053-1106  (one-vs-one decision values)
//   svm_predict           svm.cpp:1108-1150  (votes; one-class sign; SVR value)
//   svm_predict_probability svm.cpp:1152-1189 (Platt sigmoid per pair, clipped
//                                             to [1e-7, 1-1e-7], pairwise
//                                             coupling)
//   sigmoid_predict       svm.cpp:416-423
//   multiclass_probability svm.cpp:426-488   (Wu, Lin and Weng's method 2)
//   Kernel::k_function    qmatrix.cpp:244-302 (linear, poly, rbf, sigmoid,
//                                             precomputed: x[(int)sv.value])
//   SVMPredict::make_svm_node svm_util.cpp:84-95 (x[0] = {0, cnt}, x[i+1] =
//                                             {i+1, row[i]})
//   SVMPredict::do_svm_predict svm_util.cpp:41-80 (probability output for
//                                             C-SVC / nu-SVC, else decision
//                                             values)
// Host code only: a test row's kernel values come from the GPU engine; this
// is O(#SV) arithmetic per row.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <fstream>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include "../../../include/stem_kernel.h"

namespace {
struct SvmNode {  // svm_node (libsvm/svm.h:9-13)
  int index;
  double value;
};
}  // namespace

struct sk_svm_model {
  int svm_type = -1, kernel_type = -1, degree = 3;
  double gamma = 0.0, coef0 = 0.0;
  int nr_class = 0, l = 0;
  std::vector<double> rho, probA, probB;
  std::vector<int> label, nSV;
  std::vector<std::vector<double>> sv_coef;  // [nr_class - 1][l]
  std::vector<std::vector<SvmNode>> SV;  // each terminated by index -1
};

namespace {

thread_local std::string g_err;

const char* const kSvmTypes[] = {"c_svc", "nu_svc", "one_class", "epsilon_svr", "nu_svr"};
const char* const kKernelTypes[] = {"linear", "polynomial", "rbf", "sigmoid", "precomputed"};

int lookup(const std::string& s, const char* const* table, int n) {
  for (int i = 0; i < n; ++i)
    if (s == table[i]) return i;
  return -1;
}

double sparse_dot(const SvmNode* x, const SvmNode* y) {
  double s = 0.0;
  while (x->index != -1 && y->index != -1) {
    if (x->index == y->index) {
      s += x->value * y->value;
      ++x;
      ++y;
    } else if (x->index > y->index) {
      ++y;
    } else {
      ++x;
    }
  }
  return s;
}

double powi(double base, int times) {  // integer power by squaring
  double tmp = base, ret = 1.0;
  for (int t = times; t > 0; t /= 2) {
    if (t % 2 == 1) ret *= tmp;
    tmp *= tmp;
  }
  return ret;
}

// k(x, sv); x holds positions 0..n (x[i].index == i) for the precomputed
// kernel, whose SV value is the 1-based training index
double k_function(const sk_svm_model& m, const SvmNode* x, int nx, const SvmNode* y, bool& ok) {
  switch (m.kernel_type) {
    case 0:
      return sparse_dot(x, y);
    case 1:
      return powi(m.gamma * sparse_dot(x, y) + m.coef0, m.degree);
    case 2: {
      double s = 0.0;
      while (x->index != -1 && y->index != -1) {
        if (x->index == y->index) {
          const double d = x->value - y->value;
          s += d * d;
          ++x;
          ++y;
        } else if (x->index > y->index) {
          s += y->value * y->value;
          ++y;
        } else {
          s += x->value * x->value;
          ++x;
        }
      }
      for (; x->index != -1; ++x) s += x->value * x->value;
      for (; y->index != -1; ++y) s += y->value * y->value;
      return std::exp(-m.gamma * s);
    }
    case 3:
      return std::tanh(m.gamma * sparse_dot(x, y) + m.coef0);
    case 4: {
      const int k = (int)y->value;
      if (k < 0 || k >= nx) {
        ok = false;
        return 0.0;
      }
      return x[k].value;
    }
    default:
      ok = false;
      return 0.0;
  }
}

bool regression_like(const sk_svm_model& m) { return m.svm_type >= 2; }  // one-class, SVRs

bool decision_values(const sk_svm_model& m, const SvmNode* x, int nx, double* dec) {
  bool ok = true;
  if (regression_like(m)) {
    double sum = 0.0;
    for (int i = 0; i < m.l; ++i) sum += m.sv_coef[0][i] * k_function(m, x, nx, m.SV[i].data(), ok);
    dec[0] = sum - m.rho[0];
    return ok;
  }
  std::vector<double> kv(m.l);
  for (int i = 0; i < m.l; ++i) kv[i] = k_function(m, x, nx, m.SV[i].data(), ok);
  std::vector<int> start(m.nr_class, 0);
  for (int i = 1; i < m.nr_class; ++i) start[i] = start[i - 1] + m.nSV[i - 1];
  int p = 0;
  for (int i = 0; i < m.nr_class; ++i)
    for (int j = i + 1; j < m.nr_class; ++j) {
      // pair (i, j): class i's SVs weighted by their coefficient row j-1,
      // class j's by row i
      double sum = 0.0;
      const std::vector<double>& ci = m.sv_coef[j - 1];
      const std::vector<double>& cj = m.sv_coef[i];
      for (int k = 0; k < m.nSV[i]; ++k) sum += ci[start[i] + k] * kv[start[i] + k];
      for (int k = 0; k < m.nSV[j]; ++k) sum += cj[start[j] + k] * kv[start[j] + k];
      dec[p] = sum - m.rho[p];
      ++p;
    }
  return ok;
}

double predict_label(const sk_svm_model& m, const double* dec) {
  if (regression_like(m)) return m.svm_type == 2 ? (dec[0] > 0 ? 1.0 : -1.0) : dec[0];
  std::vector<int> vote(m.nr_class, 0);
  int pos = 0;
  for (int i = 0; i < m.nr_class; ++i)
    for (int j = i + 1; j < m.nr_class; ++j) {
      if (dec[pos++] > 0) ++vote[i];
      else ++vote[j];
    }
  int best = 0;
  for (int i = 1; i < m.nr_class; ++i)
    if (vote[i] > vote[best]) best = i;
  return m.label[best];
}

double sigmoid_predict(double dv, double A, double B) {
  const double f = dv * A + B;
  return f >= 0 ? std::exp(-f) / (1.0 + std::exp(-f)) : 1.0 / (1.0 + std::exp(f));
}

// Wu, Lin and Weng's method 2: minimise p^T Q p over the simplex by
// coordinate updates until every |(Qp)_t - p^T Q p| < 0.005 / k
void multiclass_probability(int k, const std::vector<std::vector<double>>& r, double* p) {
  const int max_iter = std::max(100, k);
  std::vector<std::vector<double>> Q(k, std::vector<double>(k, 0.0));
  std::vector<double> Qp(k);
  const double eps = 0.005 / k;
  for (int t = 0; t < k; ++t) {
    p[t] = 1.0 / k;
    Q[t][t] = 0.0;
    for (int j = 0; j < t; ++j) {
      Q[t][t] += r[j][t] * r[j][t];
      Q[t][j] = Q[j][t];
    }
    for (int j = t + 1; j < k; ++j) {
      Q[t][t] += r[j][t] * r[j][t];
      Q[t][j] = -r[j][t] * r[t][j];
    }
  }
  for (int iter = 0; iter < max_iter; ++iter) {
    double pQp = 0.0;
    for (int t = 0; t < k; ++t) {
      Qp[t] = 0.0;
      for (int j = 0; j < k; ++j) Qp[t] += Q[t][j] * p[j];
      pQp += p[t] * Qp[t];
    }
    double max_error = 0.0;
    for (int t = 0; t < k; ++t) max_error = std::max(max_error, std::fabs(Qp[t] - pQp));
    if (max_error < eps) break;
    for (int t = 0; t < k; ++t) {
      const double diff = (-Qp[t] + pQp) / Q[t][t];
      p[t] += diff;
      pQp = (pQp + diff * (diff * Q[t][t] + 2 * Qp[t])) / (1 + diff) / (1 + diff);
      for (int j = 0; j < k; ++j) {
        Qp[j] = (Qp[j] + diff * Q[t][j]) / (1 + diff);
        p[j] /= (1 + diff);
      }
    }
  }
}

int fail(const std::string& msg) {
  g_err = msg;
  return SK_ERR_INVALID;
}

}  // namespace

extern "C" {

int sk_svm_model_load(const char* path, sk_svm_model** out) {
  if (!path || !out) return fail("null argument");
  *out = nullptr;
  std::ifstream in(path);
  if (!in) return fail(std::string(path) + ": no such file");
  std::unique_ptr<sk_svm_model> m(new sk_svm_model());
  std::string cmd;
  bool sv_section = false;
  while (in >> cmd) {
    const int npair = m->nr_class * (m->nr_class - 1) / 2;
    auto read_vec = [&](std::vector<double>& v, int n) {
      v.resize(n);
      for (int i = 0; i < n; ++i) in >> v[i];
    };
    if (cmd == "svm_type") {
      in >> cmd;
      if ((m->svm_type = lookup(cmd, kSvmTypes, 5)) < 0) return fail("unknown svm type.");
    } else if (cmd == "kernel_type") {
      in >> cmd;
      if ((m->kernel_type = lookup(cmd, kKernelTypes, 5)) < 0) return fail("unknown kernel function.");
    } else if (cmd == "degree") {
      in >> m->degree;
    } else if (cmd == "gamma") {
      in >> m->gamma;
    } else if (cmd == "coef0") {
      in >> m->coef0;
    } else if (cmd == "nr_class") {
      in >> m->nr_class;
    } else if (cmd == "total_sv") {
      in >> m->l;
    } else if (cmd == "rho") {
      read_vec(m->rho, npair);
    } else if (cmd == "label") {
      m->label.resize(m->nr_class);
      for (int& v : m->label) in >> v;
    } else if (cmd == "probA") {
      read_vec(m->probA, npair);
    } else if (cmd == "probB") {
      read_vec(m->probB, npair);
    } else if (cmd == "nr_sv") {
      m->nSV.resize(m->nr_class);
      for (int& v : m->nSV) in >> v;
    } else if (cmd == "SV") {
      sv_section = true;
      break;
    } else {
      return fail("unknown text in model file: [" + cmd + "]");
    }
    if (!in) return fail(std::string(path) + ": bad model header");
  }
  if (!sv_section || m->svm_type < 0 || m->kernel_type < 0 || m->nr_class < 1 || m->l < 0 ||
      (int)m->rho.size() != std::max(m->nr_class * (m->nr_class - 1) / 2, 1))
    return fail(std::string(path) + ": incomplete model");
  if (!regression_like(*m) && ((int)m->label.size() != m->nr_class || (int)m->nSV.size() != m->nr_class))
    return fail(std::string(path) + ": classification model without label / nr_sv");
  std::string line;
  std::getline(in, line);  // rest of the "SV" line
  const int nc = std::max(m->nr_class - 1, 1);
  m->sv_coef.assign(nc, std::vector<double>(m->l, 0.0));
  m->SV.resize(m->l);
  for (int i = 0; i < m->l; ++i) {
    if (!std::getline(in, line)) return fail(std::string(path) + ": " + std::to_string(i) + " of " +
                                              std::to_string(m->l) + " support vectors");
    std::istringstream ls(line);
    for (int k = 0; k < nc; ++k)
      if (!(ls >> m->sv_coef[k][i])) return fail(std::string(path) + ": bad SV line");
    std::string tok;
    while (ls >> tok) {
      const size_t c = tok.find(':');
      if (c == std::string::npos) return fail(std::string(path) + ": bad SV line");
      m->SV[i].push_back({std::atoi(tok.substr(0, c).c_str()), std::atof(tok.substr(c + 1).c_str())});
    }
    m->SV[i].push_back({-1, 0.0});
  }
  *out = m.release();
  return SK_OK;
}

void sk_svm_model_free(sk_svm_model* m) { delete m; }

int sk_svm_model_info(const sk_svm_model* m, int32_t* svm_type, int32_t* nr_class, int32_t* labels,
                      int32_t* has_probability) {
  if (!m) return fail("null model");
  if (svm_type) *svm_type = m->svm_type;
  if (nr_class) *nr_class = m->nr_class;
  if (labels)
    for (int i = 0; i < (int)m->label.size(); ++i) labels[i] = m->label[i];
  if (has_probability) *has_probability = !m->probA.empty() && !m->probB.empty();
  return SK_OK;
}

int sk_svm_predict(const sk_svm_model* m, int32_t cnt, const double* row, int32_t n, int32_t probability,
                   double* label, double* values) {
  if (!m || (!row && n > 0) || !label || !values || n < 0) return fail("null argument");
  // make_svm_node: x[0] = {0, cnt}, x[i+1] = {i+1, row[i]}, terminator
  std::vector<SvmNode> x(n + 2);
  x[0] = {0, (double)cnt};
  for (int i = 0; i < n; ++i) x[i + 1] = {i + 1, row[i]};
  x[n + 1] = {-1, 0.0};
  const int k = m->nr_class;
  const int npair = std::max(k * (k - 1) / 2, 1);
  std::vector<double> dec(npair);
  if (!decision_values(*m, x.data(), n + 1, dec.data()))
    return fail("precomputed support vector index outside the kernel row");
  const bool classifier = m->svm_type == 0 || m->svm_type == 1;
  if (probability && classifier) {
    for (int i = 0; i < k; ++i) values[i] = 0.0;
    if (m->probA.empty() || m->probB.empty()) {  // svm_predict_probability falls back
      *label = predict_label(*m, dec.data());
      return SK_OK;
    }
    const double min_prob = 1e-7;
    std::vector<std::vector<double>> r(k, std::vector<double>(k, 0.0));
    int p = 0;
    for (int i = 0; i < k; ++i)
      for (int j = i + 1; j < k; ++j) {
        r[i][j] = std::min(std::max(sigmoid_predict(dec[p], m->probA[p], m->probB[p]), min_prob), 1 - min_prob);
        r[j][i] = 1 - r[i][j];
        ++p;
      }
    multiclass_probability(k, r, values);
    int best = 0;
    for (int i = 1; i < k; ++i)
      if (values[i] > values[best]) best = i;
    *label = m->label[best];
    return SK_OK;
  }
  *label = predict_label(*m, dec.data());
  for (int i = 0; i < npair; ++i) values[i] = dec[i];
  return SK_OK;
}

const char* sk_svm_last_error(void) { return g_err.c_str(); }

}  // extern "C"
