// Example-file readers: the FASTA / CLUSTAL / MAF grammars the reference's
// DataLoader<MData>::get (stem_kernel_lite/data.cpp:547-586) pulls one example
// at a time from, restated as hand-written scanners with Boost.Spirit
// classic's semantics (no skipper, greedy kleene stars that never backtrack,
// alternatives tried in order, semantic actions that fire as soon as their
// sub-parser matches and are not undone when an enclosing rule fails):
//
//   FASTA    fa_parser   common/fa.cpp:13-55      one sequence per example
//   CLUSTAL  aln_parser  common/aln.cpp:16-107    one alignment (all blocks)
//   MAF      maf_parser  common/maf.cpp:15-49     one alignment block
//
// Reading stops at the first example that does not parse (the reference's
// loader returns NULL there).  Errors the reference throws (a missing file,
// aln's format_error, the loader's "wrong alignment") become SK_ERR_INVALID.
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "stem_kernel.h"

struct sk_seqfile {
  std::vector<std::vector<std::string>> ex;  // examples -> rows
};

namespace {

thread_local std::string g_err;

int set_err(const std::string& m) {
  g_err = m;
  return SK_ERR_INVALID;
}

struct Scan {
  const char* s;
  size_t n;
  bool at(size_t p) const { return p < n; }
  bool blank(size_t p) const { return p < n && (s[p] == ' ' || s[p] == '\t'); }
  bool graph(size_t p) const { return p < n && s[p] > 0x20 && s[p] < 0x7f; }
  bool print(size_t p) const { return p < n && s[p] >= 0x20 && s[p] < 0x7f; }
  // eol_p: "\r\n" | "\r" | "\n"; returns the end or npos
  size_t eol(size_t p) const {
    if (p >= n) return std::string::npos;
    if (s[p] == '\r') return (p + 1 < n && s[p + 1] == '\n') ? p + 2 : p + 1;
    if (s[p] == '\n') return p + 1;
    return std::string::npos;
  }
  size_t blanks(size_t p) const {
    while (blank(p)) ++p;
    return p;
  }
  size_t graphs(size_t p) const {
    while (graph(p)) ++p;
    return p;
  }
  size_t prints(size_t p) const {
    while (print(p)) ++p;
    return p;
  }
  bool lit(size_t p, const char* w) const {
    const size_t k = std::strlen(w);
    return p + k <= n && std::memcmp(s + p, w, k) == 0;
  }
  // empty = *blank_p >> eol_p
  size_t empty(size_t p) const { return eol(blanks(p)); }
  // uint_p (decimal, no overflow past 2^32-1)
  size_t uint(size_t p) const {
    size_t q = p;
    unsigned long long v = 0;
    while (q < n && s[q] >= '0' && s[q] <= '9') {
      v = v * 10 + (unsigned)(s[q] - '0');
      if (v > 0xffffffffull) return std::string::npos;
      ++q;
    }
    return q > p ? q : std::string::npos;
  }
};
constexpr size_t NPOS = std::string::npos;

// fa = head >> seq;  head = '>' >> *(blank_p|graph_p) >> eol_p;
// seq_l = *(graph_p - '>' - eol_p);  seq = +(seq_l[append] >> eol_p)
size_t parse_fa(const Scan& S, size_t p, std::string& seq) {
  if (!S.at(p) || S.s[p] != '>') return NPOS;
  ++p;
  while (S.blank(p) || S.graph(p)) ++p;
  p = S.eol(p);
  if (p == NPOS) return NPOS;
  int lines = 0;
  for (;;) {
    size_t q = p;
    while (S.graph(q) && S.s[q] != '>') ++q;
    seq.append(S.s + p, q - p);  // the action fires even if eol_p then fails
    const size_t e = S.eol(q);
    if (e == NPOS) break;
    p = e;
    ++lines;
  }
  return lines ? p : NPOS;
}

// aln_parser (common/aln.cpp:16-107)
struct AlnWA {
  size_t cur_index = 0;
  std::vector<std::string> names, seqs;
};

size_t head_word(const Scan& S, size_t p) {
  if (S.lit(p, "CLUSTAL")) return p + 7;
  if (S.lit(p, "PROBCONS")) return p + 8;
  return NPOS;
}

// seq = (+graph_p - head_word)[name] >> +blank_p >> (+graph_p)[seq] >> *blank_p >> eol_p
size_t aln_seq(const Scan& S, size_t p, std::string& name, std::string& seq) {
  const size_t a = S.graphs(p);
  if (a == p) return NPOS;
  const size_t h = head_word(S, p);
  if (h != NPOS && h - p >= a - p) return NPOS;  // difference: head word as long
  size_t q = S.blanks(a);
  if (q == a) return NPOS;
  const size_t b = S.graphs(q);
  if (b == q) return NPOS;
  name.assign(S.s + p, a - p);
  seq.assign(S.s + q, b - q);
  return S.eol(S.blanks(b));
}

// body_part = +seq[push_seq] >> !status; status = *(chset("*:.")|blank_p) >> eol_p
size_t aln_body_part(const Scan& S, size_t p, AlnWA& wa, int& err) {
  int k = 0;
  std::string name, seq;
  for (;;) {
    const size_t e = aln_seq(S, p, name, seq);
    if (e == NPOS) break;
    // push_seq (:40-54)
    if (wa.cur_index >= wa.names.size()) {
      wa.names.push_back(name);
      wa.seqs.push_back(seq);
    } else if (wa.names[wa.cur_index] == name) {
      wa.seqs[wa.cur_index] += seq;
    } else {
      err = set_err("format error: broken sequence name consistency");
      return NPOS;
    }
    wa.cur_index++;
    p = e;
    ++k;
  }
  if (!k) return NPOS;
  size_t q = p;
  while (S.blank(q) || (S.at(q) && std::strchr("*:.", S.s[q]) && S.s[q])) ++q;
  const size_t e = S.eol(q);
  return e == NPOS ? p : e;
}

// reset_index (:56-72)
bool aln_reset(AlnWA& wa, int& err) {
  for (size_t i = 1; i < wa.seqs.size(); ++i)
    if (wa.seqs[i].size() != wa.seqs[0].size()) {
      err = set_err("format error: broken sequence length consistency");
      return false;
    }
  wa.cur_index = 0;
  return true;
}

// aln = header >> +empty >> body;  header = head_word >> +print_p >> eol_p
// body = body_part[reset] >> *(+empty >> body_part[reset])
size_t parse_aln(const Scan& S, size_t p, std::vector<std::string>& rows, int& err) {
  p = head_word(S, p);
  if (p == NPOS) return NPOS;
  const size_t a = S.prints(p);
  if (a == p) return NPOS;
  p = S.eol(a);
  if (p == NPOS) return NPOS;
  size_t e = S.empty(p);
  if (e == NPOS) return NPOS;
  while (e != NPOS) p = e, e = S.empty(p);
  AlnWA wa;
  p = aln_body_part(S, p, wa, err);
  if (err || p == NPOS) return NPOS;
  if (!aln_reset(wa, err)) return NPOS;
  for (;;) {
    size_t q = S.empty(p);
    if (q == NPOS) break;
    for (size_t r = S.empty(q); r != NPOS; r = S.empty(q)) q = r;
    const size_t b = aln_body_part(S, q, wa, err);
    if (err) return NPOS;
    if (b == NPOS) break;
    if (!aln_reset(wa, err)) return NPOS;
    p = b;
  }
  rows = wa.seqs;
  return p;
}

// maf = !header >> *(comment|empty) >> ali >> +seq >> *empty   (common/maf.cpp:15-49)
size_t maf_seq(const Scan& S, size_t p, std::vector<std::string>& rows) {
  size_t q = NPOS;
  if (S.at(p) && S.s[p] == 's') {
    // seq_s1 = 's' +blank +graph +blank uint +blank uint +blank
    size_t t = p + 1, u;
    bool ok = true;
    auto need_blanks = [&]() {
      u = S.blanks(t);
      ok = ok && u > t;
      t = u;
    };
    need_blanks();
    if (ok) {
      u = S.graphs(t);
      ok = u > t;
      t = u;
    }
    if (ok) need_blanks();
    if (ok) ok = (t = S.uint(t)) != NPOS;
    if (ok) need_blanks();
    if (ok) ok = (t = S.uint(t)) != NPOS;
    if (ok) need_blanks();
    // seq_s2 = sign_p +blank uint +blank (+graph)[push_back] *blank
    if (ok) ok = S.at(t) && (S.s[t] == '+' || S.s[t] == '-'), ++t;
    if (ok) need_blanks();
    if (ok) ok = (t = S.uint(t)) != NPOS;
    if (ok) need_blanks();
    if (ok) {
      u = S.graphs(t);
      ok = u > t;
      if (ok) rows.emplace_back(S.s + t, u - t);  // fires before the eol is seen
      t = S.blanks(u);
    }
    if (ok) q = t;
  }
  if (q == NPOS && S.at(p) && (S.s[p] == 'i' || S.s[p] == 'e')) {
    // seq_i = ('i'|'e') +blank +print eol
    size_t t = p + 1;
    size_t u = S.blanks(t);
    if (u > t) {
      t = u;
      u = S.prints(t);
      if (u > t) q = S.eol(u);
    }
  }
  if (q == NPOS) return NPOS;
  return S.eol(q);
}

size_t parse_maf(const Scan& S, size_t p, std::vector<std::string>& rows) {
  if (S.lit(p, "##maf")) {
    const size_t e = S.eol(S.prints(p + 5));
    if (e != NPOS) p = e;
  }
  for (;;) {
    if (S.at(p) && S.s[p] == '#') {  // comment_p("#"): to the end of the line
      size_t q = p + 1;
      while (S.at(q) && S.eol(q) == NPOS) ++q;
      p = S.at(q) ? S.eol(q) : q;
      continue;
    }
    const size_t e = S.empty(p);
    if (e == NPOS) break;
    p = e;
  }
  // ali = 'a' +blank *print eol
  if (!S.at(p) || S.s[p] != 'a') return NPOS;
  size_t t = S.blanks(p + 1);
  if (t == p + 1) return NPOS;
  p = S.eol(S.prints(t));
  if (p == NPOS) return NPOS;
  int k = 0;
  for (;;) {
    const size_t e = maf_seq(S, p, rows);
    if (e == NPOS) break;
    p = e;
    ++k;
  }
  if (!k) return NPOS;
  for (size_t e = S.empty(p); e != NPOS; e = S.empty(p)) p = e;
  return p;
}

int parse_all(const char* text, size_t len, int32_t format, sk_seqfile* F) {
  const Scan S{text, len};
  size_t p = 0;
  for (;;) {
    std::vector<std::string> rows;
    size_t e;
    int err = 0;
    if (format == SK_FMT_FASTA) {
      std::string seq;
      e = parse_fa(S, p, seq);
      rows.push_back(seq);
    } else if (format == SK_FMT_CLUSTAL) {
      e = parse_aln(S, p, rows, err);
    } else {
      e = parse_maf(S, p, rows);
    }
    if (err) return err;
    if (e == NPOS) break;
    p = e;
    // DataLoader<MData>::get (data.cpp:574-578): rows of one length
    for (const auto& r : rows)
      if (r.size() != rows.front().size()) return set_err("wrong alignment");
    F->ex.push_back(std::move(rows));
  }
  return SK_OK;
}

}  // namespace

extern "C" {

int sk_seqfile_parse(const char* text, size_t len, int32_t format, sk_seqfile** out) {
  if (!out || (!text && len) || format < SK_FMT_FASTA || format > SK_FMT_MAF)
    return set_err("invalid argument");
  *out = nullptr;
  sk_seqfile* F = new sk_seqfile;
  const int rc = parse_all(text, len, format, F);
  if (rc) {
    delete F;
    return rc;
  }
  *out = F;
  return SK_OK;
}

int sk_seqfile_read(const char* path, int32_t format, sk_seqfile** out) {
  if (!path || !out) return set_err("invalid argument");
  FILE* f = std::fopen(path, "rb");
  if (!f) return set_err(std::string(path) + ": no such file");
  std::string buf;
  char tmp[1 << 16];
  size_t k;
  while ((k = std::fread(tmp, 1, sizeof tmp, f)) > 0) buf.append(tmp, k);
  std::fclose(f);
  return sk_seqfile_parse(buf.data(), buf.size(), format, out);
}

int sk_seqfile_free(sk_seqfile* f) {
  delete f;
  return SK_OK;
}

int64_t sk_seqfile_count(const sk_seqfile* f) { return f ? (int64_t)f->ex.size() : 0; }

int32_t sk_seqfile_rows(const sk_seqfile* f, int64_t i) {
  if (!f || i < 0 || i >= (int64_t)f->ex.size()) return 0;
  return (int32_t)f->ex[i].size();
}

const char* sk_seqfile_row(const sk_seqfile* f, int64_t i, int32_t r) {
  if (!f || i < 0 || i >= (int64_t)f->ex.size() || r < 0 || r >= (int32_t)f->ex[i].size())
    return nullptr;
  return f->ex[i][r].c_str();
}

const char* sk_seqfile_last_error(void) { return g_err.c_str(); }

}  // extern "C"
