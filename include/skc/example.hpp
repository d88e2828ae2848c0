// skc/example.hpp -- the string-example side of the stem_kernel/ (4-D) and
// string_kernel/ (naive) tools: Example / ExampleSet (common/example.h:12-20),
// the legacy Fasta reader (common/fasta.h:14-40, common/fasta.cpp) and
// load_examples (common/example.cpp:10-35), with the reference's behaviour
// kept to the quirk:
//   - the constructor skips everything up to the first '>';
//   - GetNextSeq reads up to the next '>' (or the end), takes the first
//     line after leading blanks as the name and joins the whitespace-split
//     tokens of the rest as the sequence, dropping one trailing '*';
//   - at the end of the stream it returns "" and leaves the previous
//     sequence in place, so load_examples -- `while (!IsEOF() &&
//     GetNextSeq())`, "" being a non-null pointer -- appends the previous
//     sequence once more when the file ends in a bare '>'.
#ifndef SKC_EXAMPLE_HPP
#define SKC_EXAMPLE_HPP

#include <algorithm>
#include <cctype>
#include <fstream>
#include <istream>
#include <sstream>
#include <string>
#include <utility>
#include <vector>

#include "skc/core.hpp"

namespace skc {

typedef std::pair<std::string, std::string> Example;
typedef std::vector<Example> ExampleSet;

class Fasta {
 public:
  explicit Fasta(std::istream& istrm) : m_istrm(istrm) {
    std::string buf;
    std::getline(m_istrm, buf, '>');
  }
  const char* GetNextSeq() {
    std::string buf;
    std::getline(m_istrm, buf, '>');
    if (!m_istrm) return "";
    std::istringstream ss(buf);
    while (ss.get() == ' ') {
    }
    ss.unget();
    std::getline(ss, m_name);
    m_seq.erase();
    while (!ss.eof()) {
      std::string line;
      ss >> line;
      m_seq += line;
    }
    if (!m_seq.empty() && m_seq[m_seq.size() - 1] == '*') m_seq.erase(m_seq.size() - 1, 1);
    return m_seq.c_str();
  }
  const std::string& Seq() const { return m_seq; }
  const std::string& Name() const { return m_name; }
  void ToUpper() { std::transform(m_seq.begin(), m_seq.end(), m_seq.begin(), [](unsigned char c) { return (char)std::toupper(c); }); }
  void ToLower() { std::transform(m_seq.begin(), m_seq.end(), m_seq.begin(), [](unsigned char c) { return (char)std::tolower(c); }); }
  bool IsEOF() const { return m_istrm.eof(); }
  bool IsFail() const { return m_istrm.fail(); }
  bool operator!() const { return !m_istrm; }

 private:
  std::istream& m_istrm;
  std::string m_seq;
  std::string m_name;
};

// "label sequence" lines (common/example.cpp:10-25), sequences lowercased
inline uint load_examples(std::ifstream& in, ExampleSet& ex) {
  std::string buf;
  while (std::getline(in, buf)) {
    std::istringstream s(buf);
    std::string c, seq;
    s >> c >> seq;
    if (!seq.empty()) {
      std::transform(seq.begin(), seq.end(), seq.begin(), [](unsigned char ch) { return (char)std::tolower(ch); });
      ex.push_back(Example(c, seq));
    }
  }
  return (uint)ex.size();
}

// every FASTA record under one label (common/example.cpp:27-35), lowercased
inline uint load_examples(const std::string& label, Fasta& f, ExampleSet& ex) {
  while (!f.IsEOF() && f.GetNextSeq()) {
    f.ToLower();
    ex.push_back(Example(label, f.Seq()));
  }
  return (uint)ex.size();
}

// A raw-sequence example for the engine: one row; folded (use_bp) when the
// kernel's BuildSpec asks for base-pairing probabilities (the 4-D
// BPMatrix model), else none.  th = 1 keeps the (unused) DAG empty.
template <>
struct ExampleTraits<std::string> {
  static void add(sk_dataset* ds, const std::string& label, const std::string& seq, const BuildSpec& spec) {
    const char* row = seq.c_str();
    if (!spec.fold) {
      check(sk_dataset_add(ds, label.c_str(), 1, &row, nullptr, 1.0f, 0));
      return;
    }
    std::vector<std::vector<double>> bpp;
    if (spec.fold_fn) {
      bpp.emplace_back();
      spec.fold_fn(seq, (spec.fold_flags & SK_FOLD_NO_GU) != 0, bpp.back());
    } else {
      Engine::get().fold(std::vector<std::string>(1, seq), spec.fold_flags, bpp);
    }
    const double* b = bpp[0].data();
    check(sk_dataset_add(ds, label.c_str(), 1, &row, &b, 1.0f, 1));
  }
  static void mix(Fnv& f, const std::string& s) { f(s.data(), s.size() + 1); }
};

}  // namespace skc

#endif  // SKC_EXAMPLE_HPP
