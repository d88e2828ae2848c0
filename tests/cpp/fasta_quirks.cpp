// Prints what load_examples(label, Fasta, ex) of the compat headers reads
// from a file, one "label<TAB>sequence" line per example (no GPU needed).
#include <cstdio>
#include <fstream>

#include "string_kernel_compat.hpp"

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  std::ifstream in(argv[1]);
  Fasta fasta(in);
  ExampleSet ex;
  load_examples("+1", fasta, ex);
  for (const Example& e : ex) std::printf("%s\t%s\n", e.first.c_str(), e.second.c_str());
  if (argc > 2) {  // the "label sequence" line format
    std::ifstream in2(argv[2]);
    ExampleSet ex2;
    load_examples(in2, ex2);
    for (const Example& e : ex2) std::printf("%s\t%s\n", e.first.c_str(), e.second.c_str());
  }
  return 0;
}
