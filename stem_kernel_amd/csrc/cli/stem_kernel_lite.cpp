// stem_kernel_lite: the reference's kernel-matrix CLI (stem_kernel_lite/main.cpp
// with common/framework.{h,cpp}'s Options, App::train / App::predict and
// Output) over the MI355X engine, through the drop-in header
// include/stem_kernel_compat.hpp.  Same flags, positional arguments, console
// messages and output files:
//
//   stem_kernel_lite [options] output [label1 train1] ... [--test] [label1] [test1] ...
//
// Train mode writes the libsvm precomputed-kernel matrix of the training
// examples (KernelMatrix::print, common/kernel_matrix.cpp:756-770; .gz via
// zlib); predict mode (--test) writes one kernel row per test example
// (Output::kernel_output, common/framework.cpp:193-209), optionally only the
// support vectors of --model files (load_sv_index, libsvm/model.cpp:56-99),
// their self values to --norm (Output::norm_output), and each --model's
// predictions to the matching --predict file (Output::prob_output through
// SVMPredict, libsvm/svm_util.cpp:11-95: sk_svm_model_load / sk_svm_predict).
//
// Differences, by necessity: base-pairing probabilities come from the
// engine's GPU McCaskill (sk_fold_mccaskill) instead of ViennaRNA;
// --use-alifold is refused; .bz2 output goes through the
// system's libbz2.so.1 (loaded at run time: the image has the library but not
// its headers).  The
// reference's default kernel (SuStemStr without --log) only estimates memory
// and never runs App::execute (main.cpp:176-183, `//res = app.execute();`);
// here every kernel choice computes its matrix.
#include <dlfcn.h>
#include <zlib.h>

#include <algorithm>
#include <cctype>
#include <chrono>
#include <cmath>
#include <functional>
#include <memory>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "../../../include/stem_kernel_compat.hpp"

namespace {

struct Options {  // common/framework.h:37-62 + main.cpp:85-151
  // framework Options
  unsigned n_th = 1;
  bool normalize = false;
  std::string norm_output;
  bool predict_only = false;
  std::vector<std::string> trained_model_file, predict_output;
  // folding (BPMatrix::Options)
  skc::BPMatrix::Options bp;
  // kernel
  bool no_ribosum = false, no_string = false, use_log = false;
  float th = 0.01f;
  double beta = 0.3, loop_gap = 0.2, stack = 1.3, covar = 0.8;
  unsigned len_band = 10;
  double alpha = 0.2, gap = 0.8, str_match = 1.0, str_mismatch = 0.8;
  // positional
  std::string output;
  bool predict_mode = false;
  std::vector<std::string> labels, files, ts_labels, ts_files;
  std::vector<unsigned> sv_index;
};

const char* kUsage =
    "Options:\n"
    "  -h [ --help ]               show this message\n"
    "  -t [ --threads ] arg (=1)   set the number of threads\n"
    "  -n [ --normalize ]          normalize the kernel matrix\n"
    "  -x [ --norm ] arg           set the filename for norms of test examples\n"
    "  --no-matrix                 do not output matrix\n"
    "  --model arg                 the model file trained by svm-train if you already have\n"
    "  --predict arg               output file name of prediction results\n\n"
    "Kernel Options:\n"
    "  --no-ribosum                do not use the RIBOSUM substitution matrix\n"
    "  --no-string                 do not convolute the string kernel\n"
    "  --log                       use the logarithm of the kernel\n\n"
    "Options for the stem kernel:\n"
    "  -p [ --basepair ] arg (=0.01)  set the threshold of basepairing probability\n"
    "  -b [ --beta ] arg (=0.3)       weight of the RIBOSUM for the stem kernel\n"
    "  -g [ --loop-gap ] arg (=0.2)   gap weight for loop regions\n"
    "  -s [ --stack ] arg (=1.3)      match weight for stacking base pairs (with --no-ribosum)\n"
    "  -v [ --covariant ] arg (=0.8)  substitution (covariant) weight for base pairs (with\n"
    "                                 --no-ribosum)\n"
    "  --length-band arg (=10)        the band of difference of the length between bases\n\n"
    "Options for the string kernel:\n"
    "  -a [ --alpha ] arg (=0.2)      weight of the RIBOSUM for the string kernel\n"
    "  -G [ --gap ] arg (=0.8)        gap weight for the string kernel\n"
    "  --match arg (=1.0)             match weight for the string kernel (with --no-ribosum)\n"
    "  --mismatch arg (=0.8)          substitution (mismatch) weight for the string kernel (with\n"
    "                                 --no-ribosum)\n\n"
    "Folding Options:\n"
    "  --noGU                      disallow GU wobble base-pairs\n"
    "  --noClosingGU               disallow closing GU base-pairs\n"
    "  --noLonelyPairs             disallow lonely base-pairs\n"
    "  --use-alifold               use pf_alifold (not supported by the engine)\n"
    "  --pf-scale                  calculate appropriciate pf_scales using MFE (no effect)\n";

// boost::program_options-like parsing with allow_unregistered(): known
// options are consumed (long "--name value" / "--name=value", short "-x
// value" / "-xvalue"), everything else -- including "--test" -- is kept in
// order as extra arguments (main.cpp:152-163).
bool parse(int argc, char** argv, Options& o, std::vector<std::string>& extra, bool& help) {
  struct Opt {
    const char* name;
    char shrt;
    bool takes_value;
    std::function<void(const std::string&)> set;
  };
  auto to_f = [](const std::string& v) { return std::stod(v); };
  std::vector<Opt> opts = {
      {"help", 'h', false, [&](const std::string&) { help = true; }},
      {"threads", 't', true, [&](const std::string& v) { o.n_th = (unsigned)std::stoul(v); }},
      {"normalize", 'n', false, [&](const std::string&) { o.normalize = true; }},
      {"norm", 'x', true, [&](const std::string& v) { o.norm_output = v; }},
      {"no-matrix", 0, false, [&](const std::string&) { o.predict_only = true; }},
      {"model", 0, true, [&](const std::string& v) { o.trained_model_file.push_back(v); }},
      {"predict", 0, true, [&](const std::string& v) { o.predict_output.push_back(v); }},
      {"no-ribosum", 0, false, [&](const std::string&) { o.no_ribosum = true; }},
      {"no-string", 0, false, [&](const std::string&) { o.no_string = true; }},
      {"log", 0, false, [&](const std::string&) { o.use_log = true; }},
      {"basepair", 'p', true, [&](const std::string& v) { o.th = (float)to_f(v); }},
      {"beta", 'b', true, [&](const std::string& v) { o.beta = to_f(v); }},
      {"loop-gap", 'g', true, [&](const std::string& v) { o.loop_gap = to_f(v); }},
      {"stack", 's', true, [&](const std::string& v) { o.stack = to_f(v); }},
      {"covariant", 'v', true, [&](const std::string& v) { o.covar = to_f(v); }},
      {"length-band", 0, true, [&](const std::string& v) { o.len_band = (unsigned)std::stoul(v); }},
      {"alpha", 'a', true, [&](const std::string& v) { o.alpha = to_f(v); }},
      {"gap", 'G', true, [&](const std::string& v) { o.gap = to_f(v); }},
      {"match", 0, true, [&](const std::string& v) { o.str_match = to_f(v); }},
      {"mismatch", 0, true, [&](const std::string& v) { o.str_mismatch = to_f(v); }},
      {"noGU", 0, false, [&](const std::string&) { o.bp.no_GU = true; }},
      {"noClosingGU", 0, false, [&](const std::string&) { o.bp.no_closingGU = true; }},
      {"noLonelyPairs", 0, false, [&](const std::string&) { o.bp.no_LonelyPairs = true; }},
      {"use-alifold", 0, false, [&](const std::string&) { o.bp.alifold = true; }},
      {"pf-scale", 0, false, [&](const std::string&) { o.bp.use_pf_scale_mfe = true; }},
  };
  for (int k = 1; k < argc; ++k) {
    const std::string a = argv[k];
    const Opt* hit = nullptr;
    std::string val;
    bool inline_val = false;
    if (a.size() > 2 && a[0] == '-' && a[1] == '-') {
      std::string name = a.substr(2);
      const size_t eq = name.find('=');
      if (eq != std::string::npos) {
        val = name.substr(eq + 1);
        name = name.substr(0, eq);
        inline_val = true;
      }
      for (const Opt& p : opts)
        if (name == p.name) hit = &p;
    } else if (a.size() >= 2 && a[0] == '-' && a[1] != '-' && !std::isdigit((unsigned char)a[1])) {
      for (const Opt& p : opts)
        if (p.shrt && a[1] == p.shrt) hit = &p;
      if (hit && a.size() > 2) {
        val = a.substr(2);
        inline_val = true;
      }
    }
    if (!hit) {  // unregistered: an extra argument
      extra.push_back(a);
      continue;
    }
    if (hit->takes_value) {
      if (!inline_val) {
        if (k + 1 >= argc) {
          std::cerr << "the required argument for option '--" << hit->name << "' is missing" << std::endl;
          return false;
        }
        val = argv[++k];
      }
      try {
        hit->set(val);
      } catch (...) {
        std::cerr << "the argument ('" << val << "') for option '--" << hit->name << "' is invalid"
                  << std::endl;
        return false;
      }
    } else {
      hit->set("");
    }
  }
  return true;
}

// Options::parse_extra_args (common/framework.cpp:48-93)
void parse_extra_args(Options& o, const std::vector<std::string>& extra) {
  o.output = extra[0];
  size_t x = extra.size();
  for (size_t k = 0; k < extra.size(); ++k)
    if (extra[k] == "--test") x = k;
  o.predict_mode = x != extra.size();
  for (size_t i = 1; i + 1 < x + (o.predict_mode ? 0 : 1) && i + 1 < extra.size(); i += 2) {
    o.labels.push_back(extra[i]);
    o.files.push_back(extra[i + 1]);
  }
  if (o.predict_mode)
    for (size_t i = x + 1; i + 1 < extra.size(); i += 2) {
      o.ts_labels.push_back(extra[i]);
      o.ts_files.push_back(extra[i + 1]);
    }
}

// load_sv_index (libsvm/model.cpp:56-99): the "SV" section's "coef 0:idx"
// lines, 1-based -> 0-based, merged over models, sorted, unique
void load_sv_index(std::vector<unsigned>& sv, const std::vector<std::string>& models) {
  static std::string err;
  for (const std::string& m : models) {
    std::ifstream in(m);
    if (!in) {
      err = m + ": no such file";
      throw err.c_str();
    }
    std::string line;
    bool in_sv = false, seen = false;
    while (std::getline(in, line)) {
      if (!in_sv) {
        if (line == "SV") in_sv = seen = true;
        continue;
      }
      std::istringstream ls(line);
      std::string coef, idx;
      ls >> coef >> idx;
      if (idx.compare(0, 2, "0:") != 0) {
        err = m + ": bad format";
        throw err.c_str();
      }
      sv.push_back((unsigned)std::stoul(idx.substr(2)) - 1);
    }
    if (!seen) {
      err = m + ": bad format";
      throw err.c_str();
    }
  }
  std::sort(sv.begin(), sv.end());
  sv.erase(std::unique(sv.begin(), sv.end()), sv.end());
}

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// bzip2 output (common/framework.h:142-147's bzip2_compressor) through the
// system libbz2, loaded at run time: the BZ2_bzWrite* entry points of its
// stable C ABI (bzlib.h's BZFILE is opaque).
class Bz2Writer {
 public:
  explicit Bz2Writer(const std::string& path) : path_(path) {
    static std::string err;
    void* h = dlopen("libbz2.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("libbz2.so", RTLD_NOW | RTLD_LOCAL);
    if (h) {
      open_ = reinterpret_cast<OpenFn>(dlsym(h, "BZ2_bzWriteOpen"));
      write_ = reinterpret_cast<WriteFn>(dlsym(h, "BZ2_bzWrite"));
      close_ = reinterpret_cast<CloseFn>(dlsym(h, "BZ2_bzWriteClose"));
    }
    if (!open_ || !write_ || !close_) {
      err = path + ": bzip2 output needs libbz2.so.1";
      throw err.c_str();
    }
    f_ = std::fopen(path.c_str(), "wb");
    int e = 0;
    if (f_) bz_ = open_(&e, f_, 9, 0, 0);
    if (!f_ || !bz_ || e != 0) {
      if (f_) std::fclose(f_);
      f_ = nullptr;
      err = path + ": cannot open for writing";
      throw err.c_str();
    }
  }
  ~Bz2Writer() {  // on an error path only: finish() reports failures
    int e = 0;
    unsigned in = 0, out = 0;
    if (bz_) close_(&e, bz_, 1, &in, &out);
    if (f_) std::fclose(f_);
  }
  void write(const std::string& s) {
    int e = 0;
    for (size_t o = 0; o < s.size(); o += 1u << 30) {
      const int n = (int)std::min<size_t>(s.size() - o, 1u << 30);
      write_(&e, bz_, const_cast<char*>(s.data() + o), n);
      if (e != 0) fail();  // BZ_OK
    }
  }
  // flush the stream and close the file; a full disk or an I/O error throws
  void finish() {
    int e = 0;
    unsigned in = 0, out = 0;
    void* bz = bz_;
    bz_ = nullptr;
    if (bz) close_(&e, bz, 0, &in, &out);
    FILE* f = f_;
    f_ = nullptr;
    const bool closed = f ? std::fclose(f) == 0 : true;
    if (e != 0 || !closed) fail();
  }

 private:
  typedef void* (*OpenFn)(int*, FILE*, int, int, int);
  typedef void (*WriteFn)(int*, void*, void*, int);
  typedef void (*CloseFn)(int*, void*, int, unsigned*, unsigned*);
  OpenFn open_ = nullptr;
  WriteFn write_ = nullptr;
  CloseFn close_ = nullptr;
  FILE* f_ = nullptr;
  void* bz_ = nullptr;
  std::string path_;
  [[noreturn]] void fail() const {
    static std::string err;
    err = path_ + ": cannot write";
    throw err.c_str();
  }
};

// text output (plain, gzip or bzip2 by suffix, as the reference's filtering
// stream picks them, common/framework.h:142-152); predict mode streams
// through it
class TextSink {
 public:
  explicit TextSink(const std::string& path) : path_(path) {
    static std::string err;
    if (path.size() >= 4 && path.compare(path.size() - 4, 4, ".bz2") == 0) bz_.reset(new Bz2Writer(path));
    else if (path.size() >= 3 && path.compare(path.size() - 3, 3, ".gz") == 0) gz_ = gzopen(path.c_str(), "wb");
    else out_.open(path);
    if (!bz_ && (gz_ ? false : !out_.is_open())) {
      err = path + ": cannot open for writing";
      throw err.c_str();
    }
  }
  ~TextSink() {
    if (gz_) gzclose(gz_);
  }
  void write(const std::string& s) {
    if (bz_) bz_->write(s);
    else if (gz_) {
      if (!s.empty() && gzwrite(gz_, s.data(), (unsigned)s.size()) != (int)s.size()) fail();
    } else if (!(out_ << s)) fail();
  }
  // the last write: flush and close, reporting a truncated file
  void finish() {
    if (bz_) bz_->finish();
    else if (gz_) {
      gzFile g = gz_;
      gz_ = nullptr;
      if (gzclose(g) != Z_OK) fail();
    } else {
      out_.close();
      if (out_.fail()) fail();
    }
  }

 private:
  std::string path_;
  std::unique_ptr<Bz2Writer> bz_;
  gzFile gz_ = nullptr;
  std::ofstream out_;
  [[noreturn]] void fail() const {
    static std::string err;
    err = path_ + ": cannot write";
    throw err.c_str();
  }
};

void write_text(const std::string& path, const std::string& text) {
  TextSink sink(path);
  sink.write(text);
  sink.finish();
}

void flush_if_large(std::ostringstream& buf, std::unique_ptr<TextSink>& sink, const std::string& path,
                    bool final_flush = false) {
  if (path.empty()) return;
  if (!sink) sink.reset(new TextSink(path));
  if (final_flush || buf.str().size() > (size_t)10 * 1024 * 1024) {
    sink->write(buf.str());
    buf.str("");
  }
  if (final_flush) sink->finish();
}

// SVMPredict (libsvm/svm_util.cpp:11-80): one model, one prediction file;
// probability estimates requested (Output constructs it with true), so the
// file starts with the model's labels and each row is "label p1 p2 ..." for
// C-SVC / nu-SVC, else "target dec1 dec2 ..."; buffered like Output (10 MB).
class SvmPredictOut {
 public:
  SvmPredictOut(const std::string& out_file, const std::string& model_file) : out_(out_file) {
    static std::string err;
    if (!out_.is_open()) {
      err = out_file + ": cannot open for writing";
      throw err.c_str();
    }
    if (sk_svm_model_load(model_file.c_str(), &model_) != SK_OK) {
      err = model_file + ": " + sk_svm_last_error();
      throw err.c_str();
    }
    sk_svm_model_info(model_, &svm_type_, &nr_class_, nullptr, nullptr);
    std::vector<int32_t> labels(std::max(nr_class_, 1), 0);  // zeros when the model has none
    sk_svm_model_info(model_, nullptr, nullptr, labels.data(), nullptr);
    out_ << "labels ";
    for (int k = 0; k < nr_class_; ++k) out_ << labels[k] << " ";
    out_ << std::endl;
  }
  ~SvmPredictOut() {
    out_ << buf_.str();
    sk_svm_model_free(model_);
  }
  void predict(double target, unsigned cnt, const std::vector<double>& row) {
    static std::string err;
    std::vector<double> vals(std::max(nr_class_ * (nr_class_ - 1) / 2, std::max(nr_class_, 1)));
    double v = 0.0;
    if (sk_svm_predict(model_, (int32_t)cnt, row.data(), (int32_t)row.size(), 1, &v, vals.data()) != SK_OK) {
      err = sk_svm_last_error();
      throw err.c_str();
    }
    if (svm_type_ == 0 || svm_type_ == 1) {
      buf_ << v << " ";
      for (int k = 0; k < nr_class_; ++k) buf_ << vals[k] << " ";
    } else {
      buf_ << target << " ";
      for (int k = 0; k < nr_class_ * (nr_class_ - 1) / 2; ++k) buf_ << vals[k] << " ";
    }
    buf_ << std::endl;
    if (buf_.str().size() > (size_t)10 * 1024 * 1024) {
      out_ << buf_.str();
      buf_.str("");
    }
  }

 private:
  std::ofstream out_;
  std::ostringstream buf_;
  sk_svm_model* model_ = nullptr;
  int32_t svm_type_ = 0, nr_class_ = 0;
};

// App<K,LDF> (common/framework.h:100-353) over the compat types
template <class K>
class App {
 public:
  typedef skc::MData Data;
  typedef std::pair<std::string, Data> Example;
  typedef std::vector<Example> ExampleSet;
  typedef skc::DataLoaderFactory<skc::DataLoader<skc::MData>> LDF;

  App(const K& kernel, const LDF& ldf, const Options& opts) : kernel_(kernel), ldf_(ldf), opts_(opts) {}
  bool execute() const { return opts_.predict_mode ? predict() : train(); }

 private:
  bool train() const {
    ExampleSet ex;
    load_examples(ex, opts_.labels, opts_.files);
    skc::KernelMatrix<double> matrix;
    const double elapsed = matrix.calculate(ex, kernel_, opts_.normalize, opts_.n_th);
    std::cout << "elapsed time: " << elapsed << "s" << std::endl;
    std::ostringstream os;
    matrix.print(os);
    write_text(opts_.output, os.str());
    return true;
  }

  bool predict() const {
    ExampleSet ex;
    load_examples(ex, opts_.labels, opts_.files);
    std::vector<double> diag(ex.size()), vec(ex.size());
    if (opts_.normalize) {
      const double e = skc::KernelMatrix<double>::diagonal(diag, ex, opts_.sv_index, kernel_, opts_.n_th);
      std::cout << "elapsed time for diagonals: " << e << "s" << std::endl;
    }
    const bool norm = opts_.normalize || !opts_.norm_output.empty();
    std::ostringstream kout, tout;
    std::unique_ptr<TextSink> kfile, tfile;
    // Output's SVMPredict per --predict file with the --model of the same
    // position (framework.cpp:142-154)
    std::vector<std::unique_ptr<SvmPredictOut>> pout;
    for (size_t k = 0; k != opts_.predict_output.size(); ++k) {
      pout.emplace_back(new SvmPredictOut(opts_.predict_output[k], opts_.trained_model_file[k]));
    }
    unsigned cnt = 0;
    for (size_t i = 0; i != opts_.ts_files.size(); ++i) {
      double elapsed = 0.0;
      std::cout << "predicting " << opts_.ts_files[i] << std::flush;
      std::unique_ptr<typename LDF::Loader> loader(ldf_.get_loader(opts_.ts_files[i].c_str()));
      for (;;) {
        const double t0 = now_s();
        std::unique_ptr<Data> data(loader->get());
        elapsed += now_s() - t0;
        if (!data) break;
        double self = 0.0;
        elapsed += skc::KernelMatrix<double>::calculate(vec, Example(opts_.ts_labels[i], *data), ex,
                                                        opts_.sv_index, kernel_, opts_.n_th,
                                                        norm ? &self : NULL);
        if (opts_.normalize)
          for (size_t j = 0; j != vec.size(); ++j) vec[j] /= std::sqrt(diag[j] * self);
        ++cnt;
        // Output::kernel_output / norm_output (common/framework.cpp:193-234)
        if (!opts_.predict_only) {
          kout << opts_.ts_labels[i] << " 0:" << cnt << " ";
          for (size_t j = 0; j != vec.size(); ++j) kout << (j + 1) << ":" << vec[j] << " ";
          kout << std::endl;
        }
        if (!opts_.norm_output.empty()) tout << self << std::endl;
        // Output::prob_output (framework.cpp:211-221)
        for (auto& p : pout) p->predict(std::atof(opts_.ts_labels[i].c_str()), cnt, vec);
        // Output flushes its buffers past MAX = 10 MB (framework.cpp:193-234)
        flush_if_large(kout, kfile, opts_.predict_only ? std::string() : opts_.output);
        flush_if_large(tout, tfile, opts_.norm_output);
      }
      std::cout << " (" << elapsed << "s) done." << std::endl;
    }
    flush_if_large(kout, kfile, opts_.predict_only ? std::string() : opts_.output, true);
    flush_if_large(tout, tfile, opts_.norm_output, true);
    return true;
  }

  // App::load_examples (common/framework.h:308-353); no globbing: a file
  // name is taken as given
  void load_examples(ExampleSet& ex, const std::vector<std::string>& labels,
                     const std::vector<std::string>& files) const {
    for (size_t i = 0; i != files.size(); ++i) {
      double elapsed = 0.0;
      std::unique_ptr<typename LDF::Loader> loader(ldf_.get_loader(files[i].c_str()));
      std::cout << "loading " << files[i] << " as label " << labels[i] << std::flush;
      for (;;) {
        const double t0 = now_s();
        std::unique_ptr<Data> d(loader->get());
        elapsed += now_s() - t0;
        if (!d) break;
        ex.push_back(std::make_pair(labels[i], *d));
      }
      std::cout << " (" << elapsed << "s) done." << std::endl;
    }
  }

  K kernel_;
  LDF ldf_;
  const Options& opts_;
};

template <class K>
bool run(const K& kernel, const Options& o) {
  skc::DataLoaderFactory<skc::DataLoader<skc::MData>> ldf(o.th, o.bp);
  App<K> app(kernel, ldf, o);
  return app.execute();
}

}  // namespace

int main(int argc, char** argv) {
  Options o;
  std::vector<std::string> extra;
  bool help = false;
  if (!parse(argc, argv, o, extra, help)) return 1;
  if (help || extra.size() < 3) {
    std::cout << "Kernel Matrix Calculator for Stem Kernels" << std::endl
              << "Usage:" << std::endl
              << " " << argv[0]
              << " [options] output [label1 training-data1] ... [--test] [label1] [test-data1] ...\n\n"
              << kUsage << std::endl;
    return 1;
  }
  parse_extra_args(o, extra);
  bool res = false;
  try {
    if (o.predict_output.size() > o.trained_model_file.size())
      throw "--predict: every prediction file needs the --model of the same position";
    if (o.bp.alifold) throw "--use-alifold is not supported by the engine's fold";
    if (o.predict_mode && !o.trained_model_file.empty()) load_sv_index(o.sv_index, o.trained_model_file);
    // kernel choice: main.cpp:166-214
    if (!o.no_string && !o.no_ribosum) {
      if (!o.use_log)
        res = run(skc::SuStemStrKernel<double, skc::MData>(o.alpha, o.beta, o.loop_gap, o.gap, o.len_band), o);
      else
        res = run(skc::LSuStemStrKernel<double, skc::MData>(o.alpha, o.beta, o.loop_gap, o.gap, o.len_band), o);
    } else if (o.no_string && !o.no_ribosum) {
      if (!o.use_log)
        res = run(skc::SuStemKernel<double, skc::MData>(o.loop_gap, o.beta, o.len_band), o);
      else
        res = run(skc::LSuStemKernel<double, skc::MData>(o.loop_gap, o.beta, o.len_band), o);
    } else if (!o.no_string && o.no_ribosum) {
      res = run(skc::SiStemStrKernel<double, skc::MData>(o.loop_gap, o.stack, o.covar, o.gap, o.str_match,
                                                         o.str_mismatch, o.len_band),
                o);
    } else {
      res = run(skc::SiStemKernel<double, skc::MData>(o.loop_gap, o.stack, o.covar, o.len_band), o);
    }
  } catch (const char* str) {
    std::cout << str << std::endl;
  }
  return res ? 0 : 1;
}
