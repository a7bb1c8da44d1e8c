// spm_encode — drop-in for the reference CLI (src/spm_encode_main.cc:52-223)
// for --output_format=id|piece, with batched device encoding.
//
// The reference encodes one line at a time (spm_encode_main.cc:189-191).
// Here lines are read in batches (--batch_lines), normalized and encoded on
// the device in one call per batch (SentencePieceProcessor::EncodeBatch;
// ids also get the device id epilogue); the output is byte-identical:
// one output line per input line, pieces / ids joined by " ".  Lines are
// read with std::getline semantics (a trailing '\r' is kept,
// filesystem.cc:42-44).
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <string>
#include <vector>

#include "processor.h"

namespace {

struct Flags {
  std::string model, output_format = "piece", output, extra_options;
  long batch_lines = 1 << 20;
};

void Usage(const char *argv0) {
  std::cout << "Usage: " << argv0 << " [options] files\n\n"
            << "   --model (model file name)  type: string default: \n"
            << "   --output_format (choose from piece or id)  type: string default: piece\n"
            << "   --output (output filename)  type: string default: \n"
            << "   --extra_options (':' separated encoder extra options, e.g., "
               "\"reverse:bos:eos\")  type: string default: \n"
            << "   --batch_lines (lines per device batch)  type: int64 default: 1048576\n";
}

[[noreturn]] void Die(const std::string &msg) {
  std::cerr << msg << std::endl;
  std::exit(1);
}

// CommandLineGetFlag semantics (flags.cc): --k=v, --k v, -k=v; bare --k is
// "true" for booleans.
bool GetFlag(int argc, char **argv, int *i, std::string *key, std::string *value) {
  std::string a = argv[*i];
  if (a.size() < 2 || a[0] != '-') return false;
  a = a.substr(a[1] == '-' ? 2 : 1);
  const size_t eq = a.find('=');
  if (eq != std::string::npos) {
    *key = a.substr(0, eq);
    *value = a.substr(eq + 1);
    return true;
  }
  *key = a;
  if (*i + 1 < argc && argv[*i + 1][0] != '-') {
    *value = argv[++*i];
  } else {
    *value = "true";
  }
  return true;
}

}  // namespace

int main(int argc, char **argv) {
  Flags f;
  std::vector<std::string> rest;
  for (int i = 1; i < argc; ++i) {
    std::string k, v;
    if (!GetFlag(argc, argv, &i, &k, &v)) {
      rest.push_back(argv[i]);
      continue;
    }
    if (k == "help") {
      Usage(argv[0]);
      return 0;
    } else if (k == "version") {
      std::cout << "sentencepiece-mi355x 0.1.82" << std::endl;
      return 0;
    } else if (k == "model") {
      f.model = v;
    } else if (k == "output_format") {
      f.output_format = v;
    } else if (k == "output") {
      f.output = v;
    } else if (k == "extra_options") {
      f.extra_options = v;
    } else if (k == "batch_lines") {
      f.batch_lines = std::max(1L, std::atol(v.c_str()));
    } else if (k == "minloglevel") {
    } else {
      Usage(argv[0]);
      Die("Unknown/Invalid flag " + k);
    }
  }
  if (f.model.empty()) {
    Usage(argv[0]);
    Die("--model is required.");
  }
  if (f.output_format != "id" && f.output_format != "piece")
    Die("output_format \"" + f.output_format +
        "\": only piece and id are implemented by the device engine");

  spm_amd::SentencePieceProcessor sp;
  auto st = sp.Load(f.model);
  if (!st.ok()) Die(st.message);
  st = sp.SetEncodeExtraOptions(f.extra_options);
  if (!st.ok()) Die(st.message);

  std::ofstream ofs;
  std::ostream *out = &std::cout;
  if (!f.output.empty()) {
    ofs.open(f.output, std::ios::binary);
    if (!ofs) Die("\"" + f.output + "\": cannot open");
    out = &ofs;
  }
  if (rest.empty()) rest.push_back("");  // stdin

  std::vector<std::string> batch;
  std::vector<std::vector<int>> ids;
  std::vector<std::vector<std::string>> pieces;
  std::string buf;
  auto flush = [&]() {
    if (batch.empty()) return;
    auto s = f.output_format == "id" ? sp.EncodeBatch(batch, &ids, nullptr)
                                     : sp.EncodeBatch(batch, nullptr, &pieces);
    if (!s.ok()) Die(s.message);
    for (size_t i = 0; i < batch.size(); ++i) {
      buf.clear();
      if (f.output_format == "id") {
        for (size_t k = 0; k < ids[i].size(); ++k) {
          if (k) buf += ' ';
          buf += std::to_string(ids[i][k]);
        }
      } else {
        for (size_t k = 0; k < pieces[i].size(); ++k) {
          if (k) buf += ' ';
          buf += pieces[i][k];
        }
      }
      buf += '\n';
      out->write(buf.data(), buf.size());
    }
    batch.clear();
  };
  for (const auto &fn : rest) {
    std::ifstream ifs;
    std::istream *in = &std::cin;
    if (!fn.empty()) {
      ifs.open(fn, std::ios::binary);
      if (!ifs) Die("\"" + fn + "\": No such file or directory");
      in = &ifs;
    }
    std::string line;
    while (std::getline(*in, line)) {
      batch.push_back(line);
      if (static_cast<long>(batch.size()) >= f.batch_lines) flush();
    }
  }
  flush();
  return 0;
}
