// Model-config check: the reference reads its model dimensions from a YAML file
// (crates/pocket-tts/config/b6369a24.yaml, deserialized by serde in config.rs:1-124, loaded by
// TTSModel::load, config.rs:111-115). This engine compiles the b6369a24 dimensions into its
// kernels (SURVEY §8 constants), so the YAML is not a source of shapes here: it is checked.
// Every hot-path key the reference's config states must be present and equal the compiled value;
// anything else (weights paths, tokenizer, comments) is ignored. Another variant is a rebuild.
//
// The reader covers the subset the reference's config files use: nested block mappings by
// indentation ("key: value" / "key:"), block sequences of scalars ("- v"), '#' comments.
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "common.h"

namespace ptts {
namespace {

std::string trim(const std::string& s) {
  const size_t a = s.find_first_not_of(" \t\r");
  if (a == std::string::npos) return "";
  const size_t b = s.find_last_not_of(" \t\r");
  return s.substr(a, b - a + 1);
}

// A '#' starts a comment only at the start of the line or after whitespace, and never inside a
// quoted scalar ('...' or "..."): "tok#1" and "'a # b'" keep their '#'.
std::string strip_comment(const std::string& line) {
  char quote = 0;
  for (size_t i = 0; i < line.size(); ++i) {
    const char ch = line[i];
    if (quote) {
      if (ch == quote) quote = 0;
    } else if (ch == '\'' || ch == '"') {
      quote = ch;
    } else if (ch == '#' && (i == 0 || line[i - 1] == ' ' || line[i - 1] == '\t')) {
      return line.substr(0, i);
    }
  }
  return line;
}

// flattened "a.b.c" -> scalar, sequences joined with ','
std::map<std::string, std::string> read_yaml(const std::string& path) {
  std::ifstream f(path);
  if (!f) throw Error(PTTS_ERR_INVALID, "cannot open model config " + path);
  std::map<std::string, std::string> out;
  std::vector<std::pair<int, std::string>> stack;  // (indent, key) of the open mappings
  std::string line, seq_key;
  int seq_indent = -1, lineno = 0;
  while (std::getline(f, line)) {
    ++lineno;
    line = strip_comment(line);
    if (trim(line).empty()) continue;
    const int ind = (int)line.find_first_not_of(' ');
    const std::string body = trim(line);
    if (body[0] == '-') {  // sequence item of the last key
      if (seq_key.empty() || ind < seq_indent)
        throw Error(PTTS_ERR_INVALID, "model config line " + std::to_string(lineno) + ": unexpected sequence item");
      std::string& v = out[seq_key];
      v += (v.empty() ? "" : ",") + trim(body.substr(1));
      continue;
    }
    const size_t c = body.find(':');
    if (c == std::string::npos)
      throw Error(PTTS_ERR_INVALID, "model config line " + std::to_string(lineno) + ": expected 'key: value'");
    while (!stack.empty() && stack.back().first >= ind) stack.pop_back();
    std::string key;
    for (auto& e : stack) key += e.second + ".";
    key += trim(body.substr(0, c));
    const std::string val = trim(body.substr(c + 1));
    if (val.empty()) {  // opens a mapping or a sequence
      stack.push_back({ind, trim(body.substr(0, c))});
      seq_key = key;
      seq_indent = ind;
      out.erase(key);
    } else {
      out[key] = val;
      seq_key.clear();
    }
  }
  return out;
}

}  // namespace

void check_model_config(const char* path) {
  if (!path || !*path) return;
  const std::map<std::string, std::string> y = read_yaml(path);
  // the compiled variant (b6369a24.yaml:6-56; the engine's constants in engine.h / kernels.h)
  static const char* const want[][2] = {
      {"flow_lm.dtype", "float32"},
      {"flow_lm.flow.depth", "6"},
      {"flow_lm.flow.dim", "512"},
      {"flow_lm.transformer.d_model", "1024"},
      {"flow_lm.transformer.hidden_scale", "4"},
      {"flow_lm.transformer.max_period", "10000"},
      {"flow_lm.transformer.num_heads", "16"},
      {"flow_lm.transformer.num_layers", "6"},
      {"flow_lm.lookup_table.dim", "1024"},
      {"flow_lm.lookup_table.n_bins", "4000"},
      {"mimi.dtype", "float32"},
      {"mimi.sample_rate", "24000"},
      {"mimi.channels", "1"},
      {"mimi.frame_rate", "12.5"},
      {"mimi.seanet.dimension", "512"},
      {"mimi.seanet.channels", "1"},
      {"mimi.seanet.n_filters", "64"},
      {"mimi.seanet.n_residual_layers", "1"},
      {"mimi.seanet.ratios", "6,5,4"},
      {"mimi.seanet.kernel_size", "7"},
      {"mimi.seanet.residual_kernel_size", "3"},
      {"mimi.seanet.last_kernel_size", "3"},
      {"mimi.seanet.dilation_base", "2"},
      {"mimi.seanet.compress", "2"},
      {"mimi.seanet.pad_mode", "constant"},  // the convs' zero left padding is compiled in
      {"mimi.transformer.d_model", "512"},
      {"mimi.transformer.num_heads", "8"},
      {"mimi.transformer.num_layers", "2"},
      {"mimi.transformer.layer_scale", "0.01"},
      {"mimi.transformer.context", "250"},
      {"mimi.transformer.dim_feedforward", "2048"},
      {"mimi.transformer.input_dimension", "512"},
      {"mimi.transformer.output_dimensions", "512"},
      {"mimi.quantizer.dimension", "32"},
      {"mimi.quantizer.output_dimension", "512"},
  };
  for (const auto& w : want) {
    auto it = y.find(w[0]);
    if (it == y.end())
      throw Error(PTTS_ERR_INVALID, std::string("model config ") + path + ": missing " + w[0]);
    // numbers compare by value (12.5 == 12.50, 1e4 == 10000), everything else as text
    char* e1 = nullptr;
    char* e2 = nullptr;
    const double a = strtod(it->second.c_str(), &e1), b = strtod(w[1], &e2);
    const bool num = !it->second.empty() && *e1 == '\0' && *e2 == '\0';
    if (num ? a != b : it->second != w[1])
      throw Error(PTTS_ERR_INVALID, std::string("model config ") + path + ": " + w[0] + " = " + it->second +
                                        ", this build implements " + w[1] + " (variant b6369a24; rebuild for another)");
  }
}

}  // namespace ptts
