// pm_config.cpp — host-side configuration handling of the drop-in boundary.
//
//   aicp_hip_parse_pm_yaml            the libpointmatcher chain subset loaded by
//                                     PointmatcherRegistration::applyConfig
//                                     (pointmatcher_registration.cpp:48-68, icp_.loadFromYaml)
//   aicp_hip_replace_ratio_config_file fileIO.cpp:179-214 (text rewrite, byte for byte)
//   aicp_hip_autotune_ratio           app.cpp:197-205 + the ostream/lexical_cast round trip
//
// yaml-cpp is not available in this image; the chain files only use block maps, block lists,
// plain scalars and comments, which the small parser below covers.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <limits>
#include <sstream>
#include <string>
#include <utility>
#include <vector>

#include "../../include/aicp_hip.h"

namespace {

struct Y {
  enum T { Null, Scalar, Map, List } t = Null;
  std::string s;
  std::vector<std::pair<std::string, Y>> map;
  std::vector<Y> list;
  const Y* get(const std::string& k) const {
    if (t != Map) return nullptr;
    for (auto& kv : map)
      if (kv.first == k) return &kv.second;
    return nullptr;
  }
};

struct Line {
  int indent;
  std::string text;
};

std::string trim(const std::string& s) {
  size_t a = s.find_first_not_of(" \t\r");
  if (a == std::string::npos) return "";
  size_t b = s.find_last_not_of(" \t\r");
  return s.substr(a, b - a + 1);
}

std::string unquote(const std::string& s) {
  if (s.size() >= 2 && ((s.front() == '"' && s.back() == '"') || (s.front() == '\'' && s.back() == '\'')))
    return s.substr(1, s.size() - 2);
  return s;
}

std::vector<Line> lex(std::istream& in) {
  std::vector<Line> out;
  std::string raw;
  while (std::getline(in, raw)) {
    // strip comments ('#' at line start or after whitespace, outside quotes)
    bool sq = false, dq = false;
    size_t cut = std::string::npos;
    for (size_t i = 0; i < raw.size(); ++i) {
      const char c = raw[i];
      if (c == '\'' && !dq) sq = !sq;
      if (c == '"' && !sq) dq = !dq;
      if (c == '#' && !sq && !dq && (i == 0 || raw[i - 1] == ' ' || raw[i - 1] == '\t')) {
        cut = i;
        break;
      }
    }
    if (cut != std::string::npos) raw = raw.substr(0, cut);
    for (auto& ch : raw)
      if (ch == '\t') ch = ' ';
    const std::string t = trim(raw);
    if (t.empty() || t == "---") continue;
    int ind = 0;
    while (ind < (int)raw.size() && raw[ind] == ' ') ++ind;
    out.push_back({ind, t});
  }
  return out;
}

// split "key: value" / "key:" ; returns false if the text has no mapping colon
bool split_kv(const std::string& t, std::string& k, std::string& v) {
  size_t p = std::string::npos;
  for (size_t i = 0; i < t.size(); ++i)
    if (t[i] == ':' && (i + 1 == t.size() || t[i + 1] == ' ')) {
      p = i;
      break;
    }
  if (p == std::string::npos) return false;
  k = unquote(trim(t.substr(0, p)));
  v = trim(t.substr(p + 1));
  return true;
}

Y parse_block(const std::vector<Line>& L, size_t& i, int indent);

Y parse_value_after(const std::vector<Line>& L, size_t& i, int parent_indent, const std::string& v) {
  Y y;
  if (!v.empty()) {
    if (v == "{}" ) {
      y.t = Y::Map;
    } else if (v == "[]") {
      y.t = Y::List;
    } else {
      y.t = Y::Scalar;
      y.s = unquote(v);
    }
    return y;
  }
  if (i < L.size() && L[i].indent > parent_indent) return parse_block(L, i, L[i].indent);
  // a list may sit at the same indent as its key
  if (i < L.size() && L[i].indent == parent_indent && L[i].text.rfind("- ", 0) == 0)
    return parse_block(L, i, L[i].indent);
  return y;  // null
}

Y parse_block(const std::vector<Line>& L, size_t& i, int indent) {
  Y y;
  if (i >= L.size()) return y;
  const bool isList = L[i].text == "-" || L[i].text.rfind("- ", 0) == 0;
  if (isList) {
    y.t = Y::List;
    while (i < L.size() && L[i].indent == indent &&
           (L[i].text == "-" || L[i].text.rfind("- ", 0) == 0)) {
      const std::string item = trim(L[i].text.substr(1));
      const int item_indent = indent + 2;
      ++i;
      std::string k, v;
      if (item.empty()) {
        y.list.push_back(parse_value_after(L, i, indent, ""));
      } else if (split_kv(item, k, v)) {
        Y m;
        m.t = Y::Map;
        m.map.emplace_back(k, parse_value_after(L, i, item_indent, v));
        while (i < L.size() && L[i].indent == item_indent && L[i].text.rfind("- ", 0) != 0) {
          std::string k2, v2;
          if (!split_kv(L[i].text, k2, v2)) break;
          ++i;
          m.map.emplace_back(k2, parse_value_after(L, i, item_indent, v2));
        }
        y.list.push_back(m);
      } else {
        Y s;
        s.t = Y::Scalar;
        s.s = unquote(item);
        y.list.push_back(s);
      }
    }
    return y;
  }
  std::string k, v;
  if (!split_kv(L[i].text, k, v)) {  // bare scalar block ("inspector:\n  NullInspector")
    y.t = Y::Scalar;
    y.s = unquote(L[i].text);
    ++i;
    return y;
  }
  y.t = Y::Map;
  while (i < L.size() && L[i].indent == indent) {
    if (!split_kv(L[i].text, k, v)) break;
    ++i;
    y.map.emplace_back(k, parse_value_after(L, i, indent, v));
  }
  return y;
}

bool to_float(const Y* y, float& out) {
  if (!y || y->t != Y::Scalar) return false;
  const char* s = y->s.c_str();
  char* end = nullptr;
  const float v = std::strtof(s, &end);  // boost::lexical_cast<float>
  if (end == s) return false;
  out = v;
  return true;
}
bool to_int(const Y* y, int32_t& out) {
  float f;
  if (!to_float(y, f)) return false;
  out = (int32_t)f;
  return true;
}

// element of a filter/checker list: a map with one key (class name) -> params map
bool list_items(const Y* y, std::vector<std::pair<std::string, const Y*>>& out) {
  out.clear();
  if (!y || y->t == Y::Null) return true;
  if (y->t != Y::List) return false;
  for (auto& it : y->list) {
    if (it.t == Y::Scalar) {
      out.emplace_back(it.s, nullptr);
    } else if (it.t == Y::Map && it.map.size() == 1) {
      out.emplace_back(it.map[0].first, &it.map[0].second);
    } else {
      return false;
    }
  }
  return true;
}

// A single-key map ("matcher: {KDTreeMatcher: {...}}") or a bare name.
bool single(const Y* y, std::string& name, const Y*& params) {
  if (!y) return false;
  if (y->t == Y::Scalar) {
    name = y->s;
    params = nullptr;
    return true;
  }
  if (y->t == Y::Map && y->map.size() == 1) {
    name = y->map[0].first;
    params = &y->map[0].second;
    return true;
  }
  return false;
}

const Y* param(const Y* params, const char* k) { return params ? params->get(k) : nullptr; }

}  // namespace

extern "C" {

void aicp_hip_default_config(aicp_icp_config* c) {
  // icp_autotuned_default.yaml:9-51
  c->knn_normals = 20;
  c->nn_epsilon = 3.16f;
  c->nn_max_dist = std::numeric_limits<float>::infinity();
  c->trimmed_ratio = 0.70f;
  c->max_iter = 20;
  c->min_diff_rot = 0.001f;
  c->min_diff_trans = 0.01f;
  c->smooth_length = 4;
  c->bucket_size = 8;
  c->knn_match = 1;
}

int aicp_hip_parse_pm_yaml(const char* path, aicp_icp_config* out) {
  if (!path || !out) return AICP_ERR_INVALID;
  std::ifstream f(path);
  if (!f.good()) return AICP_ERR_INVALID;  // "Cannot open config file" -> exit(1)
  std::vector<Line> L = lex(f);
  size_t i = 0;
  Y root = parse_block(L, i, L.empty() ? 0 : L[0].indent);
  if (root.t != Y::Map || i != L.size()) return AICP_ERR_INVALID;
  aicp_icp_config c;
  // libpointmatcher 1.2.x parameter defaults of the chain elements
  c.knn_normals = 5;
  c.nn_epsilon = 0.f;
  c.nn_max_dist = std::numeric_limits<float>::infinity();
  c.trimmed_ratio = 0.85f;
  c.max_iter = 40;
  c.min_diff_rot = 0.001f;
  c.min_diff_trans = 0.001f;
  c.smooth_length = 3;
  c.bucket_size = 8;
  c.knn_match = 1;
  bool haveRefNormals = false, haveCounter = false, haveDifferential = false;
  std::vector<std::pair<std::string, const Y*>> items;

  for (auto& kv : root.map) {
    const std::string& key = kv.first;
    const Y* v = &kv.second;
    if (key == "readingDataPointsFilters" || key == "referenceDataPointsFilters") {
      if (!list_items(v, items)) return AICP_ERR_INVALID;
      for (auto& it : items) {
        if (it.first != "SurfaceNormalDataPointsFilter") return AICP_ERR_UNSUPPORTED;
        float eps = 0;
        if (to_float(param(it.second, "epsilon"), eps) && eps != 0.f) return AICP_ERR_UNSUPPORTED;
        int32_t keepNormals = 1;
        to_int(param(it.second, "keepNormals"), keepNormals);
        if (key == "referenceDataPointsFilters") {
          if (!keepNormals) return AICP_ERR_UNSUPPORTED;
          int32_t knn = 5;
          to_int(param(it.second, "knn"), knn);
          c.knn_normals = knn;
          haveRefNormals = true;
        }
      }
    } else if (key == "readingStepDataPointsFilters") {
      if (!list_items(v, items)) return AICP_ERR_INVALID;
      if (!items.empty()) return AICP_ERR_UNSUPPORTED;
    } else if (key == "matcher") {
      std::string name;
      const Y* p;
      if (!single(v, name, p)) return AICP_ERR_INVALID;
      if (name != "KDTreeMatcher") return AICP_ERR_UNSUPPORTED;
      to_int(param(p, "knn"), c.knn_match);
      to_float(param(p, "epsilon"), c.nn_epsilon);
      to_float(param(p, "maxDist"), c.nn_max_dist);
      int32_t st = 1;
      if (to_int(param(p, "searchType"), st) && st != 1) return AICP_ERR_UNSUPPORTED;
      if (c.knn_match != 1) return AICP_ERR_UNSUPPORTED;
    } else if (key == "outlierFilters") {
      if (!list_items(v, items)) return AICP_ERR_INVALID;
      if (items.size() != 1 || items[0].first != "TrimmedDistOutlierFilter") return AICP_ERR_UNSUPPORTED;
      to_float(param(items[0].second, "ratio"), c.trimmed_ratio);
    } else if (key == "errorMinimizer") {
      std::string name;
      const Y* p;
      if (!single(v, name, p)) return AICP_ERR_INVALID;
      if (name != "PointToPlaneErrorMinimizer") return AICP_ERR_UNSUPPORTED;
      int32_t f2d = 0;
      if (to_int(param(p, "force2D"), f2d) && f2d) return AICP_ERR_UNSUPPORTED;
    } else if (key == "transformationCheckers") {
      if (!list_items(v, items)) return AICP_ERR_INVALID;
      for (auto& it : items) {
        if (it.first == "CounterTransformationChecker") {
          to_int(param(it.second, "maxIterationCount"), c.max_iter);
          haveCounter = true;
        } else if (it.first == "DifferentialTransformationChecker") {
          to_float(param(it.second, "minDiffRotErr"), c.min_diff_rot);
          to_float(param(it.second, "minDiffTransErr"), c.min_diff_trans);
          to_int(param(it.second, "smoothLength"), c.smooth_length);
          haveDifferential = true;
        } else {
          return AICP_ERR_UNSUPPORTED;
        }
      }
    } else if (key == "transformations") {
      if (!list_items(v, items)) return AICP_ERR_INVALID;
      for (auto& it : items)
        if (it.first != "RigidTransformation") return AICP_ERR_UNSUPPORTED;
    } else if (key == "inspector" || key == "logger") {
      // observability only
    } else {
      return AICP_ERR_UNSUPPORTED;
    }
  }
  if (!haveRefNormals || !haveCounter) return AICP_ERR_UNSUPPORTED;
  if (!haveDifferential) {
    c.min_diff_rot = -1.f;  // never fires
    c.min_diff_trans = -1.f;
    c.smooth_length = 1;
  }
  *out = c;
  return AICP_OK;
}

int aicp_hip_replace_ratio_config_file(const char* in_file, const char* out_file, float ratio) {
  if (!in_file || !out_file) return AICP_ERR_INVALID;
  std::ifstream in;
  in.open(in_file, std::fstream::in);
  std::ofstream out;
  out.open(out_file, std::ofstream::out);
  if (!in || !out) return AICP_ERR_INVALID;
  const std::string word = "ratio: ";
  std::stringstream with;
  with << "ratio: " << ratio;
  const std::string replacement = with.str();
  const size_t len = word.length() + 4;
  std::string line;
  while (!in.eof()) {  // the reference's loop, including its extra trailing newline
    std::getline(in, line);
    const size_t pos = line.find(word);
    if (pos != std::string::npos) line.replace(pos, len, replacement);
    out << line << '\n';
  }
  return AICP_OK;
}

float aicp_hip_autotune_ratio(float overlap_percent) {
  float current_ratio = overlap_percent / 100.0;
  if (current_ratio < 0.25)
    current_ratio = 0.25;
  else if (current_ratio > 0.70)
    current_ratio = 0.70;
  std::stringstream ss;
  ss << current_ratio;
  return std::strtof(ss.str().c_str(), nullptr);
}

}  // extern "C"
