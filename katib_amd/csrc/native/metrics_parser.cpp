#include "metrics_parser.hpp"

#include <cctype>
#include <cerrno>
#include <charconv>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <sstream>

#include "json_mini.hpp"

namespace katib {

static const char* kDefaultFilter = R"(([\w|-]+)\s*=\s*([+-]?\d*(\.\d+)?([Ee][+-]?\d+)?))";

static inline bool is_word(unsigned char c) { return std::isalnum(c) || c == '_'; }
static inline bool is_name_char(unsigned char c) { return is_word(c) || c == '|' || c == '-'; }
static inline bool is_re2_space(unsigned char c) {
  return c == ' ' || c == '\t' || c == '\n' || c == '\f' || c == '\r';
}
static inline bool is_digit(unsigned char c) { return c >= '0' && c <= '9'; }

std::string trim_space(const std::string& s) {
  // strings.TrimSpace (ASCII subset + \v)
  size_t b = 0, e = s.size();
  auto sp = [](unsigned char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\v' || c == '\f'; };
  while (b < e && sp(s[b])) ++b;
  while (e > b && sp(s[e - 1])) --e;
  return s.substr(b, e - b);
}

// Exact emulation of RE2 FindAllStringSubmatch for the default filter.
void default_filter_scan(const std::string& line, std::vector<std::pair<std::string, std::string>>& out) {
  const size_t n = line.size();
  size_t i = 0;
  while (i < n) {
    if (!is_name_char(line[i])) {
      ++i;
      continue;
    }
    // maximal name run starting at i; a shorter name never matches because the
    // next char would be a name char (neither \s nor '=').
    size_t j = i;
    while (j < n && is_name_char(line[j])) ++j;
    size_t k = j;
    while (k < n && is_re2_space(line[k])) ++k;
    if (k >= n || line[k] != '=') {
      // no match at any start inside this run either: the run always ends at j
      i = j;
      continue;
    }
    ++k;
    while (k < n && is_re2_space(line[k])) ++k;
    size_t vs = k;
    if (k < n && (line[k] == '+' || line[k] == '-')) ++k;
    while (k < n && is_digit(line[k])) ++k;
    if (k + 1 < n && line[k] == '.' && is_digit(line[k + 1])) {
      k += 1;
      while (k < n && is_digit(line[k])) ++k;
    }
    if (k < n && (line[k] == 'e' || line[k] == 'E')) {
      size_t e = k + 1;
      if (e < n && (line[e] == '+' || line[e] == '-')) ++e;
      if (e < n && is_digit(line[e])) {
        while (e < n && is_digit(line[e])) ++e;
        k = e;
      }
    }
    out.emplace_back(line.substr(i, j - i), line.substr(vs, k - vs));
    i = k > i ? k : i + 1;
  }
}

bool go_parse_float(const std::string& s, double& v) {
  if (s.empty()) return false;
  unsigned char c0 = s[0];
  if (std::isspace(c0)) return false;
  std::string t = s;
  // Go accepts underscores only with base prefixes; reject hex (strtod takes it)
  if (t.find('x') != std::string::npos || t.find('X') != std::string::npos) return false;
  const char* b = t.c_str();
  char* e = nullptr;
  errno = 0;
  v = strtod(b, &e);
  if (e != b + t.size()) return false;
  if (errno == ERANGE && std::isfinite(v) && v != 0) return false;
  return true;
}

std::string go_format_float_f(double v) {
  char buf[512];
  auto r = std::to_chars(buf, buf + sizeof(buf), v, std::chars_format::fixed);
  if (r.ec != std::errc()) return "";
  return std::string(buf, r.ptr);
}

std::string line_timestamp(const std::string& line) {
  size_t sp = line.find(' ');
  if (sp == std::string::npos) return zero_time_str();
  std::string tok = line.substr(0, sp);
  Timestamp t;
  if (!parse_rfc3339(tok, t)) return zero_time_str();
  return tok;
}

// Go's regexp (RE2 syntax) -> std::regex ECMAScript. RE2 reads a brace that does not
// form a repetition `{n}`, `{n,}`, `{n,m}` as a literal; ECMAScript rejects it, so such
// braces are escaped (the reference's own examples use `{metricName: ...}` filters).
// Named groups `(?P<n>` / `(?<n>` become plain capturing groups, `\A`/`\z` anchors
// map to ^/$, `\Q...\E` quoting is expanded and a leading `(?i)` sets icase.
std::string re2_to_ecmascript(const std::string& re, bool* icase) {
  std::string out;
  size_t i = 0;
  const size_t n = re.size();
  if (icase) *icase = false;
  if (re.compare(0, 4, "(?i)") == 0) {
    if (icase) *icase = true;
    i = 4;
  }
  bool in_class = false;
  auto quantifier_len = [&](size_t at) -> size_t {  // length of a valid {..} repetition at `at`, else 0
    size_t k = at + 1, d1 = 0, d2 = 0;
    while (k < n && is_digit(re[k])) ++k, ++d1;
    if (d1 == 0) return 0;
    if (k < n && re[k] == ',') {
      ++k;
      while (k < n && is_digit(re[k])) ++k, ++d2;
    }
    if (k < n && re[k] == '}') return k - at + 1;
    return 0;
  };
  while (i < n) {
    char c = re[i];
    if (c == '\\' && i + 1 < n) {
      char d = re[i + 1];
      if (!in_class && d == 'A') {
        out += '^';
      } else if (!in_class && d == 'z') {
        out += '$';
      } else if (d == 'Q') {
        size_t e = re.find("\\E", i + 2);
        std::string lit = re.substr(i + 2, e == std::string::npos ? std::string::npos : e - i - 2);
        for (char l : lit) {
          if (std::strchr("\\^$.|?*+()[]{}/-", l)) out += '\\';
          out += l;
        }
        i = e == std::string::npos ? n : e + 2;
        continue;
      } else {
        out += c;
        out += d;
      }
      i += 2;
      continue;
    }
    if (in_class) {
      if (c == ']') in_class = false;
      out += c;
      ++i;
      continue;
    }
    if (c == '[') {
      in_class = true;
      out += c;
      ++i;
      if (i < n && re[i] == '^') out += re[i++];
      if (i < n && re[i] == ']') out += "\\]", ++i;  // leading ']' is literal in RE2
      continue;
    }
    if (c == '(' && re.compare(i, 4, "(?P<") == 0) {
      size_t e = re.find('>', i);
      if (e != std::string::npos) {
        out += '(';
        i = e + 1;
        continue;
      }
    }
    if (c == '(' && re.compare(i, 3, "(?<") == 0 && i + 3 < n && re[i + 3] != '=' && re[i + 3] != '!') {
      size_t e = re.find('>', i);
      if (e != std::string::npos) {
        out += '(';
        i = e + 1;
        continue;
      }
    }
    if (c == '{') {
      const size_t q = quantifier_len(i);
      const bool has_atom = !out.empty() && out.back() != '(' && out.back() != '|';
      if (q && has_atom) {
        out.append(re, i, q);
        i += q;
        continue;
      }
      out += "\\{";
      ++i;
      continue;
    }
    if (c == '}') {
      out += "\\}";
      ++i;
      continue;
    }
    out += c;
    ++i;
  }
  return out;
}

MetricsParser::MetricsParser(std::vector<std::string> names, std::vector<std::string> filters, MetricsFormat fmt)
    : names_(std::move(names)), filters_(std::move(filters)), fmt_(fmt) {
  if (filters_.empty()) filters_.push_back(kDefaultFilter);
  for (const auto& f : filters_) {
    if (f == kDefaultFilter) {
      regexes_.push_back(nullptr);
    } else {
      try {
        bool icase = false;
        const std::string ecma = re2_to_ecmascript(f, &icase);
        auto flags = std::regex::ECMAScript;
        if (icase) flags |= std::regex::icase;
        regexes_.push_back(std::make_shared<std::regex>(ecma, flags));
      } catch (const std::regex_error&) {
        // regexp.Compile errors are ignored by GetFilterRegexpList (nil regexp);
        // validation rejects such filters before we get here.
        regexes_.push_back(std::make_shared<std::regex>("$^"));
      }
    }
  }
}

std::vector<std::pair<std::string, std::string>> MetricsParser::matches(const std::string& line) const {
  std::vector<std::pair<std::string, std::string>> out;
  for (const auto& re : regexes_) {
    if (!re) {
      default_filter_scan(line, out);
      continue;
    }
    auto begin = std::sregex_iterator(line.begin(), line.end(), *re);
    for (auto it = begin; it != std::sregex_iterator(); ++it) {
      const std::smatch& m = *it;
      if (m.size() < 3) continue;
      out.emplace_back(m[1].str(), m[2].str());
    }
  }
  return out;
}

static bool json_line_timestamp(const json::Value& obj, std::string& ts) {
  ts = zero_time_str();
  const json::Value* v = obj.get("timestamp");
  if (!v) return true;
  if (v->type == json::Value::String) {
    Timestamp t;
    if (!v->str.empty() && parse_rfc3339(v->str, t)) ts = v->str;
    return true;
  }
  if (v->type != json::Value::Number) return true;
  std::string s = go_format_float_f(v->num);
  size_t dot = s.find('.');
  std::string ip = dot == std::string::npos ? s : s.substr(0, dot);
  long long sec, nsec = 0;
  try {
    size_t pos;
    sec = std::stoll(ip, &pos);
    if (pos != ip.size()) return true;
    if (dot != std::string::npos) {
      std::string fp = s.substr(dot + 1);
      if (fp.size() > 18) return true;  // strconv.ParseInt overflow -> warning, no timestamp
      nsec = std::stoll(fp, &pos);
    }
  } catch (...) {
    return true;
  }
  Timestamp t;
  t.sec = sec + nsec / 1000000000LL;
  t.nsec = static_cast<int32_t>(nsec % 1000000000LL);
  ts = format_rfc3339_nano(t);
  return true;
}

bool MetricsParser::parse_line(const std::string& line, std::vector<LogTuple>& out) const {
  if (fmt_ == MetricsFormat::Json) {
    if (line.empty()) return true;
    json::Value obj;
    if (!json::parse(line, obj) || obj.type != json::Value::Object) return false;
    std::string ts;
    json_line_timestamp(obj, ts);
    for (const auto& m : names_) {
      const json::Value* v = obj.get(m);
      if (!v || v->type != json::Value::String) continue;
      out.emplace_back(ts, m, v->str);
    }
    return true;
  }
  bool is_metric_line = false;
  for (const auto& m : names_) {
    if (line.find(m) != std::string::npos) {
      is_metric_line = true;
      break;
    }
  }
  if (!is_metric_line) return true;
  std::string ts = line_timestamp(line);
  for (const auto& kv : matches(line)) {
    std::string name = trim_space(kv.first);
    std::string value = trim_space(kv.second);
    for (const auto& m : names_) {
      if (name != m) continue;
      out.emplace_back(ts, name, value);
      break;
    }
  }
  return true;
}

bool MetricsParser::parse_content(const std::string& content, std::vector<LogTuple>& out, std::string* err) const {
  size_t start = 0;
  while (start <= content.size()) {
    size_t nl = content.find('\n', start);
    std::string line = content.substr(start, nl == std::string::npos ? std::string::npos : nl - start);
    if (!parse_line(line, out)) {
      if (err) *err = "failed to parse the json object: " + line;
      return false;
    }
    if (nl == std::string::npos) break;
    start = nl + 1;
  }
  if (!names_.empty()) {
    bool seen = false;
    for (const auto& l : out)
      if (std::get<1>(l) == names_[0]) {
        seen = true;
        break;
      }
    if (!seen) {
      out.clear();
      out.emplace_back(zero_time_str(), names_[0], "unavailable");
    }
  }
  return true;
}

void MetricsParser::rule_values(const std::string& line, const std::vector<std::string>& rule_names,
                                std::vector<std::pair<std::string, double>>& out) const {
  if (fmt_ == MetricsFormat::Json) {
    json::Value obj;
    if (!json::parse(line, obj) || obj.type != json::Value::Object) return;
    for (const auto& r : rule_names) {
      const json::Value* v = obj.get(r);
      if (!v || v->type != json::Value::String) continue;
      double d;
      if (go_parse_float(trim_space(v->str), d)) out.emplace_back(r, d);
    }
    return;
  }
  bool is_rule_line = false;
  for (const auto& r : rule_names)
    if (line.find(r) != std::string::npos) {
      is_rule_line = true;
      break;
    }
  if (!is_rule_line) return;
  for (const auto& kv : matches(line)) {
    std::string name = trim_space(kv.first);
    double d;
    if (!go_parse_float(trim_space(kv.second), d)) continue;
    for (const auto& r : rule_names)
      if (r == name) {
        out.emplace_back(name, d);
        break;
      }
  }
}

}  // namespace katib
