// Metrics line parser: the native replacement of the file/StdOut metrics
// collector's parsing (reference pkg/metricscollector/v1beta1/file-metricscollector/
// file-metricscollector.go:45-252 and cmd/.../file-metricscollector/main.go:143-391).
//
// TEXT format: the default filter ([\w|-]+)\s*=\s*([+-]?\d*(\.\d+)?([Ee][+-]?\d+)?)
// runs on a hand-written scanner that reproduces RE2 leftmost-first
// FindAllStringSubmatch exactly (no regex engine on the hot path); custom
// filters use std::regex (ECMAScript ~ RE2 for the two-group patterns the
// validator admits).  An optional leading RFC3339 token is the line timestamp,
// otherwise the zero time 0001-01-01T00:00:00Z is used (reference parity).
// JSON format: one object per line; only *string* metric values are taken, and
// "timestamp" may be an RFC3339Nano string or float seconds (parity incl. the
// fractional-digits-as-nanoseconds quirk of parseTimestamp).
#pragma once
#include <memory>
#include <regex>
#include <string>
#include <utility>
#include <vector>

#include "obs_store.hpp"

namespace katib {

enum class MetricsFormat { Text = 0, Json = 1 };

class MetricsParser {
 public:
  MetricsParser(std::vector<std::string> metric_names, std::vector<std::string> filters, MetricsFormat fmt);

  // Collect metric logs from one line. Returns false on a JSON syntax error.
  bool parse_line(const std::string& line, std::vector<LogTuple>& out) const;
  // Whole-file collection (CollectObservationLog): appends the "unavailable"
  // objective row when the objective never appears.
  bool parse_content(const std::string& content, std::vector<LogTuple>& out, std::string* err = nullptr) const;
  // Numeric (name, value) pairs for early-stopping rule evaluation, with the
  // watchMetricsFile pre-filter semantics (line must mention a rule metric).
  void rule_values(const std::string& line, const std::vector<std::string>& rule_names,
                   std::vector<std::pair<std::string, double>>& out) const;

  const std::vector<std::string>& metric_names() const { return names_; }
  MetricsFormat format() const { return fmt_; }

  // exposed for tests: all (name, value) submatches of the filters on a line
  std::vector<std::pair<std::string, std::string>> matches(const std::string& line) const;

 private:
  std::vector<std::string> names_;
  std::vector<std::string> filters_;
  std::vector<std::shared_ptr<std::regex>> regexes_;  // nullptr == default fast path
  MetricsFormat fmt_;
};

void default_filter_scan(const std::string& line, std::vector<std::pair<std::string, std::string>>& out);
std::string line_timestamp(const std::string& line);
bool go_parse_float(const std::string& s, double& v);
std::string trim_space(const std::string& s);
std::string re2_to_ecmascript(const std::string& re, bool* icase = nullptr);
std::string go_format_float_f(double v);

}  // namespace katib
