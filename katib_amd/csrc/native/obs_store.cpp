#include "obs_store.hpp"

#include <algorithm>
#include <cerrno>
#include <cstdlib>
#include <fstream>

#include "json_mini.hpp"

namespace katib {

std::string json_escape(const std::string& s) {
  std::string o;
  o.reserve(s.size() + 2);
  for (unsigned char c : s) {
    switch (c) {
      case '"': o += "\\\""; break;
      case '\\': o += "\\\\"; break;
      case '\n': o += "\\n"; break;
      case '\r': o += "\\r"; break;
      case '\t': o += "\\t"; break;
      default:
        if (c < 0x20) {
          char b[8];
          snprintf(b, sizeof(b), "\\u%04x", c);
          o += b;
        } else {
          o += static_cast<char>(c);
        }
    }
  }
  return o;
}

ObservationStore::~ObservationStore() { close_journal(); }

uint32_t ObservationStore::intern(const std::string& name) {
  auto it = metric_ids_.find(name);
  if (it != metric_ids_.end()) return it->second;
  uint32_t id = static_cast<uint32_t>(metric_names_.size());
  metric_names_.push_back(name);
  metric_ids_.emplace(name, id);
  return id;
}

bool ObservationStore::report(const std::string& trial, const std::vector<LogTuple>& logs, std::string* err) {
  std::vector<LogRow> parsed;
  parsed.reserve(logs.size());
  for (const auto& l : logs) {
    const std::string& ts = std::get<0>(l);
    if (ts.empty()) continue;
    Timestamp t;
    if (!parse_rfc3339(ts, t)) {
      if (err) *err = "Error parsing start time " + ts;
      return false;
    }
    LogRow r;
    r.ts = t;
    r.ts_str = ts;
    r.value = std::get<2>(l);
    r.metric = 0;
    parsed.push_back(std::move(r));
  }
  std::lock_guard<std::mutex> g(mu_);
  auto& vec = rows_[trial];
  size_t i = 0;
  for (const auto& l : logs) {
    if (std::get<0>(l).empty()) continue;
    parsed[i].metric = intern(std::get<1>(l));
    ++i;
  }
  vec.insert(vec.end(), std::make_move_iterator(parsed.begin()), std::make_move_iterator(parsed.end()));
  journal_write("report", trial, &logs);
  return true;
}

std::vector<LogTuple> ObservationStore::get(const std::string& trial, const std::string& metric,
                                            const std::string& start, const std::string& end,
                                            std::string* err) const {
  std::vector<LogTuple> out;
  Timestamp ts_start, ts_end;
  bool has_start = !start.empty(), has_end = !end.empty();
  if (has_start && !parse_rfc3339(start, ts_start)) {
    if (err) *err = "Error parsing start time " + start;
    return out;
  }
  if (has_end && !parse_rfc3339(end, ts_end)) {
    if (err) *err = "Error parsing completion time " + end;
    return out;
  }
  std::lock_guard<std::mutex> g(mu_);
  auto it = rows_.find(trial);
  if (it == rows_.end()) return out;
  int64_t mid = -1;
  if (!metric.empty()) {
    auto m = metric_ids_.find(metric);
    if (m == metric_ids_.end()) return out;
    mid = m->second;
  }
  std::vector<const LogRow*> sel;
  sel.reserve(it->second.size());
  for (const auto& r : it->second) {
    if (mid >= 0 && r.metric != static_cast<uint32_t>(mid)) continue;
    if (has_start && r.ts < ts_start) continue;
    if (has_end && r.ts > ts_end) continue;
    sel.push_back(&r);
  }
  std::stable_sort(sel.begin(), sel.end(), [](const LogRow* a, const LogRow* b) { return a->ts < b->ts; });
  out.reserve(sel.size());
  for (const LogRow* r : sel) out.emplace_back(format_rfc3339_nano(r->ts), metric_names_[r->metric], r->value);
  return out;
}

void ObservationStore::remove(const std::string& trial) {
  std::lock_guard<std::mutex> g(mu_);
  rows_.erase(trial);
  journal_write("delete", trial, nullptr);
}

std::vector<std::string> ObservationStore::trials() const {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<std::string> out;
  for (const auto& kv : rows_) out.push_back(kv.first);
  std::sort(out.begin(), out.end());
  return out;
}

size_t ObservationStore::size(const std::string& trial) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = rows_.find(trial);
  return it == rows_.end() ? 0 : it->second.size();
}

size_t ObservationStore::total_rows() const {
  std::lock_guard<std::mutex> g(mu_);
  size_t n = 0;
  for (const auto& kv : rows_) n += kv.second.size();
  return n;
}

static bool parse_float(const std::string& s, double& v) {
  // strconv.ParseFloat(s, 64): whole string must be a number; accepts inf/nan spellings.
  if (s.empty()) return false;
  const char* b = s.c_str();
  char* e = nullptr;
  errno = 0;
  v = strtod(b, &e);
  if (e != b + s.size()) return false;
  // strtod accepts hex floats and leading spaces which Go rejects
  if (s[0] == ' ' || s[0] == '\t' || s[0] == '\n') return false;
  if (s.find("0x") != std::string::npos || s.find("0X") != std::string::npos) return false;
  return true;
}

std::vector<MetricSummary> ObservationStore::reduce(const std::string& trial,
                                                    const std::vector<std::string>& names) const {
  const std::string unavailable = "unavailable";
  struct Acc {
    std::string min, max, latest;
    double fmin = 0, fmax = 0;
    bool has_ts = false;
    Timestamp ts;
  };
  std::vector<Acc> acc(names.size(), Acc{unavailable, unavailable, unavailable});
  std::lock_guard<std::mutex> g(mu_);
  auto it = rows_.find(trial);
  if (it != rows_.end()) {
    std::vector<int> slot(metric_names_.size(), -1);
    for (size_t i = 0; i < names.size(); ++i) {
      auto m = metric_ids_.find(names[i]);
      if (m != metric_ids_.end()) slot[m->second] = static_cast<int>(i);
    }
    // rows in the order GetObservationLog returns them (by time, stable)
    std::vector<const LogRow*> sel;
    for (const auto& r : it->second)
      if (r.metric < slot.size() && slot[r.metric] >= 0) sel.push_back(&r);
    std::stable_sort(sel.begin(), sel.end(), [](const LogRow* a, const LogRow* b) { return a->ts < b->ts; });
    for (const LogRow* r : sel) {
      Acc& a = acc[slot[r->metric]];
      double f;
      if (parse_float(r->value, f)) {
        if (a.min == unavailable) {
          a.min = a.max = r->value;
          a.fmin = a.fmax = f;
        } else if (f < a.fmin) {
          a.min = r->value;
          a.fmin = f;
        } else if (f > a.fmax) {
          a.max = r->value;
          a.fmax = f;
        }
      }
      if (!a.has_ts || !(a.ts > r->ts)) {
        a.has_ts = true;
        a.ts = r->ts;
        a.latest = r->value;
      }
    }
  }
  std::vector<MetricSummary> out;
  for (size_t i = 0; i < names.size(); ++i) out.emplace_back(names[i], acc[i].min, acc[i].max, acc[i].latest);
  return out;
}

bool ObservationStore::open_journal(const std::string& path) {
  std::lock_guard<std::mutex> g(mu_);
  if (journal_) fclose(journal_);
  journal_ = fopen(path.c_str(), "a");
  return journal_ != nullptr;
}

void ObservationStore::close_journal() {
  std::lock_guard<std::mutex> g(mu_);
  if (journal_) {
    fclose(journal_);
    journal_ = nullptr;
  }
}

void ObservationStore::journal_write(const std::string& op, const std::string& trial,
                                     const std::vector<LogTuple>* logs) {
  if (!journal_) return;
  std::string line = "{\"op\":\"" + op + "\",\"trial\":\"" + json_escape(trial) + "\"";
  if (logs) {
    line += ",\"logs\":[";
    bool first = true;
    for (const auto& l : *logs) {
      if (std::get<0>(l).empty()) continue;
      if (!first) line += ",";
      first = false;
      line += "[\"" + json_escape(std::get<0>(l)) + "\",\"" + json_escape(std::get<1>(l)) + "\",\"" +
              json_escape(std::get<2>(l)) + "\"]";
    }
    line += "]";
  }
  line += "}\n";
  fwrite(line.data(), 1, line.size(), journal_);
  fflush(journal_);
}

size_t ObservationStore::load_journal(const std::string& path) {
  std::ifstream in(path);
  if (!in) return 0;
  std::string line;
  size_t n = 0;
  FILE* saved;
  {
    std::lock_guard<std::mutex> g(mu_);
    saved = journal_;
    journal_ = nullptr;  // do not re-journal replayed ops
  }
  while (std::getline(in, line)) {
    if (line.empty()) continue;
    json::Value v;
    if (!json::parse(line, v) || v.type != json::Value::Object) continue;
    const json::Value* op = v.get("op");
    const json::Value* trial = v.get("trial");
    if (!op || !trial) continue;
    if (op->str == "delete") {
      remove(trial->str);
    } else if (op->str == "report") {
      const json::Value* logs = v.get("logs");
      std::vector<LogTuple> lt;
      if (logs && logs->type == json::Value::Array) {
        for (const auto& row : logs->arr) {
          if (row.type != json::Value::Array || row.arr.size() != 3) continue;
          lt.emplace_back(row.arr[0].str, row.arr[1].str, row.arr[2].str);
        }
      }
      report(trial->str, lt);
    }
    ++n;
  }
  std::lock_guard<std::mutex> g(mu_);
  journal_ = saved;
  return n;
}

}  // namespace katib
