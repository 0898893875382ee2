// In-memory observation-log store: the MI355X-node replacement for
// katib-db-manager + MySQL/Postgres (reference: cmd/db-manager/v1beta1/main.go,
// pkg/db/v1beta1/mysql/mysql.go:67-166, common/kdb.go:23-30).
//
// * Per-trial append-only vectors of (timestamp, metric id, value); metric names
//   are interned so a log row is 24 bytes + the value string.
// * get() implements GetObservationLog: optional metric filter, optional
//   [start, end] closed time range, rows ordered by time (stable, i.e. insertion
//   order breaks ties exactly like the auto-increment id does in the SQL table).
// * reduce() implements the trial controller's getMetrics()
//   (trial_controller_util.go:165-217) including its quirk that one value can
//   update min OR max but not both ("else if").
// * Optional append-only journal (one JSON line per batch) gives durability for
//   the FromVolume resume policy; load_journal() replays it.
// Thread-safe: the gRPC DBManager facade and the scheduler share one instance.
#pragma once
#include <cstdio>
#include <mutex>
#include <string>
#include <tuple>
#include <unordered_map>
#include <vector>

#include "timeutil.hpp"

namespace katib {

struct LogRow {
  Timestamp ts;
  uint32_t metric;
  std::string ts_str;  // original string (kept verbatim for round-trip)
  std::string value;
};

using LogTuple = std::tuple<std::string, std::string, std::string>;  // (timestamp, name, value)
using MetricSummary = std::tuple<std::string, std::string, std::string, std::string>;  // name,min,max,latest

class ObservationStore {
 public:
  ObservationStore() = default;
  ~ObservationStore();

  // ReportObservationLog. Rows with empty timestamps are skipped (mysql.go:72).
  // Returns false (and stores nothing) if a timestamp does not parse.
  bool report(const std::string& trial, const std::vector<LogTuple>& logs, std::string* err = nullptr);
  std::vector<LogTuple> get(const std::string& trial, const std::string& metric, const std::string& start,
                            const std::string& end, std::string* err = nullptr) const;
  void remove(const std::string& trial);
  std::vector<std::string> trials() const;
  size_t size(const std::string& trial) const;
  size_t total_rows() const;
  std::vector<MetricSummary> reduce(const std::string& trial, const std::vector<std::string>& metric_names) const;

  bool open_journal(const std::string& path);
  size_t load_journal(const std::string& path);
  void close_journal();

 private:
  uint32_t intern(const std::string& name);
  void journal_write(const std::string& op, const std::string& trial, const std::vector<LogTuple>* logs);

  mutable std::mutex mu_;
  std::unordered_map<std::string, std::vector<LogRow>> rows_;
  std::unordered_map<std::string, uint32_t> metric_ids_;
  std::vector<std::string> metric_names_;
  FILE* journal_ = nullptr;
};

std::string json_escape(const std::string& s);

}  // namespace katib
