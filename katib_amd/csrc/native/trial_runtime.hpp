// Trial runtime: process supervisor + live metrics collection + early-stopping
// enforcement + GPU slot pool. One instance per scheduler process.
//
// It replaces, on a single MI355X node, what the reference spreads over
// Kubernetes Jobs/Pods, the pod-mutating webhook and the metrics-collector
// sidecar:
//   * spawn(): fork/exec of the trial command in its own process group with
//     stdout+stderr on a pipe (the `sh -c "cmd 1>metrics.log 2>&1 && echo
//     completed > $$$$.pid"` wrapper of pod/utils.go:152-197), every line also
//     teed to the trial's log file;
//   * live line parsing with MetricsParser, rule evaluation with the
//     best-so-far objective and startStep countdown of
//     file-metricscollector/main.go:143-391, SIGTERM to the process group when
//     every rule is met (early stop), then SIGKILL after a grace period;
//   * epoll + waitpid instead of 1 s /proc polling (pns.go:40-181);
//   * activeDeadlineSeconds enforcement;
//   * warm worker processes (one per GPU slot, HIP context already created)
//     that run trial after trial from a line protocol - the per-trial pod start
//     cost disappears, which is what moves completed-trials/hour;
//   * SlotPool: device assignment for parallelTrialCount trials on 8 GPUs,
//     with quarantine of a device after repeated faults.
#pragma once
#include <sys/types.h>

#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <tuple>
#include <vector>

#include "metrics_parser.hpp"
#include "obs_store.hpp"

namespace katib {

enum class CollectorKind { StdOut = 0, File = 1, TfEvent = 2, None = 3, Custom = 4, Prometheus = 5 };
enum class Comparison { Equal = 0, Less = 1, Greater = 2 };

struct StopRule {
  std::string name;
  double value = 0;
  Comparison comparison = Comparison::Less;
  int start_step = 0;
};

struct CollectorConfig {
  CollectorKind kind = CollectorKind::StdOut;
  std::vector<std::string> metric_names;  // objective first
  std::vector<std::string> filters;
  MetricsFormat format = MetricsFormat::Text;
  std::string file_path;
  std::vector<StopRule> rules;
  int objective_type = 0;  // 1 minimize, 2 maximize
};

enum class EventType { Exited = 0, EarlyStopTriggered = 1, WorkerReady = 2, WorkerDied = 3 };

struct Event {
  EventType type;
  std::string trial;
  int worker = -1;
  int exit_code = 0;
  int signal = 0;
  bool early_stopped = false;
  bool killed = false;
  bool deadline_exceeded = false;
  bool metrics_error = false;
  std::string message;
};

class SlotPool {
 public:
  SlotPool(int n_devices, int slots_per_device);
  // returns device ids (size n) or empty if not enough free slots
  // n slots (least-loaded devices first); distinct: on n different devices or nothing
  std::vector<int> acquire(int n, bool distinct = false);
  void release(const std::vector<int>& devices);
  void quarantine(int device);
  void record_fault(int device, int threshold);
  int free_slots() const;
  int capacity() const;
  std::vector<int> quarantined() const;

 private:
  mutable std::mutex mu_;
  int n_, per_;
  std::vector<int> used_;
  std::vector<int> faults_;
  std::set<int> bad_;
};

class TrialRuntime {
 public:
  explicit TrialRuntime(std::shared_ptr<ObservationStore> store);
  ~TrialRuntime();

  // Spawn a trial process. env entries are "K=V" added on top of the parent env.
  pid_t spawn(const std::string& trial, const std::vector<std::string>& argv, const std::vector<std::string>& env,
              const std::string& cwd, const std::string& log_path, const CollectorConfig& cfg,
              double deadline_seconds);
  // Supervise a process started elsewhere (the fork server, controller/zygote.py) exactly like a
  // spawned one: `pid` must be this process's child (re-parented: child subreaper) and its own
  // process-group leader; `fd` is the read end of its stdout/stderr pipe (taken over, closed at exit).
  bool adopt(const std::string& trial, pid_t pid, int fd, const std::string& log_path, const CollectorConfig& cfg,
             double deadline_seconds);
  // Warm worker: a long-lived process speaking the \x1e line protocol.
  int spawn_worker(const std::vector<std::string>& argv, const std::vector<std::string>& env, const std::string& cwd,
                   const std::string& log_path);
  bool assign(int worker, const std::string& trial, const std::string& payload, const std::string& log_path,
              const CollectorConfig& cfg, double deadline_seconds);
  bool kill_trial(const std::string& trial, bool early_stop);
  void stop_worker(int worker);
  void shutdown();

  std::vector<Event> poll(int timeout_ms);

  bool running(const std::string& trial) const;
  std::vector<std::string> running_trials() const;
  std::vector<std::string> tail(const std::string& trial) const;
  std::vector<LogTuple> live_logs(const std::string& trial) const;
  int worker_pid(int worker) const;
  bool worker_idle(int worker) const;
  bool worker_alive(int worker) const;
  int num_running() const;
  // Child subreaper mode (controller/zygote.py): orphaned descendants of trials re-parent to this
  // process. With `on`, poll() also reaps zombie children this runtime does not track, except the
  // pids in `keep` (children that their own owner waits for, e.g. the fork server's Popen) and
  // children in this process's own process group (a caller's subprocess.run / Popen waits for
  // those itself). Returns the number of orphans reaped so far.
  void set_reap_orphans(bool on, const std::vector<int>& keep);
  long orphans_reaped() const;

 private:
  void track(const std::string& trial, pid_t pid, int fd, const std::string& log_path, const CollectorConfig& cfg,
             double deadline_seconds);
  struct Proc;
  struct Worker;
  void add_fd(int fd);
  void del_fd(int fd);
  void handle_line(Proc& p, const std::string& line);
  void handle_worker_output(Worker& w, const char* data, size_t n, std::vector<Event>& ev);
  void read_fd(int fd, std::vector<Event>& ev);
  void tail_file(Proc& p);
  void finalize(Proc& p, int status_code, int sig, std::vector<Event>& ev, bool from_worker);
  void eval_rules(Proc& p, const std::string& line);
  void trigger_early_stop(Proc& p, std::vector<Event>* ev);
  void reap(std::vector<Event>& ev);
  void check_deadlines(std::vector<Event>& ev);
  void reap_orphans();

  std::shared_ptr<ObservationStore> store_;
  int epfd_ = -1;
  std::map<std::string, std::unique_ptr<Proc>> procs_;  // trial -> proc
  std::map<int, std::unique_ptr<Worker>> workers_;      // id -> worker
  std::map<int, std::string> fd_trial_;                 // pipe fd -> trial (process trials)
  std::map<int, int> fd_worker_;                        // pipe fd -> worker id
  std::map<pid_t, std::string> pid_trial_;
  std::map<pid_t, int> pid_worker_;
  int next_worker_ = 0;
  bool reap_orphans_ = false;
  std::set<pid_t> keep_;
  double orphan_scan_at_ = 0.0;
  long orphans_reaped_ = 0;
  mutable std::mutex mu_;
};

}  // namespace katib
