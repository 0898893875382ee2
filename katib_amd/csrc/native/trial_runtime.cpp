#include "trial_runtime.hpp"

#include <dirent.h>
#include <fcntl.h>
#include <signal.h>
#include <sys/epoll.h>
#include <sys/prctl.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstring>
#include <fstream>
#include <sstream>

extern char** environ;

namespace katib {

static const double kTermGraceSeconds = 10.0;
static const size_t kTailLines = 64;
static const char kProtoMark = '\x1e';

static double mono_now() {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

// ----------------------------------------------------------------------------------- SlotPool
SlotPool::SlotPool(int n_devices, int slots_per_device)
    : n_(n_devices), per_(std::max(1, slots_per_device)), used_(n_devices, 0), faults_(n_devices, 0) {}

std::vector<int> SlotPool::acquire(int n, bool distinct) {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<int> out;
  if (n <= 0) return out;
  // least-loaded devices first so parallel trials spread one per GPU
  // A multi-GPU trial takes n slots on n distinct devices when it can; with more slots
  // than devices per trial (slots_per_device > 1, e.g. a 2-rank trial on a 1-GPU box)
  // the remaining slots are stacked on the least-loaded devices already chosen.
  std::vector<int> order;
  int free_total = 0;
  for (int d = 0; d < n_; ++d)
    if (!bad_.count(d) && used_[d] < per_) {
      order.push_back(d);
      free_total += per_ - used_[d];
    }
  if (free_total < n) return out;
  // a single process that drives n GPUs needs n DIFFERENT devices (stacking is for rank plans,
  // where each slot is its own process)
  if (distinct && (int)order.size() < n) return out;
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return used_[a] < used_[b]; });
  std::vector<int> take(n_, 0);
  int got = 0;
  while (got < n) {  // round-robin over the candidates: distinct devices first
    for (int d : order) {
      if (got == n) break;
      if (used_[d] + take[d] < per_) {
        take[d]++;
        got++;
      }
    }
  }
  for (int d = 0; d < n_; ++d)
    for (int k = 0; k < take[d]; ++k) {
      used_[d]++;
      out.push_back(d);
    }
  return out;
}

void SlotPool::release(const std::vector<int>& devices) {
  std::lock_guard<std::mutex> g(mu_);
  for (int d : devices)
    if (d >= 0 && d < n_ && used_[d] > 0) used_[d]--;
}

void SlotPool::quarantine(int device) {
  std::lock_guard<std::mutex> g(mu_);
  if (device >= 0 && device < n_) bad_.insert(device);
}

void SlotPool::record_fault(int device, int threshold) {
  std::lock_guard<std::mutex> g(mu_);
  if (device < 0 || device >= n_) return;
  if (++faults_[device] >= threshold) bad_.insert(device);
}

int SlotPool::free_slots() const {
  std::lock_guard<std::mutex> g(mu_);
  int f = 0;
  for (int d = 0; d < n_; ++d)
    if (!bad_.count(d)) f += per_ - used_[d];
  return f;
}

int SlotPool::capacity() const {
  std::lock_guard<std::mutex> g(mu_);
  return (n_ - static_cast<int>(bad_.size())) * per_;
}

std::vector<int> SlotPool::quarantined() const {
  std::lock_guard<std::mutex> g(mu_);
  return std::vector<int>(bad_.begin(), bad_.end());
}

// ----------------------------------------------------------------------------------- runtime
struct TrialRuntime::Proc {
  std::string trial;
  pid_t pid = -1;
  int fd = -1;
  int worker = -1;
  FILE* log = nullptr;
  std::string partial;
  std::unique_ptr<MetricsParser> parser;
  CollectorConfig cfg;
  std::vector<StopRule> rules;
  std::vector<std::string> rule_names;
  std::map<std::string, int> start_steps;
  bool has_opt = false;
  double opt = 0;
  bool early_stopped = false, killed = false, deadline_exceeded = false, metrics_error = false;
  std::vector<LogTuple> logs;
  std::deque<std::string> tail;
  double deadline = 0;
  double term_sent_at = 0;
  long file_off = 0;
  std::string file_partial;
};

struct TrialRuntime::Worker {
  int id = -1;
  pid_t pid = -1;
  int in_fd = -1;
  int out_fd = -1;
  FILE* log = nullptr;
  std::string partial;
  std::string current;
  bool ready = false;
  bool alive = true;
};

TrialRuntime::TrialRuntime(std::shared_ptr<ObservationStore> store) : store_(std::move(store)) {
  epfd_ = epoll_create1(EPOLL_CLOEXEC);
  signal(SIGPIPE, SIG_IGN);
}

TrialRuntime::~TrialRuntime() {
  shutdown();
  if (epfd_ >= 0) close(epfd_);
}

void TrialRuntime::add_fd(int fd) {
  struct epoll_event ev;
  memset(&ev, 0, sizeof(ev));
  ev.events = EPOLLIN | EPOLLHUP | EPOLLRDHUP;
  ev.data.fd = fd;
  epoll_ctl(epfd_, EPOLL_CTL_ADD, fd, &ev);
}

void TrialRuntime::del_fd(int fd) { epoll_ctl(epfd_, EPOLL_CTL_DEL, fd, nullptr); }

static std::vector<char*> to_cstrs(const std::vector<std::string>& v) {
  std::vector<char*> out;
  for (const auto& s : v) out.push_back(const_cast<char*>(s.c_str()));
  out.push_back(nullptr);
  return out;
}

static std::vector<std::string> merged_env(const std::vector<std::string>& extra) {
  std::map<std::string, std::string> m;
  std::vector<std::string> order;
  for (char** e = environ; e && *e; ++e) {
    std::string kv(*e);
    size_t eq = kv.find('=');
    if (eq == std::string::npos) continue;
    std::string k = kv.substr(0, eq);
    if (!m.count(k)) order.push_back(k);
    m[k] = kv.substr(eq + 1);
  }
  for (const auto& kv : extra) {
    size_t eq = kv.find('=');
    if (eq == std::string::npos) continue;
    std::string k = kv.substr(0, eq);
    if (!m.count(k)) order.push_back(k);
    m[k] = kv.substr(eq + 1);
  }
  std::vector<std::string> out;
  for (const auto& k : order) out.push_back(k + "=" + m[k]);
  return out;
}

// fork + exec with stdout/stderr on `out_w`, stdin on `in_r` (or /dev/null).
static pid_t fork_exec(const std::vector<std::string>& argv, const std::vector<std::string>& env,
                       const std::string& cwd, int out_w, int in_r, std::string* err) {
  if (argv.empty()) {
    if (err) *err = "empty command";
    return -1;
  }
  std::vector<std::string> envs = merged_env(env);
  std::vector<char*> cargv = to_cstrs(argv), cenv = to_cstrs(envs);
  int errpipe[2];
  if (pipe2(errpipe, O_CLOEXEC) != 0) {
    if (err) *err = strerror(errno);
    return -1;
  }
  pid_t parent = getpid();
  pid_t pid = fork();
  if (pid < 0) {
    if (err) *err = strerror(errno);
    close(errpipe[0]);
    close(errpipe[1]);
    return -1;
  }
  if (pid == 0) {
    // child: only async-signal-safe calls until exec
    setpgid(0, 0);
    prctl(PR_SET_PDEATHSIG, SIGKILL);
    if (getppid() != parent) _exit(127);
    signal(SIGPIPE, SIG_DFL);
    int devnull = open("/dev/null", O_RDONLY);
    dup2(in_r >= 0 ? in_r : devnull, 0);
    dup2(out_w, 1);
    dup2(out_w, 2);
    if (!cwd.empty() && chdir(cwd.c_str()) != 0) {
      int e = errno;
      (void)!write(errpipe[1], &e, sizeof(e));
      _exit(127);
    }
    execvpe(cargv[0], cargv.data(), cenv.data());
    int e = errno;
    (void)!write(errpipe[1], &e, sizeof(e));
    _exit(127);
  }
  setpgid(pid, pid);
  close(errpipe[1]);
  int child_errno = 0;
  ssize_t r = read(errpipe[0], &child_errno, sizeof(child_errno));
  close(errpipe[0]);
  if (r == sizeof(child_errno)) {
    int st;
    waitpid(pid, &st, 0);
    if (err) *err = std::string("exec ") + argv[0] + ": " + strerror(child_errno);
    return -1;
  }
  return pid;
}

static CollectorConfig normalize(const CollectorConfig& c) { return c; }

pid_t TrialRuntime::spawn(const std::string& trial, const std::vector<std::string>& argv,
                          const std::vector<std::string>& env, const std::string& cwd, const std::string& log_path,
                          const CollectorConfig& cfg, double deadline_seconds) {
  std::lock_guard<std::mutex> g(mu_);
  if (procs_.count(trial)) return -1;
  int p[2];
  if (pipe2(p, O_CLOEXEC) != 0) return -1;
  std::string err;
  pid_t pid = fork_exec(argv, env, cwd, p[1], -1, &err);
  close(p[1]);
  if (pid < 0) {
    close(p[0]);
    // record the failure as a log line so the trial fails visibly
    if (!log_path.empty()) {
      FILE* f = fopen(log_path.c_str(), "a");
      if (f) {
        fprintf(f, "katib-amd: %s\n", err.c_str());
        fclose(f);
      }
    }
    return -1;
  }
  track(trial, pid, p[0], log_path, cfg, deadline_seconds);
  return pid;
}

bool TrialRuntime::adopt(const std::string& trial, pid_t pid, int fd, const std::string& log_path,
                         const CollectorConfig& cfg, double deadline_seconds) {
  std::lock_guard<std::mutex> g(mu_);
  if (procs_.count(trial) || pid <= 0 || fd < 0) return false;
  fcntl(fd, F_SETFD, fcntl(fd, F_GETFD) | FD_CLOEXEC);
  track(trial, pid, fd, log_path, cfg, deadline_seconds);
  return true;
}

// register a running trial process (mu_ held): its stdout pipe, collector and deadline
void TrialRuntime::track(const std::string& trial, pid_t pid, int fd, const std::string& log_path,
                         const CollectorConfig& cfg, double deadline_seconds) {
  int p[1] = {fd};
  fcntl(p[0], F_SETFL, fcntl(p[0], F_GETFL) | O_NONBLOCK);
  auto proc = std::make_unique<Proc>();
  proc->trial = trial;
  proc->pid = pid;
  proc->fd = p[0];
  proc->cfg = normalize(cfg);
  proc->parser = std::make_unique<MetricsParser>(cfg.metric_names, cfg.filters, cfg.format);
  proc->rules = cfg.rules;
  for (const auto& r : cfg.rules) {
    proc->rule_names.push_back(r.name);
    if (r.start_step != 0) proc->start_steps[r.name] = r.start_step;
  }
  if (!log_path.empty()) proc->log = fopen(log_path.c_str(), "a");
  if (deadline_seconds > 0) proc->deadline = mono_now() + deadline_seconds;
  fd_trial_[p[0]] = trial;
  pid_trial_[pid] = trial;
  add_fd(p[0]);
  procs_[trial] = std::move(proc);
}

int TrialRuntime::spawn_worker(const std::vector<std::string>& argv, const std::vector<std::string>& env,
                               const std::string& cwd, const std::string& log_path) {
  std::lock_guard<std::mutex> g(mu_);
  int out[2], in[2];
  if (pipe2(out, O_CLOEXEC) != 0) return -1;
  if (pipe2(in, O_CLOEXEC) != 0) {
    close(out[0]);
    close(out[1]);
    return -1;
  }
  std::string err;
  pid_t pid = fork_exec(argv, env, cwd, out[1], in[0], &err);
  close(out[1]);
  close(in[0]);
  if (pid < 0) {
    close(out[0]);
    close(in[1]);
    return -1;
  }
  fcntl(out[0], F_SETFL, fcntl(out[0], F_GETFL) | O_NONBLOCK);
  auto w = std::make_unique<Worker>();
  w->id = next_worker_++;
  w->pid = pid;
  w->in_fd = in[1];
  w->out_fd = out[0];
  if (!log_path.empty()) w->log = fopen(log_path.c_str(), "a");
  fd_worker_[out[0]] = w->id;
  pid_worker_[pid] = w->id;
  add_fd(out[0]);
  int id = w->id;
  workers_[id] = std::move(w);
  return id;
}

bool TrialRuntime::assign(int worker, const std::string& trial, const std::string& payload,
                          const std::string& log_path, const CollectorConfig& cfg, double deadline_seconds) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = workers_.find(worker);
  if (it == workers_.end() || !it->second->alive || !it->second->current.empty() || procs_.count(trial)) return false;
  Worker& w = *it->second;
  auto proc = std::make_unique<Proc>();
  proc->trial = trial;
  proc->pid = w.pid;
  proc->worker = worker;
  proc->cfg = cfg;
  proc->parser = std::make_unique<MetricsParser>(cfg.metric_names, cfg.filters, cfg.format);
  proc->rules = cfg.rules;
  for (const auto& r : cfg.rules) {
    proc->rule_names.push_back(r.name);
    if (r.start_step != 0) proc->start_steps[r.name] = r.start_step;
  }
  if (!log_path.empty()) proc->log = fopen(log_path.c_str(), "a");
  if (deadline_seconds > 0) proc->deadline = mono_now() + deadline_seconds;
  std::string line = payload;
  line.erase(std::remove(line.begin(), line.end(), '\n'), line.end());
  line += "\n";
  size_t off = 0;
  while (off < line.size()) {
    ssize_t n = write(w.in_fd, line.data() + off, line.size() - off);
    if (n < 0) {
      if (errno == EINTR) continue;
      if (proc->log) fclose(proc->log);
      return false;
    }
    off += static_cast<size_t>(n);
  }
  w.current = trial;
  procs_[trial] = std::move(proc);
  return true;
}

void TrialRuntime::handle_line(Proc& p, const std::string& raw) {
  std::string line = raw;
  if (!line.empty() && line.back() == '\r') line.pop_back();
  if (p.log) {
    fwrite(line.data(), 1, line.size(), p.log);
    fputc('\n', p.log);
  }
  p.tail.push_back(line);
  if (p.tail.size() > kTailLines) p.tail.pop_front();
  if (p.cfg.kind == CollectorKind::StdOut) {
    if (!p.parser->parse_line(line, p.logs)) p.metrics_error = true;
    if (!p.rules.empty() && !p.early_stopped) eval_rules(p, line);
  }
}

void TrialRuntime::eval_rules(Proc& p, const std::string& line) {
  std::vector<std::pair<std::string, double>> vals;
  p.parser->rule_values(line, p.rule_names, vals);
  const std::string obj = p.cfg.metric_names.empty() ? std::string() : p.cfg.metric_names[0];
  for (const auto& nv : vals) {
    for (size_t idx = 0; idx < p.rules.size();) {
      StopRule rule = p.rules[idx];
      if (rule.name != nv.first) {
        ++idx;
        continue;
      }
      double v = nv.second;
      if (rule.name == obj) {
        if (!p.has_opt) {
          p.opt = v;
          p.has_opt = true;
        } else if (p.cfg.objective_type == 2 && v > p.opt) {
          p.opt = v;
        } else if (p.cfg.objective_type == 1 && v < p.opt) {
          p.opt = v;
        }
        v = p.opt;
      }
      auto ss = p.start_steps.find(rule.name);
      if (ss != p.start_steps.end()) {
        ss->second--;
        if (ss->second != 0) {
          ++idx;
          continue;
        }
      }
      bool hit = (rule.comparison == Comparison::Equal && v == rule.value) ||
                 (rule.comparison == Comparison::Less && v < rule.value) ||
                 (rule.comparison == Comparison::Greater && v > rule.value);
      if (hit) {
        p.rules[idx] = p.rules.back();
        p.rules.pop_back();
      } else {
        ++idx;
      }
    }
  }
  if (p.rules.empty()) trigger_early_stop(p, nullptr);
}

void TrialRuntime::trigger_early_stop(Proc& p, std::vector<Event>*) {
  if (p.early_stopped) return;
  p.early_stopped = true;
  p.term_sent_at = mono_now();
  if (p.worker >= 0) {
    kill(p.pid, SIGUSR1);
  } else {
    kill(-p.pid, SIGTERM);
  }
}

void TrialRuntime::tail_file(Proc& p) {
  if (p.cfg.kind != CollectorKind::File || p.cfg.file_path.empty() || p.rules.empty() || p.early_stopped) return;
  FILE* f = fopen(p.cfg.file_path.c_str(), "r");
  if (!f) return;
  if (fseek(f, p.file_off, SEEK_SET) != 0) {
    fclose(f);
    return;
  }
  char buf[65536];
  size_t n;
  while ((n = fread(buf, 1, sizeof(buf), f)) > 0) {
    p.file_off += static_cast<long>(n);
    p.file_partial.append(buf, n);
  }
  fclose(f);
  size_t pos;
  while ((pos = p.file_partial.find('\n')) != std::string::npos) {
    std::string line = p.file_partial.substr(0, pos);
    p.file_partial.erase(0, pos + 1);
    if (!p.early_stopped) eval_rules(p, line);
  }
}

void TrialRuntime::handle_worker_output(Worker& w, const char* data, size_t n, std::vector<Event>& ev) {
  w.partial.append(data, n);
  size_t pos;
  while ((pos = w.partial.find('\n')) != std::string::npos) {
    std::string line = w.partial.substr(0, pos);
    w.partial.erase(0, pos + 1);
    if (!line.empty() && line[0] == kProtoMark) {
      if (line.compare(1, 5, "READY") == 0) {
        w.ready = true;
        Event e;
        e.type = EventType::WorkerReady;
        e.worker = w.id;
        ev.push_back(e);
      } else if (line.compare(1, 3, "END") == 0) {
        int code = atoi(line.c_str() + 4);
        if (!w.current.empty()) {
          auto it = procs_.find(w.current);
          std::string cur = w.current;
          w.current.clear();
          if (it != procs_.end()) finalize(*it->second, code, 0, ev, true);
        }
      }
      continue;
    }
    if (!w.current.empty()) {
      auto it = procs_.find(w.current);
      if (it != procs_.end()) {
        handle_line(*it->second, line);
        continue;
      }
    }
    if (w.log) {
      fwrite(line.data(), 1, line.size(), w.log);
      fputc('\n', w.log);
      fflush(w.log);
    }
  }
}

void TrialRuntime::read_fd(int fd, std::vector<Event>& ev) {
  char buf[65536];
  auto wt = fd_worker_.find(fd);
  while (true) {
    ssize_t n = read(fd, buf, sizeof(buf));
    if (n > 0) {
      if (wt != fd_worker_.end()) {
        auto w = workers_.find(wt->second);
        if (w != workers_.end()) handle_worker_output(*w->second, buf, static_cast<size_t>(n), ev);
      } else {
        auto tt = fd_trial_.find(fd);
        if (tt == fd_trial_.end()) return;
        auto p = procs_.find(tt->second);
        if (p == procs_.end()) return;
        Proc& pr = *p->second;
        pr.partial.append(buf, static_cast<size_t>(n));
        size_t pos;
        while ((pos = pr.partial.find('\n')) != std::string::npos) {
          std::string line = pr.partial.substr(0, pos);
          pr.partial.erase(0, pos + 1);
          handle_line(pr, line);
        }
      }
      continue;
    }
    if (n == 0) {  // EOF: stop watching; the process is reaped by waitpid
      del_fd(fd);
      return;
    }
    if (errno == EINTR) continue;
    return;  // EAGAIN
  }
}

void TrialRuntime::finalize(Proc& p, int code, int sig, std::vector<Event>& ev, bool from_worker) {
  if (!p.partial.empty()) {
    std::string rest = p.partial;
    p.partial.clear();
    handle_line(p, rest);
  }
  bool report = false;
  if (p.cfg.kind == CollectorKind::File) {
    std::ifstream in(p.cfg.file_path, std::ios::binary);
    if (in) {
      std::stringstream ss;
      ss << in.rdbuf();
      p.logs.clear();
      std::string err;
      if (!p.parser->parse_content(ss.str(), p.logs, &err)) p.metrics_error = true;
    } else if (!p.cfg.metric_names.empty()) {
      p.logs.clear();
      p.logs.emplace_back(zero_time_str(), p.cfg.metric_names[0], "unavailable");
    }
    report = true;
  } else if (p.cfg.kind == CollectorKind::StdOut) {
    if (!p.cfg.metric_names.empty()) {
      bool seen = false;
      for (const auto& l : p.logs)
        if (std::get<1>(l) == p.cfg.metric_names[0]) {
          seen = true;
          break;
        }
      if (!seen) {
        p.logs.clear();
        p.logs.emplace_back(zero_time_str(), p.cfg.metric_names[0], "unavailable");
      }
    }
    report = true;
  }
  if (report && !p.metrics_error) store_->report(p.trial, p.logs);
  if (p.log) {
    fclose(p.log);
    p.log = nullptr;
  }
  Event e;
  e.type = EventType::Exited;
  e.trial = p.trial;
  e.worker = p.worker;
  e.exit_code = code;
  e.signal = sig;
  e.early_stopped = p.early_stopped;
  e.killed = p.killed;
  e.deadline_exceeded = p.deadline_exceeded;
  e.metrics_error = p.metrics_error;
  if (!p.tail.empty()) e.message = p.tail.back();
  ev.push_back(e);
  if (!from_worker) {
    if (p.fd >= 0) {
      del_fd(p.fd);
      close(p.fd);
      fd_trial_.erase(p.fd);
    }
    pid_trial_.erase(p.pid);
  }
  procs_.erase(p.trial);  // destroys p
}

void TrialRuntime::reap(std::vector<Event>& ev) {
  std::vector<std::pair<pid_t, std::string>> tr(pid_trial_.begin(), pid_trial_.end());
  for (auto& kv : tr) {
    int st;
    pid_t r = waitpid(kv.first, &st, WNOHANG);
    if (r != kv.first) continue;
    auto it = procs_.find(kv.second);
    if (it == procs_.end()) continue;
    Proc& p = *it->second;
    if (p.fd >= 0) read_fd(p.fd, ev);  // drain what is left in the pipe
    int code = WIFEXITED(st) ? WEXITSTATUS(st) : 128 + (WIFSIGNALED(st) ? WTERMSIG(st) : 0);
    int sig = WIFSIGNALED(st) ? WTERMSIG(st) : 0;
    // the process group may still hold children: terminate them with their leader
    kill(-p.pid, SIGKILL);
    finalize(p, code, sig, ev, false);
  }
  std::vector<std::pair<pid_t, int>> wk(pid_worker_.begin(), pid_worker_.end());
  for (auto& kv : wk) {
    int st;
    pid_t r = waitpid(kv.first, &st, WNOHANG);
    if (r != kv.first) continue;
    auto wi = workers_.find(kv.second);
    if (wi == workers_.end()) continue;
    Worker& w = *wi->second;
    read_fd(w.out_fd, ev);
    w.alive = false;
    int sig = WIFSIGNALED(st) ? WTERMSIG(st) : 0;
    int code = WIFEXITED(st) ? WEXITSTATUS(st) : 128 + sig;
    if (!w.current.empty()) {
      auto it = procs_.find(w.current);
      w.current.clear();
      if (it != procs_.end()) finalize(*it->second, code == 0 ? 1 : code, sig, ev, true);
    }
    Event e;
    e.type = EventType::WorkerDied;
    e.worker = w.id;
    e.exit_code = code;
    e.signal = sig;
    ev.push_back(e);
    kill(-w.pid, SIGKILL);
    del_fd(w.out_fd);
    close(w.out_fd);
    close(w.in_fd);
    if (w.log) fclose(w.log);
    fd_worker_.erase(w.out_fd);
    pid_worker_.erase(w.pid);
    workers_.erase(wi);
  }
}

void TrialRuntime::check_deadlines(std::vector<Event>&) {
  double t = mono_now();
  for (auto& kv : procs_) {
    Proc& p = *kv.second;
    if (p.deadline > 0 && t > p.deadline && !p.deadline_exceeded) {
      p.deadline_exceeded = true;
      p.term_sent_at = t;
      if (p.worker >= 0) kill(p.pid, SIGUSR1);
      else kill(-p.pid, SIGKILL);
    }
    if (p.term_sent_at > 0 && t - p.term_sent_at > kTermGraceSeconds) {
      // escalation: for workers this kills the worker (it did not honour SIGUSR1)
      kill(-p.pid, SIGKILL);
      p.term_sent_at = t + 1e9;
    }
    tail_file(p);
  }
}

// Orphans re-parented to this process (child subreaper): zombie children that no table here knows.
// waitpid(-1) would also take the exit status of a tracked trial or of a child some other code in
// this process waits for, so the zombies are found by pid instead: /proc/<pid>/stat with this process
// as parent and state Z, at most once a second. Children in this process's own process group are left
// alone (every trial and worker leads its own group; a Popen / subprocess.run of the scheduler's own
// code stays in ours and is reaped by its caller), as are the pids registered in keep_.
void TrialRuntime::reap_orphans() {
  if (!reap_orphans_) return;
  double t = mono_now();
  if (t < orphan_scan_at_) return;
  orphan_scan_at_ = t + 1.0;
  const pid_t self = getpid(), grp = getpgrp();
  DIR* d = opendir("/proc");
  if (!d) return;
  std::vector<pid_t> zombies;
  while (struct dirent* de = readdir(d)) {
    const char* nm = de->d_name;
    if (nm[0] < '1' || nm[0] > '9') continue;
    char path[64];
    snprintf(path, sizeof(path), "/proc/%s/stat", nm);
    FILE* f = fopen(path, "re");
    if (!f) continue;
    char buf[512];
    size_t len = fread(buf, 1, sizeof(buf) - 1, f);
    fclose(f);
    buf[len] = 0;
    const char* rp = strrchr(buf, ')');  // comm may hold spaces and parentheses
    if (!rp) continue;
    char state = 0;
    int ppid = 0, pgrp = 0;
    if (sscanf(rp + 1, " %c %d %d", &state, &ppid, &pgrp) != 3) continue;
    if (state != 'Z' || ppid != self || pgrp == grp) continue;
    pid_t pid = static_cast<pid_t>(atoi(nm));
    if (pid_trial_.count(pid) || pid_worker_.count(pid) || keep_.count(pid)) continue;
    zombies.push_back(pid);
  }
  closedir(d);
  for (pid_t pid : zombies) {
    int st;
    if (waitpid(pid, &st, WNOHANG) == pid) ++orphans_reaped_;
  }
}

void TrialRuntime::set_reap_orphans(bool on, const std::vector<int>& keep) {
  std::lock_guard<std::mutex> g(mu_);
  reap_orphans_ = on;
  keep_.clear();
  for (int p : keep) keep_.insert(static_cast<pid_t>(p));
  orphan_scan_at_ = 0.0;
}

long TrialRuntime::orphans_reaped() const {
  std::lock_guard<std::mutex> g(mu_);
  return orphans_reaped_;
}

std::vector<Event> TrialRuntime::poll(int timeout_ms) {
  std::vector<Event> ev;
  struct epoll_event evs[64];
  int n = epoll_wait(epfd_, evs, 64, timeout_ms);
  std::lock_guard<std::mutex> g(mu_);
  for (int i = 0; i < n; ++i) read_fd(evs[i].data.fd, ev);
  reap(ev);
  reap_orphans();
  check_deadlines(ev);
  return ev;
}

bool TrialRuntime::kill_trial(const std::string& trial, bool early_stop) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = procs_.find(trial);
  if (it == procs_.end()) return false;
  Proc& p = *it->second;
  if (early_stop) {
    trigger_early_stop(p, nullptr);
    return true;
  }
  p.killed = true;
  p.term_sent_at = mono_now();
  if (p.worker >= 0) kill(p.pid, SIGUSR1);
  else kill(-p.pid, SIGTERM);
  return true;
}

void TrialRuntime::stop_worker(int worker) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = workers_.find(worker);
  if (it == workers_.end()) return;
  Worker& w = *it->second;
  if (w.in_fd >= 0) {
    close(w.in_fd);  // EOF on stdin: worker exits its loop
    w.in_fd = open("/dev/null", O_WRONLY | O_CLOEXEC);
  }
}

void TrialRuntime::shutdown() {
  std::lock_guard<std::mutex> g(mu_);
  for (auto& kv : pid_trial_) kill(-kv.first, SIGKILL);
  for (auto& kv : pid_worker_) kill(-kv.first, SIGKILL);
  for (auto& kv : pid_trial_) {
    int st;
    waitpid(kv.first, &st, 0);
  }
  for (auto& kv : pid_worker_) {
    int st;
    waitpid(kv.first, &st, 0);
  }
  for (auto& kv : procs_)
    if (kv.second->log) fclose(kv.second->log);
  for (auto& kv : workers_) {
    if (kv.second->log) fclose(kv.second->log);
    if (kv.second->out_fd >= 0) close(kv.second->out_fd);
    if (kv.second->in_fd >= 0) close(kv.second->in_fd);
  }
  for (auto& kv : fd_trial_) close(kv.first);
  procs_.clear();
  workers_.clear();
  fd_trial_.clear();
  fd_worker_.clear();
  pid_trial_.clear();
  pid_worker_.clear();
}

bool TrialRuntime::running(const std::string& trial) const {
  std::lock_guard<std::mutex> g(mu_);
  return procs_.count(trial) > 0;
}

std::vector<std::string> TrialRuntime::running_trials() const {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<std::string> out;
  for (const auto& kv : procs_) out.push_back(kv.first);
  return out;
}

std::vector<std::string> TrialRuntime::tail(const std::string& trial) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = procs_.find(trial);
  if (it == procs_.end()) return {};
  return std::vector<std::string>(it->second->tail.begin(), it->second->tail.end());
}

std::vector<LogTuple> TrialRuntime::live_logs(const std::string& trial) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = procs_.find(trial);
  if (it == procs_.end()) return {};
  return it->second->logs;
}

int TrialRuntime::worker_pid(int worker) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = workers_.find(worker);
  return it == workers_.end() ? -1 : it->second->pid;
}

bool TrialRuntime::worker_idle(int worker) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = workers_.find(worker);
  return it != workers_.end() && it->second->alive && it->second->ready && it->second->current.empty();
}

bool TrialRuntime::worker_alive(int worker) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = workers_.find(worker);
  return it != workers_.end() && it->second->alive;
}

int TrialRuntime::num_running() const {
  std::lock_guard<std::mutex> g(mu_);
  return static_cast<int>(procs_.size());
}

}  // namespace katib
