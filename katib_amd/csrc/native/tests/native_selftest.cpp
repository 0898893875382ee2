// Host-side self-test of the native runtime, built standalone (no Python) so it can run
// under AddressSanitizer + UndefinedBehaviorSanitizer and under ThreadSanitizer
// (katib_amd/_build.py build_selftest; tests/test_sanitizers.py). The reference runs
// `go test` without -race; here the pieces that own concurrency
// (observation store shared by the supervisor thread and the API, trial runtime with its
// event poll loop and process supervision) are exercised from several threads.
//
// Exit code 0 = all checks passed; a failed CHECK prints the expression and exits 1;
// a sanitizer report aborts with its own non-zero code.
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "../metrics_parser.hpp"
#include "../obs_store.hpp"
#include "../samplers.hpp"
#include "../status_engine.hpp"
#include "../trial_runtime.hpp"

using namespace katib;

#define CHECK(c)                                                          \
  do {                                                                    \
    if (!(c)) {                                                           \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::exit(1);                                                       \
    }                                                                     \
  } while (0)

static void test_store_concurrent() {
  ObservationStore st;
  const int kThreads = 4, kRows = 200;
  std::vector<std::thread> th;
  std::atomic<int> reads{0};
  for (int t = 0; t < kThreads; ++t)
    th.emplace_back([&, t] {
      const std::string trial = "trial-" + std::to_string(t);
      for (int i = 0; i < kRows; ++i) {
        char ts[64];
        std::snprintf(ts, sizeof ts, "2026-10-16T07:%02d:%02d.%06dZ", (i / 60) % 60, i % 60, i);
        std::string err;
        CHECK(st.report(trial, {LogTuple{ts, "loss", std::to_string(1.0 / (i + 1))}}, &err));
        if (i % 10 == 0) {
          auto r = st.get(trial, "loss", "", "", &err);
          CHECK(err.empty() && (int)r.size() == i + 1);
          auto red = st.reduce(trial, {"loss"});
          CHECK(red.size() == 1);
          reads++;
        }
      }
    });
  for (auto& x : th) x.join();
  CHECK(st.total_rows() == (size_t)kThreads * kRows);
  CHECK(reads.load() == kThreads * kRows / 10);
  auto red = st.reduce("trial-0", {"loss"});
  CHECK(std::get<0>(red[0]) == "loss");
  std::string err;
  CHECK(!st.report("bad", {LogTuple{"not-a-time", "loss", "1"}}, &err) && !err.empty());
  st.remove("trial-1");
  CHECK(st.size("trial-1") == 0);
}

static void test_parser() {
  MetricsParser p({"accuracy", "loss"}, {}, MetricsFormat::Text);
  std::vector<LogTuple> out;
  CHECK(p.parse_line("epoch 1: accuracy=0.91 loss=0.3", out));
  CHECK(out.size() == 2 && std::get<1>(out[0]) == "accuracy");
  out.clear();
  CHECK(p.parse_content("loss=0.5\nloss=0.4\n", out));
  bool unavailable = false;
  for (auto& r : out) unavailable |= std::get<2>(r) == "unavailable";
  CHECK(unavailable);  // objective never reported
  MetricsParser pf({"acc"}, {"([\\w|-]+)\\s*:\\s*([+-]?\\d*(\\.\\d+)?)"}, MetricsFormat::Text);
  auto m = pf.matches("acc: 0.5 other: 2");
  CHECK(m.size() == 2);
  MetricsParser pj({"acc"}, {}, MetricsFormat::Json);
  out.clear();
  CHECK(pj.parse_line("{\"acc\": \"0.7\", \"timestamp\": 1700000000.5}", out));
  CHECK(out.size() == 1);
  double v = 0;
  CHECK(go_parse_float("1e-3", v) && std::fabs(v - 1e-3) < 1e-15);
}

static void test_samplers() {
  CmaEs es({0.0, 0.0}, 0.5, {-3, -3}, {3, 3}, 7);
  for (int g = 0; g < 30 && !es.should_stop(); ++g) {
    std::vector<std::vector<double>> xs;
    std::vector<double> fs;
    for (int i = 0; i < es.popsize(); ++i) {
      auto x = es.ask();
      CHECK(x[0] >= -3 && x[0] <= 3 && x[1] >= -3 && x[1] <= 3);
      fs.push_back((x[0] - 1) * (x[0] - 1) + (x[1] + 0.5) * (x[1] + 0.5));
      xs.push_back(x);
    }
    es.tell(xs, fs);
  }
  auto mu = es.mean();
  CHECK(std::fabs(mu[0] - 1) < 0.2 && std::fabs(mu[1] + 0.5) < 0.2);
  std::vector<TpeDim> dims(2);
  std::vector<std::vector<double>> xs;
  std::vector<double> ls;
  for (int i = 0; i < 20; ++i) {
    xs.push_back({i / 20.0, 1 - i / 20.0});
    ls.push_back(std::fabs(i / 20.0 - 0.3));
  }
  TpeSettings s;
  auto x = tpe_sample(dims, xs, ls, s, 3);
  CHECK(x.size() == 2 && x[0] >= 0 && x[0] <= 1);
}

static void test_slots_concurrent() {
  SlotPool pool(8, 2);
  std::vector<std::thread> th;
  std::atomic<int> got{0};
  for (int t = 0; t < 4; ++t)
    th.emplace_back([&] {
      for (int i = 0; i < 100; ++i) {
        auto d = pool.acquire(1);
        if (!d.empty()) {
          got++;
          pool.release(d);
        }
      }
    });
  for (auto& x : th) x.join();
  CHECK(got.load() > 0 && pool.free_slots() == pool.capacity());
  pool.record_fault(3, 2);
  pool.record_fault(3, 2);
  CHECK(pool.quarantined().size() == 1 && pool.capacity() == 14);
  // multi-slot trials: distinct devices first, then stacked slots
  SlotPool one(1, 2);
  auto two = one.acquire(2);
  CHECK(two.size() == 2 && two[0] == 0 && two[1] == 0 && one.free_slots() == 0);
  CHECK(one.acquire(1).empty());
  SlotPool four(4, 2);
  auto a = four.acquire(3);
  CHECK(a.size() == 3 && a[0] != a[1] && a[1] != a[2]);
  auto b = four.acquire(5);
  CHECK(b.size() == 5 && four.free_slots() == 0);
}

static void test_runtime() {
  auto store = std::make_shared<ObservationStore>();
  TrialRuntime rt(store);
  CollectorConfig cfg;
  cfg.metric_names = {"score"};
  cfg.objective_type = 2;
  char tmpl[] = "/tmp/katib_selftest_XXXXXX";
  const char* dir = mkdtemp(tmpl);
  CHECK(dir != nullptr);
  const int kTrials = 6;
  for (int i = 0; i < kTrials; ++i) {
    const std::string name = "t" + std::to_string(i);
    const std::string cmd = "for s in 1 2 3; do echo score=$((s * " + std::to_string(i + 1) + ")); done";
    pid_t pid = rt.spawn(name, {"/bin/sh", "-c", cmd}, {"KATIB_SELFTEST=1"}, dir,
                         std::string(dir) + "/" + name + ".log", cfg, 30.0);
    CHECK(pid > 0);
  }
  // a trial killed mid-run and one that exceeds its deadline
  CHECK(rt.spawn("sleeper", {"/bin/sh", "-c", "sleep 30"}, {}, dir, std::string(dir) + "/s.log", cfg, 30.0) > 0);
  CHECK(rt.spawn("late", {"/bin/sh", "-c", "sleep 30"}, {}, dir, std::string(dir) + "/l.log", cfg, 0.3) > 0);
  std::atomic<bool> stop{false};
  std::thread reader([&] {  // API-side reads racing the supervisor's writes
    while (!stop.load()) {
      for (int i = 0; i < kTrials; ++i) (void)store->size("t" + std::to_string(i));
      (void)rt.num_running();
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
  });
  int exited = 0, deadline = 0;
  bool killed = false;
  auto t0 = std::chrono::steady_clock::now();
  while (exited < kTrials + 2 && std::chrono::steady_clock::now() - t0 < std::chrono::seconds(20)) {
    if (!killed && rt.running("sleeper")) killed = rt.kill_trial("sleeper", false);
    for (auto& ev : rt.poll(50)) {
      if (ev.type != EventType::Exited) continue;
      exited++;
      if (ev.deadline_exceeded) deadline++;
      if (ev.trial[0] == 't') CHECK(ev.exit_code == 0);
    }
  }
  stop = true;
  reader.join();
  CHECK(exited == kTrials + 2);
  CHECK(deadline == 1);
  for (int i = 0; i < kTrials; ++i) {
    auto red = store->reduce("t" + std::to_string(i), {"score"});
    CHECK(std::get<3>(red[0]) == std::to_string(3 * (i + 1)));  // latest
  }
  rt.shutdown();
  for (int i = 0; i < kTrials; ++i) unlink((std::string(dir) + "/t" + std::to_string(i) + ".log").c_str());
  unlink((std::string(dir) + "/s.log").c_str());
  unlink((std::string(dir) + "/l.log").c_str());
  rmdir(dir);
}

static void test_status_engine() {
  std::vector<TrialFacts> ts(4);
  ts[0].name = "a"; ts[0].conditions = kCondCreated | kCondSucceeded; ts[0].has_metric = true;
  ts[0].min = ts[0].max = ts[0].latest = "0.4"; ts[0].strategy = MetricStrategy::Min;
  ts[1] = ts[0]; ts[1].name = "b"; ts[1].min = "0.2";
  ts[2].name = "c"; ts[2].conditions = kCondCreated | kCondRunning;
  ts[3].name = "d"; ts[3].conditions = kCondKilled | kCondFailed;
  TrialsSummary s = summarize_trials(ts, ObjectiveType::Minimize, true, 0.25);
  CHECK(s.best == 1 && s.goal_reached);
  StatusCounts c = counts_of(s);
  CHECK(c.succeeded == 2 && c.running == 1 && c.killed == 1 && c.failed == 0);
  CHECK(decide_condition(c, false, false, true, 1, true, 10) == ConditionOutcome::Running);
  c.metrics_unavailable = 1;
  CHECK(decide_condition(c, false, false, true, 1, true, 10) == ConditionOutcome::MaxFailedReached);
  AdmissionPlan p = plan_admission(c, 3, true, 10, 5, 0);
  CHECK(p.delete_count == 0 && p.add_count == 2 && p.requests == 7);
  CHECK(plan_restart(true, ResumePolicy::LongRunning, true, 12, 10, false) == RestartAction::Restart);
}

int main() {
  test_status_engine();
  test_store_concurrent();
  test_parser();
  test_samplers();
  test_slots_concurrent();
  test_runtime();
  std::printf("native_selftest: ok\n");
  return 0;
}
