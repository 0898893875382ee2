// pybind11 bindings for the native runtime (`katib_amd._native`).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <optional>
#include <regex>

#include "metrics_parser.hpp"
#include "obs_store.hpp"
#include "samplers.hpp"
#include "status_engine.hpp"
#include "timeutil.hpp"
#include "trial_runtime.hpp"

namespace py = pybind11;
using namespace katib;

namespace {

// ${trialParameters.X} substitution (manifest/generator.go:99-186 applyParameters,
// the final strings.Replace loop) + the leftover-placeholder scan of the validator.
std::string render_template(std::string tpl, const std::map<std::string, std::string>& values) {
  for (const auto& kv : values) {
    const std::string ph = "${trialParameters." + kv.first + "}";
    size_t pos = 0;
    while ((pos = tpl.find(ph, pos)) != std::string::npos) {
      tpl.replace(pos, ph.size(), kv.second);
      pos += kv.second.size();
    }
  }
  return tpl;
}

std::vector<std::string> unresolved_placeholders(const std::string& tpl) {
  static const std::regex re(R"(\$\{trialParameters\..+?\})");
  std::vector<std::string> out;
  for (auto it = std::sregex_iterator(tpl.begin(), tpl.end(), re); it != std::sregex_iterator(); ++it)
    out.push_back(it->str());
  return out;
}

CollectorConfig make_cfg(const py::dict& d) {
  CollectorConfig c;
  if (d.contains("kind")) c.kind = static_cast<CollectorKind>(d["kind"].cast<int>());
  if (d.contains("metric_names")) c.metric_names = d["metric_names"].cast<std::vector<std::string>>();
  if (d.contains("filters")) c.filters = d["filters"].cast<std::vector<std::string>>();
  if (d.contains("format")) c.format = static_cast<MetricsFormat>(d["format"].cast<int>());
  if (d.contains("file_path")) c.file_path = d["file_path"].cast<std::string>();
  if (d.contains("objective_type")) c.objective_type = d["objective_type"].cast<int>();
  if (d.contains("rules")) {
    for (auto r : d["rules"].cast<py::list>()) {
      py::dict rd = r.cast<py::dict>();
      StopRule s;
      s.name = rd["name"].cast<std::string>();
      s.value = rd["value"].cast<double>();
      s.comparison = static_cast<Comparison>(rd["comparison"].cast<int>());
      s.start_step = rd.contains("start_step") ? rd["start_step"].cast<int>() : 0;
      c.rules.push_back(s);
    }
  }
  return c;
}

py::dict event_dict(const Event& e) {
  py::dict d;
  static const char* names[] = {"exited", "early_stop_triggered", "worker_ready", "worker_died"};
  d["type"] = names[static_cast<int>(e.type)];
  d["trial"] = e.trial;
  d["worker"] = e.worker;
  d["exit_code"] = e.exit_code;
  d["signal"] = e.signal;
  d["early_stopped"] = e.early_stopped;
  d["killed"] = e.killed;
  d["deadline_exceeded"] = e.deadline_exceeded;
  d["metrics_error"] = e.metrics_error;
  d["message"] = e.message;
  return d;
}

// (pending, running, succeeded, failed, killed, early_stopped, metrics_unavailable)
using CountsTuple = std::tuple<int, int, int, int, int, int, int>;
StatusCounts counts_from(const CountsTuple& t) {
  StatusCounts c;
  std::tie(c.pending, c.running, c.succeeded, c.failed, c.killed, c.early_stopped, c.metrics_unavailable) = t;
  return c;
}

}  // namespace

PYBIND11_MODULE(_native, m) {
  m.doc() = "katib_amd native runtime: observation store, metrics parser, trial supervisor, samplers";

  m.def("render_template", &render_template);
  m.def("unresolved_placeholders", &unresolved_placeholders);
  m.def("parse_rfc3339", [](const std::string& s) -> py::object {
    Timestamp t;
    if (!parse_rfc3339(s, t)) return py::none();
    return py::make_tuple(t.sec, t.nsec);
  });
  m.def("format_rfc3339_nano", [](int64_t sec, int32_t nsec) {
    Timestamp t;
    t.sec = sec;
    t.nsec = nsec;
    return format_rfc3339_nano(t);
  });
  m.def("default_filter_scan", [](const std::string& line) {
    std::vector<std::pair<std::string, std::string>> out;
    default_filter_scan(line, out);
    return out;
  });
  m.def("re2_to_ecmascript", [](const std::string& re) {
    bool icase = false;
    std::string out = re2_to_ecmascript(re, &icase);
    return py::make_tuple(out, icase);
  });

  py::class_<ObservationStore, std::shared_ptr<ObservationStore>>(m, "ObservationStore")
      .def(py::init<>())
      .def("report",
           [](ObservationStore& s, const std::string& trial, const std::vector<LogTuple>& logs) {
             std::string err;
             py::gil_scoped_release rel;
             if (!s.report(trial, logs, &err)) throw std::invalid_argument(err);
           })
      .def(
          "get",
          [](const ObservationStore& s, const std::string& trial, const std::string& metric, const std::string& start,
             const std::string& end) {
            std::string err;
            auto r = s.get(trial, metric, start, end, &err);
            if (!err.empty()) throw std::invalid_argument(err);
            return r;
          },
          py::arg("trial"), py::arg("metric") = "", py::arg("start") = "", py::arg("end") = "")
      .def("remove", &ObservationStore::remove)
      .def("trials", &ObservationStore::trials)
      .def("size", &ObservationStore::size)
      .def("total_rows", &ObservationStore::total_rows)
      .def("reduce", &ObservationStore::reduce)
      .def("open_journal", &ObservationStore::open_journal)
      .def("load_journal", &ObservationStore::load_journal)
      .def("close_journal", &ObservationStore::close_journal);

  py::class_<MetricsParser>(m, "MetricsParser")
      .def(py::init([](std::vector<std::string> names, std::vector<std::string> filters, int fmt) {
             return new MetricsParser(std::move(names), std::move(filters), static_cast<MetricsFormat>(fmt));
           }),
           py::arg("metric_names"), py::arg("filters") = std::vector<std::string>{}, py::arg("format") = 0)
      .def("parse_line",
           [](const MetricsParser& p, const std::string& line) {
             std::vector<LogTuple> out;
             if (!p.parse_line(line, out)) throw std::invalid_argument("failed to parse the json object: " + line);
             return out;
           })
      .def("parse_content",
           [](const MetricsParser& p, const std::string& content) {
             std::vector<LogTuple> out;
             std::string err;
             if (!p.parse_content(content, out, &err)) throw std::invalid_argument(err);
             return out;
           })
      .def("rule_values",
           [](const MetricsParser& p, const std::string& line, const std::vector<std::string>& names) {
             std::vector<std::pair<std::string, double>> out;
             p.rule_values(line, names, out);
             return out;
           })
      .def("matches", &MetricsParser::matches);

  py::class_<SlotPool, std::shared_ptr<SlotPool>>(m, "SlotPool")
      .def(py::init<int, int>(), py::arg("n_devices"), py::arg("slots_per_device") = 1)
      .def("acquire", &SlotPool::acquire, py::arg("n"), py::arg("distinct") = false)
      .def("release", &SlotPool::release)
      .def("quarantine", &SlotPool::quarantine)
      .def("record_fault", &SlotPool::record_fault)
      .def("free_slots", &SlotPool::free_slots)
      .def("capacity", &SlotPool::capacity)
      .def("quarantined", &SlotPool::quarantined);

  py::class_<TrialRuntime>(m, "TrialRuntime")
      .def(py::init<std::shared_ptr<ObservationStore>>())
      .def(
          "spawn",
          [](TrialRuntime& r, const std::string& trial, const std::vector<std::string>& argv,
             const std::vector<std::string>& env, const std::string& cwd, const std::string& log_path,
             const py::dict& cfg, double deadline) {
            CollectorConfig c = make_cfg(cfg);
            py::gil_scoped_release rel;
            return static_cast<int>(r.spawn(trial, argv, env, cwd, log_path, c, deadline));
          },
          py::arg("trial"), py::arg("argv"), py::arg("env"), py::arg("cwd"), py::arg("log_path"), py::arg("collector"),
          py::arg("deadline") = 0.0)
      .def(
          "adopt",
          [](TrialRuntime& r, const std::string& trial, int pid, int fd, const std::string& log_path,
             const py::dict& cfg, double deadline) {
            CollectorConfig c = make_cfg(cfg);
            py::gil_scoped_release rel;
            return r.adopt(trial, static_cast<pid_t>(pid), fd, log_path, c, deadline);
          },
          py::arg("trial"), py::arg("pid"), py::arg("fd"), py::arg("log_path"), py::arg("collector"),
          py::arg("deadline") = 0.0)
      .def(
          "spawn_worker",
          [](TrialRuntime& r, const std::vector<std::string>& argv, const std::vector<std::string>& env,
             const std::string& cwd, const std::string& log_path) {
            py::gil_scoped_release rel;
            return r.spawn_worker(argv, env, cwd, log_path);
          },
          py::arg("argv"), py::arg("env"), py::arg("cwd"), py::arg("log_path"))
      .def(
          "assign",
          [](TrialRuntime& r, int worker, const std::string& trial, const std::string& payload,
             const std::string& log_path, const py::dict& cfg, double deadline) {
            CollectorConfig c = make_cfg(cfg);
            return r.assign(worker, trial, payload, log_path, c, deadline);
          },
          py::arg("worker"), py::arg("trial"), py::arg("payload"), py::arg("log_path"), py::arg("collector"),
          py::arg("deadline") = 0.0)
      .def("kill_trial", &TrialRuntime::kill_trial, py::arg("trial"), py::arg("early_stop") = false)
      .def("stop_worker", &TrialRuntime::stop_worker)
      .def("set_reap_orphans", &TrialRuntime::set_reap_orphans, py::arg("on"), py::arg("keep") = std::vector<int>{})
      .def("orphans_reaped", &TrialRuntime::orphans_reaped)
      .def("shutdown", &TrialRuntime::shutdown)
      .def("poll",
           [](TrialRuntime& r, int timeout_ms) {
             std::vector<Event> ev;
             {
               py::gil_scoped_release rel;
               ev = r.poll(timeout_ms);
             }
             py::list out;
             for (const auto& e : ev) out.append(event_dict(e));
             return out;
           })
      .def("running", &TrialRuntime::running)
      .def("running_trials", &TrialRuntime::running_trials)
      .def("tail", &TrialRuntime::tail)
      .def("live_logs", &TrialRuntime::live_logs)
      .def("worker_pid", &TrialRuntime::worker_pid)
      .def("worker_idle", &TrialRuntime::worker_idle)
      .def("worker_alive", &TrialRuntime::worker_alive)
      .def("num_running", &TrialRuntime::num_running);

  py::class_<SobolEngine>(m, "SobolEngine")
      .def(py::init<int, const std::vector<int64_t>&, const std::vector<std::vector<int64_t>>&>())
      .def("point", &SobolEngine::point)
      .def("points", &SobolEngine::points)
      .def_property_readonly("dim", &SobolEngine::dim);

  py::class_<CmaEs>(m, "CmaEs")
      .def(py::init<const std::vector<double>&, double, const std::vector<double>&, const std::vector<double>&,
                    uint64_t, int>(),
           py::arg("mean"), py::arg("sigma"), py::arg("lower"), py::arg("upper"), py::arg("seed") = 0,
           py::arg("popsize") = 0)
      .def("ask", &CmaEs::ask)
      .def("tell", &CmaEs::tell)
      .def("should_stop", &CmaEs::should_stop)
      .def_property_readonly("popsize", &CmaEs::popsize)
      .def_property_readonly("generation", &CmaEs::generation)
      .def_property_readonly("dim", &CmaEs::dim)
      .def_property_readonly("sigma", &CmaEs::sigma)
      .def_property_readonly("mean", &CmaEs::mean)
      .def_property_readonly("cov", &CmaEs::cov);

  m.def(
      "tpe_sample",
      [](const std::vector<py::dict>& dims, const std::vector<std::vector<double>>& xs,
         const std::vector<double>& losses, const py::dict& settings, uint64_t seed) {
        std::vector<TpeDim> td;
        for (const auto& d : dims) {
          TpeDim t;
          t.kind = d.contains("kind") ? d["kind"].cast<int>() : 0;
          t.low = d.contains("low") ? d["low"].cast<double>() : 0;
          t.high = d.contains("high") ? d["high"].cast<double>() : 1;
          t.q = d.contains("q") ? d["q"].cast<double>() : 0;
          t.n_choices = d.contains("n_choices") ? d["n_choices"].cast<int>() : 0;
          td.push_back(t);
        }
        TpeSettings s;
        if (settings.contains("gamma")) s.gamma = settings["gamma"].cast<double>();
        if (settings.contains("gamma_mode")) s.gamma_mode = settings["gamma_mode"].cast<int>();
        if (settings.contains("prior_weight")) s.prior_weight = settings["prior_weight"].cast<double>();
        if (settings.contains("n_ei_candidates")) s.n_ei_candidates = settings["n_ei_candidates"].cast<int>();
        if (settings.contains("multivariate")) s.multivariate = settings["multivariate"].cast<bool>();
        if (settings.contains("consider_magic_clip"))
          s.consider_magic_clip = settings["consider_magic_clip"].cast<bool>();
        if (settings.contains("linear_forgetting"))
          s.linear_forgetting = settings["linear_forgetting"].cast<int>();
        return tpe_sample(td, xs, losses, s, seed);
      },
      py::arg("dims"), py::arg("xs"), py::arg("losses"), py::arg("settings"), py::arg("seed") = 0);

  // ---- experiment status engine (status_engine.hpp) ----
  // trials: [(name, condition_mask, has_metric, min, max, latest, strategy)]
  m.def(
      "summarize_trials",
      [](const std::vector<std::tuple<std::string, uint32_t, bool, std::string, std::string, std::string, int>>& rows,
         int objective_type, std::optional<double> goal) {
        std::vector<TrialFacts> facts;
        facts.reserve(rows.size());
        for (const auto& r : rows) {
          TrialFacts f;
          std::tie(f.name, f.conditions, f.has_metric, f.min, f.max, f.latest, std::ignore) = r;
          f.strategy = static_cast<MetricStrategy>(std::get<6>(r));
          facts.push_back(std::move(f));
        }
        TrialsSummary s;
        {
          py::gil_scoped_release nogil;
          s = summarize_trials(facts, static_cast<ObjectiveType>(objective_type), goal.has_value(),
                               goal.value_or(0.0));
        }
        std::vector<std::vector<int>> buckets(s.buckets.begin(), s.buckets.end());
        return py::make_tuple(buckets, s.best, s.goal_reached);
      },
      py::arg("trials"), py::arg("objective_type"), py::arg("goal") = py::none());
  m.def("objective_value", [](bool has_metric, const std::string& mn, const std::string& mx, const std::string& latest,
                              int strategy) {
    TrialFacts f;
    f.has_metric = has_metric;
    f.min = mn;
    f.max = mx;
    f.latest = latest;
    f.strategy = static_cast<MetricStrategy>(strategy);
    return objective_value(f);
  });
  m.def(
      "decide_condition",
      [](const CountsTuple& c, bool goal_reached, bool suggestion_done, std::optional<int> max_failed,
         std::optional<int> max_trials) {
        return static_cast<int>(decide_condition(counts_from(c), goal_reached, suggestion_done, max_failed.has_value(),
                                                 max_failed.value_or(0), max_trials.has_value(),
                                                 max_trials.value_or(0)));
      },
      py::arg("counts"), py::arg("goal_reached"), py::arg("suggestion_done"), py::arg("max_failed") = py::none(),
      py::arg("max_trials") = py::none());
  m.def(
      "plan_admission",
      [](const CountsTuple& c, int parallel, std::optional<int> max_trials, int n_trials, int es_without_obs) {
        AdmissionPlan p = plan_admission(counts_from(c), parallel, max_trials.has_value(), max_trials.value_or(0),
                                         n_trials, es_without_obs);
        return py::make_tuple(p.delete_count, p.add_count, p.requests);
      },
      py::arg("counts"), py::arg("parallel"), py::arg("max_trials"), py::arg("n_trials"),
      py::arg("early_stopped_without_observation"));
  m.def(
      "classify_exit",
      [](bool early_stopped, int exit_code, bool warm_worker, bool run_early_stopped, bool deadline_exceeded,
         bool trial_killed, int attempt, int backoff_limit) {
        ExitFacts f;
        f.early_stopped = early_stopped;
        f.exit_code = exit_code;
        f.warm_worker = warm_worker;
        f.run_early_stopped = run_early_stopped;
        f.deadline_exceeded = deadline_exceeded;
        f.trial_killed = trial_killed;
        f.attempt = attempt;
        f.backoff_limit = backoff_limit;
        return static_cast<int>(classify_exit(f));
      },
      py::arg("early_stopped"), py::arg("exit_code"), py::arg("warm_worker"), py::arg("run_early_stopped"),
      py::arg("deadline_exceeded"), py::arg("trial_killed"), py::arg("attempt"), py::arg("backoff_limit"));
  m.def(
      "trial_transition",
      [](int job, uint32_t conditions, bool observation_available) {
        return static_cast<int>(trial_transition(job, conditions, observation_available));
      },
      py::arg("job"), py::arg("conditions"), py::arg("observation_available"));
  m.def(
      "plan_restart",
      [](bool succeeded_by_max_trials, int policy, std::optional<int> max_trials, int trials, bool has_running) {
        return static_cast<int>(plan_restart(succeeded_by_max_trials, static_cast<ResumePolicy>(policy),
                                             max_trials.has_value(), max_trials.value_or(0), trials, has_running));
      },
      py::arg("succeeded_by_max_trials"), py::arg("resume_policy"), py::arg("max_trials"), py::arg("trials"),
      py::arg("has_running_trials"));
}
