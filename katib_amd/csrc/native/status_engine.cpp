// Experiment status engine - see status_engine.hpp for the reference mapping.
#include "status_engine.hpp"

#include <algorithm>

#include "metrics_parser.hpp"  // go_parse_float (strconv.ParseFloat semantics)

namespace katib {

namespace {

const char* const kUnavailable = "unavailable";  // consts.UnavailableMetricValue (const.go)

}  // namespace

TrialBucket classify(uint32_t c) {
  // updateTrialsSummary's if/else chain order (status_util.go:71-92)
  if (c & kCondKilled) return TrialBucket::Killed;
  if (c & kCondFailed) return TrialBucket::Failed;
  if (c & kCondSucceeded) return TrialBucket::Succeeded;
  if (c & kCondEarlyStopped) return TrialBucket::EarlyStopped;
  if (c & kCondRunning) return TrialBucket::Running;
  if (c & kCondMetricsUnavailable) return TrialBucket::MetricsUnavailable;
  return TrialBucket::Pending;
}

std::string objective_value(const TrialFacts& t) {
  if (!t.has_metric) return kUnavailable;
  switch (t.strategy) {
    case MetricStrategy::Min:
      return t.min == kUnavailable ? t.latest : t.min;
    case MetricStrategy::Max:
      return t.max == kUnavailable ? t.latest : t.max;
    case MetricStrategy::Latest:
      return t.latest;
    default:
      return kUnavailable;
  }
}

TrialsSummary summarize_trials(const std::vector<TrialFacts>& trials, ObjectiveType type, bool has_goal,
                               double goal) {
  TrialsSummary s;
  double best_val = 0.0;  // bestTrialValue starts at 0 (status_util.go)
  for (int i = 0; i < static_cast<int>(trials.size()); ++i) {
    const TrialFacts& t = trials[i];
    s.buckets[static_cast<int>(classify(t.conditions))].push_back(i);
    const std::string v = objective_value(t);
    if (v == kUnavailable) continue;
    double x;
    if (!go_parse_float(v, x)) {
      s.best = i;  // non-numeric metric: the latest trial wins (status_util.go:99-104)
      continue;
    }
    // Reference semantics, kept exactly: only the FIRST trial with any metric initialises
    // the best value; when a non-numeric metric set best first, numeric trials compare
    // against the zero-initialised value (status_util.go:99-110).
    if (s.best == -1) {
      best_val = x;
      s.best = i;
    }
    if (type == ObjectiveType::Minimize) {
      if (x < best_val) {
        best_val = x;
        s.best = i;
      }
      if (has_goal && best_val <= goal) s.goal_reached = true;
    } else if (type == ObjectiveType::Maximize) {
      if (x > best_val) {
        best_val = x;
        s.best = i;
      }
      if (has_goal && best_val >= goal) s.goal_reached = true;
    }
  }
  return s;
}

StatusCounts counts_of(const TrialsSummary& s) {
  StatusCounts c;
  c.killed = static_cast<int>(s.buckets[static_cast<int>(TrialBucket::Killed)].size());
  c.failed = static_cast<int>(s.buckets[static_cast<int>(TrialBucket::Failed)].size());
  c.succeeded = static_cast<int>(s.buckets[static_cast<int>(TrialBucket::Succeeded)].size());
  c.early_stopped = static_cast<int>(s.buckets[static_cast<int>(TrialBucket::EarlyStopped)].size());
  c.running = static_cast<int>(s.buckets[static_cast<int>(TrialBucket::Running)].size());
  c.metrics_unavailable = static_cast<int>(s.buckets[static_cast<int>(TrialBucket::MetricsUnavailable)].size());
  c.pending = static_cast<int>(s.buckets[static_cast<int>(TrialBucket::Pending)].size());
  return c;
}

ConditionOutcome decide_condition(const StatusCounts& c, bool goal_reached, bool suggestion_done,
                                  bool has_max_failed, int max_failed, bool has_max_trials, int max_trials) {
  // status_util.go:189-191: MetricsUnavailable counts as completed AND as failed here.
  const int completed = c.succeeded + c.failed + c.killed + c.early_stopped + c.metrics_unavailable;
  const int failed = c.failed + c.metrics_unavailable;
  const int active = c.pending + c.running;
  if (goal_reached) return ConditionOutcome::GoalReached;
  if (has_max_failed && failed != 0 && failed >= max_failed) return ConditionOutcome::MaxFailedReached;
  if (has_max_trials && completed >= max_trials) return ConditionOutcome::MaxTrialsReached;
  if (suggestion_done && active == 0) return ConditionOutcome::SuggestionEndReached;
  return ConditionOutcome::Running;
}

AdmissionPlan plan_admission(const StatusCounts& c, int parallel, bool has_max_trials, int max_trials, int n_trials,
                             int early_stopped_without_observation) {
  AdmissionPlan p;
  const int active = c.pending + c.running;
  // experiment_controller.go:280: MetricsUnavailable is NOT completed in this count
  const int completed = c.succeeded + c.failed + c.killed + c.early_stopped;
  if (active > parallel) {
    p.delete_count = active - parallel;
  } else if (active < parallel) {
    const int required = has_max_trials ? std::min(max_trials - completed, parallel) : parallel;
    p.add_count = std::max(required - active, 0);
  }
  if (p.add_count > 0) p.requests = n_trials + p.add_count - early_stopped_without_observation;
  return p;
}

ExitOutcome classify_exit(const ExitFacts& f) {
  if (f.early_stopped || f.exit_code == 0 || (f.warm_worker && f.exit_code == 3 && f.run_early_stopped))
    return ExitOutcome::Succeeded;
  if (f.deadline_exceeded) return ExitOutcome::DeadlineExceeded;
  if (f.trial_killed) return ExitOutcome::Killed;
  if (f.attempt <= f.backoff_limit) return ExitOutcome::Retry;
  return ExitOutcome::Failed;
}

TrialTransition trial_transition(int job, uint32_t c, bool observation_available) {
  const bool failed = c & kCondFailed, succeeded = c & kCondSucceeded, early = c & kCondEarlyStopped,
             mu = c & kCondMetricsUnavailable;
  if (job == 2) return (!failed && !early) ? TrialTransition::MarkFailed : TrialTransition::None;
  if (job != 1) return TrialTransition::None;
  // the reference's if / else-if chain, with the local early-stop handling
  if (observation_available && !succeeded)
    return early ? TrialTransition::CompleteObserved : TrialTransition::MarkSucceeded;
  if (!mu && !early) return TrialTransition::MarkMetricsUnavailable;
  if (early) return TrialTransition::CompleteEarlyStopped;
  return TrialTransition::None;
}

RestartAction plan_restart(bool succeeded_by_max_trials, ResumePolicy policy, bool has_max_trials, int max_trials,
                           int trials, bool has_running_trials) {
  const bool restartable =
      succeeded_by_max_trials && (policy == ResumePolicy::LongRunning || policy == ResumePolicy::FromVolume);
  if (restartable && ((has_max_trials && max_trials > trials) || (!has_max_trials && trials != 0)))
    return RestartAction::Restart;
  return has_running_trials ? RestartAction::KeepGoing : RestartAction::None;
}

}  // namespace katib
