// Experiment status engine: the decision core of the katib-controller reconcile
// loop, in C++ like the reference's Go controller.
//
//   objective_value    getObjectiveMetricValue      (experiment/util/status_util.go:151-183)
//   summarize_trials   updateTrialsSummary          (status_util.go:57-148): bucket
//                      every trial (Killed > Failed > Succeeded > EarlyStopped > Running >
//                      MetricsUnavailable > Pending), pick the optimal trial by the
//                      objective's metric strategy (a non-numeric value makes the latest
//                      trial "best"), evaluate the goal (<= minimize, >= maximize).
//   decide_condition   UpdateExperimentStatusCondition (status_util.go:187-235): goal ->
//                      maxFailedTrialCount (failed + metricsUnavailable) -> maxTrialCount
//                      (completed incl. metricsUnavailable) -> suggestion end -> Running.
//   plan_admission     ReconcileTrials + ReconcileSuggestions demand
//                      (experiment_controller.go:274-330, 445-493): delete the newest
//                      trials above parallelTrialCount, or add
//                      min(maxTrialCount - completed, parallel) - active trials, and
//                      request len(trials) + add - (early-stopped trials without an
//                      observation) assignments from the suggestion service.
//   plan_restart       Reconcile's restart branch (experiment_controller.go:187-212 and
//                      IsCompletedExperimentRestartable, status_util.go:240-246).
//
// Pure functions over plain structs: the Python manager (katib_amd/controller/manager.py)
// owns the objects and applies the decisions.
#pragma once
#include <array>
#include <cstdint>
#include <string>
#include <vector>

namespace katib {

enum class TrialBucket : int {
  Killed = 0,
  Failed,
  Succeeded,
  EarlyStopped,
  Running,
  MetricsUnavailable,
  Pending,
};
constexpr int kNumBuckets = 7;

enum class ObjectiveType : int { Unknown = 0, Minimize = 1, Maximize = 2 };
enum class MetricStrategy : int { None = 0, Min = 1, Max = 2, Latest = 3 };

// Condition bits of a Trial whose status is "True" (trial_types.go:107-126).
enum TrialCondBit : uint32_t {
  kCondCreated = 1u << 0,
  kCondRunning = 1u << 1,
  kCondSucceeded = 1u << 2,
  kCondKilled = 1u << 3,
  kCondFailed = 1u << 4,
  kCondMetricsUnavailable = 1u << 5,
  kCondEarlyStopped = 1u << 6,
};

struct TrialFacts {
  std::string name;
  uint32_t conditions = 0;  // TrialCondBit mask
  bool has_metric = false;  // observation carries the objective metric
  std::string min, max, latest;
  MetricStrategy strategy = MetricStrategy::None;  // the trial objective's strategy for its metric
};

struct TrialsSummary {
  std::array<std::vector<int>, kNumBuckets> buckets;  // trial indices per TrialBucket, input order
  int best = -1;                                      // index of the optimal trial, -1 = none
  bool goal_reached = false;
};

struct StatusCounts {
  int pending = 0, running = 0, succeeded = 0, failed = 0, killed = 0, early_stopped = 0, metrics_unavailable = 0;
};

enum class ConditionOutcome : int {
  Running = 0,
  GoalReached,
  MaxFailedReached,
  MaxTrialsReached,
  SuggestionEndReached,
};

struct AdmissionPlan {
  int delete_count = 0;  // newest trials to delete (active > parallel)
  int add_count = 0;     // trials to create
  int requests = 0;      // Suggestion.spec.requests when add_count > 0
};

enum class ResumePolicy : int { Never = 0, LongRunning, FromVolume };

enum class RestartAction : int {
  None = 0,     // completed and staying so (no running trials left)
  Restart,      // flip to Restarting (and, for FromVolume, restart the suggestion)
  KeepGoing,    // completed but trials still running: reconcile them
};

// ---- trial state machine (trial controller) ----
// What a finished primary process means for its trial (manager.py _on_runtime_event, the
// local analogue of the Job controller + backoffLimit feeding trial_controller.go:263-310).
enum class ExitOutcome : int {
  Succeeded = 0,     // job status Succeeded (exit 0, or early-stopped by the collector)
  DeadlineExceeded,  // job Failed, reason DeadlineExceeded (activeDeadlineSeconds)
  Killed,            // the trial was killed: keep the Killed condition, job phase Failed
  Retry,             // back to Pending (attempt <= backoffLimit)
  Failed,            // job Failed, reason Error
};
struct ExitFacts {
  bool early_stopped = false;       // the collector's stop rules fired
  int exit_code = 0;
  bool warm_worker = false;         // ran inside a warm worker (exit code 3 = stopped by signal)
  bool run_early_stopped = false;   // an early stop was requested for this run
  bool deadline_exceeded = false;
  bool trial_killed = false;
  int attempt = 0;
  int backoff_limit = 0;
};
ExitOutcome classify_exit(const ExitFacts& f);

// UpdateTrialStatusCondition (trial_controller_util.go:42-122): the condition change for a
// trial whose job reached `job` (0 running, 1 succeeded, 2 failed).
enum class TrialTransition : int {
  None = 0,
  MarkFailed,              // Failed + completion time + event + counter
  MarkSucceeded,           // Succeeded (observation available)
  CompleteObserved,        // observation available but already EarlyStopped: completion time only
  MarkMetricsUnavailable,  // succeeded job without the objective metric
  CompleteEarlyStopped,    // early-stopped trial without an observation: completion time only
};
TrialTransition trial_transition(int job, uint32_t conditions, bool observation_available);

TrialBucket classify(uint32_t conditions);
std::string objective_value(const TrialFacts& t);
TrialsSummary summarize_trials(const std::vector<TrialFacts>& trials, ObjectiveType type, bool has_goal,
                               double goal);
StatusCounts counts_of(const TrialsSummary& s);
ConditionOutcome decide_condition(const StatusCounts& c, bool goal_reached, bool suggestion_done,
                                  bool has_max_failed, int max_failed, bool has_max_trials, int max_trials);
AdmissionPlan plan_admission(const StatusCounts& c, int parallel, bool has_max_trials, int max_trials, int n_trials,
                             int early_stopped_without_observation);
RestartAction plan_restart(bool succeeded_by_max_trials, ResumePolicy policy, bool has_max_trials, int max_trials,
                           int trials, bool has_running_trials);

}  // namespace katib
