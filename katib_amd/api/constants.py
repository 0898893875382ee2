"""Constants of the v1beta1 API surface.

Values are the strings users see in Experiment YAML, conditions, labels and
reasons (reference: ``pkg/controller.v1beta1/consts/const.go:25-181``,
``pkg/apis/controller/experiments/v1beta1/constants.go:19-51``,
``pkg/controller.v1beta1/experiment/util/status_util.go:34-42``,
``pkg/controller.v1beta1/trial/trial_controller_status.go:25-40``).
"""

API_VERSION = "kubeflow.org/v1beta1"
KIND_EXPERIMENT = "Experiment"
KIND_TRIAL = "Trial"
KIND_SUGGESTION = "Suggestion"

# --- experiment defaults ------------------------------------------------------------------
DEFAULT_TRIAL_PARALLEL_COUNT = 3
DEFAULT_RESUME_POLICY = "Never"
RESUME_NEVER = "Never"
RESUME_LONG_RUNNING = "LongRunning"
RESUME_FROM_VOLUME = "FromVolume"
RESUME_POLICIES = (RESUME_NEVER, RESUME_LONG_RUNNING, RESUME_FROM_VOLUME)

DEFAULT_JOB_SUCCESS_CONDITION = 'status.conditions.#(type=="Complete")#|#(status=="True")#'
DEFAULT_JOB_FAILURE_CONDITION = 'status.conditions.#(type=="Failed")#|#(status=="True")#'
DEFAULT_KUBEFLOW_JOB_SUCCESS_CONDITION = 'status.conditions.#(type=="Succeeded")#|#(status=="True")#'
DEFAULT_KUBEFLOW_JOB_FAILURE_CONDITION = 'status.conditions.#(type=="Failed")#|#(status=="True")#'
DEFAULT_KUBEFLOW_JOB_PRIMARY_POD_LABELS = {"training.kubeflow.org/job-role": "master"}
KUBEFLOW_JOB_KINDS = ("TFJob", "PyTorchJob", "XGBoostJob", "MXJob", "MPIJob")
JOB_KIND_JOB = "Job"
# native kind: a local process trial that needs no Kubernetes object at all
JOB_KIND_LOCAL = "LocalProcess"

# --- parameter / objective enums ---------------------------------------------------------
PARAMETER_DOUBLE = "double"
PARAMETER_INT = "int"
PARAMETER_DISCRETE = "discrete"
PARAMETER_CATEGORICAL = "categorical"
PARAMETER_TYPES = (PARAMETER_DOUBLE, PARAMETER_INT, PARAMETER_DISCRETE, PARAMETER_CATEGORICAL)

OBJECTIVE_MINIMIZE = "minimize"
OBJECTIVE_MAXIMIZE = "maximize"

STRATEGY_MIN = "min"
STRATEGY_MAX = "max"
STRATEGY_LATEST = "latest"

COMPARISON_EQUAL = "equal"
COMPARISON_LESS = "less"
COMPARISON_GREATER = "greater"

# --- metrics collector --------------------------------------------------------------------
COLLECTOR_STDOUT = "StdOut"
COLLECTOR_FILE = "File"
COLLECTOR_TFEVENT = "TensorFlowEvent"
COLLECTOR_PROMETHEUS = "PrometheusMetric"
COLLECTOR_CUSTOM = "Custom"
COLLECTOR_NONE = "None"
COLLECTOR_KINDS = (COLLECTOR_STDOUT, COLLECTOR_FILE, COLLECTOR_TFEVENT, COLLECTOR_PROMETHEUS,
                   COLLECTOR_CUSTOM, COLLECTOR_NONE)
DEFAULT_FILE_PATH = "/var/log/katib/metrics.log"
DEFAULT_TFEVENT_DIR_PATH = "/var/log/katib/tfevent/"
DEFAULT_PROMETHEUS_PATH = "/metrics"
DEFAULT_PROMETHEUS_PORT = 8080
FS_KIND_DIRECTORY = "Directory"
FS_KIND_FILE = "File"
FORMAT_TEXT = "TEXT"
FORMAT_JSON = "JSON"
# pkg/metricscollector/v1beta1/common/const.go:47
DEFAULT_METRICS_FILTER = r"([\w|-]+)\s*=\s*([+-]?\d*(\.\d+)?([Ee][+-]?\d+)?)"
TIMESTAMP_JSON_KEY = "timestamp"
TRAINING_COMPLETED = "completed"
TRAINING_EARLY_STOPPED = "early-stopped"

UNAVAILABLE_METRIC_VALUE = "unavailable"

# --- labels / names ----------------------------------------------------------------------
LABEL_EXPERIMENT_NAME = "katib.kubeflow.org/experiment"
LABEL_SUGGESTION_NAME = "katib.kubeflow.org/suggestion"
LABEL_TRIAL_NAME = "katib.kubeflow.org/trial"
LABEL_DEPLOYMENT_NAME = "katib.kubeflow.org/deployment"
LABEL_TRIAL_TEMPLATE_CONFIGMAP_NAME = "katib.kubeflow.org/component"
LABEL_TRIAL_TEMPLATE_CONFIGMAP_VALUE = "trial-templates"
LABEL_METRICS_COLLECTOR_INJECTION = "katib.kubeflow.org/metrics-collector-injection"
ANNOTATION_ISTIO_SIDECAR_INJECT = "sidecar.istio.io/inject"

TRIAL_TEMPLATE_PARAM_REPLACE_FORMAT = "${trialParameters.%s}"
TRIAL_TEMPLATE_PARAM_REPLACE_REGEX = r"\$\{trialParameters\..+?\}"
TRIAL_TEMPLATE_META_REPLACE_REGEX = r"\$\{trialSpec\.(.+?)\}"
TRIAL_TEMPLATE_META_PARSE_REGEX = r"(.+)\[(.+)]"
TRIAL_TEMPLATE_META_KEYS = ("Name", "Namespace", "Kind", "APIVersion", "Annotations", "Labels")

SUGGESTION_VOLUME_MOUNT_KEY = "suggestion_trial_dir"
DEFAULT_SUGGESTION_PORT = 6789
DEFAULT_EARLY_STOPPING_PORT = 6788
DEFAULT_DB_MANAGER_PORT = 6789
DEFAULT_GRPC_RETRY_ATTEMPTS = 10
DEFAULT_GRPC_RETRY_PERIOD_S = 3.0
DEFAULT_GRPC_SERVICE = "manager.v1beta1.Suggestion"

# finalizers (experiment_controller_util.go / trial_controller.go)
FINALIZER_UPDATE_PROMETHEUS_METRICS = "update-prometheus-metrics"
FINALIZER_CLEAN_METRICS_IN_DB = "clean-metrics-in-db"

# --- condition types ---------------------------------------------------------------------
EXPERIMENT_CREATED = "Created"
EXPERIMENT_RUNNING = "Running"
EXPERIMENT_RESTARTING = "Restarting"
EXPERIMENT_SUCCEEDED = "Succeeded"
EXPERIMENT_FAILED = "Failed"

TRIAL_CREATED = "Created"
TRIAL_RUNNING = "Running"
TRIAL_SUCCEEDED = "Succeeded"
TRIAL_KILLED = "Killed"
TRIAL_FAILED = "Failed"
TRIAL_METRICS_UNAVAILABLE = "MetricsUnavailable"
TRIAL_EARLY_STOPPED = "EarlyStopped"

SUGGESTION_CREATED = "Created"
SUGGESTION_DEPLOYMENT_READY = "DeploymentReady"
SUGGESTION_RUNNING = "Running"
SUGGESTION_SUCCEEDED = "Succeeded"
SUGGESTION_FAILED = "Failed"

CONDITION_TRUE = "True"
CONDITION_FALSE = "False"
CONDITION_UNKNOWN = "Unknown"

# --- reasons -----------------------------------------------------------------------------
EXPERIMENT_CREATED_REASON = "ExperimentCreated"
EXPERIMENT_RUNNING_REASON = "ExperimentRunning"
EXPERIMENT_RESTARTING_REASON = "ExperimentRestarting"
EXPERIMENT_GOAL_REACHED_REASON = "ExperimentGoalReached"
EXPERIMENT_MAX_TRIALS_REACHED_REASON = "ExperimentMaxTrialsReached"
EXPERIMENT_SUGGESTION_END_REACHED_REASON = "ExperimentSuggestionEndReached"
EXPERIMENT_FAILED_REASON = "ExperimentFailed"

TRIAL_CREATED_REASON = "TrialCreated"
TRIAL_RUNNING_REASON = "TrialRunning"
TRIAL_SUCCEEDED_REASON = "TrialSucceeded"
TRIAL_METRICS_UNAVAILABLE_REASON = "MetricsUnavailable"
TRIAL_FAILED_REASON = "TrialFailed"
TRIAL_KILLED_REASON = "TrialKilled"
TRIAL_EARLY_STOPPED_REASON = "TrialEarlyStopped"

JOB_CREATED_REASON = "JobCreated"
JOB_DELETED_REASON = "JobDeleted"
JOB_SUCCEEDED_REASON = "JobSucceeded"
JOB_METRICS_UNAVAILABLE_REASON = "MetricsUnavailable"
JOB_FAILED_REASON = "JobFailed"
JOB_RUNNING_REASON = "JobRunning"

SUGGESTION_CREATED_REASON = "SuggestionCreated"
SUGGESTION_DEPLOYMENT_READY_REASON = "DeploymentReady"
SUGGESTION_DEPLOYMENT_NOT_READY_REASON = "DeploymentNotReady"
SUGGESTION_RUNNING_REASON = "SuggestionRunning"
SUGGESTION_SUCCEEDED_REASON = "SuggestionSucceeded"
SUGGESTION_FAILED_REASON = "SuggestionFailed"
SUGGESTION_RESTARTING_REASON = "Suggestion is restarting"

RECONCILE_ERROR_REASON = "ReconcileError"

# --- algorithm registry (katib-config.yaml:1-61 -> in-process implementations) ----------
SUGGESTION_ALGORITHMS = (
    "random", "tpe", "grid", "hyperband", "bayesianoptimization", "cmaes", "sobol",
    "multivariate-tpe", "enas", "darts", "pbt",
)
EARLY_STOPPING_ALGORITHMS = ("medianstop",)
