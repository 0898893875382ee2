"""``KatibClient`` - the Katib Python SDK surface on top of the node-local scheduler
(reference ``sdk/python/v1beta1/kubeflow/katib/api/katib_client.py:30-1280``).

Same method names, arguments and return types (v1beta1 models); instead of the
Kubernetes API server the client talks to an in-process
:class:`katib_amd.controller.manager.Manager` running its event loop in a
background thread (or a manager passed in). ``get_trial_metrics`` reads the
native observation store directly, or a remote DBManager over gRPC when a
``db_manager_address`` other than the default is given.

``tune()`` keeps the reference semantics - the objective's source is extracted
with ``inspect.getsource``, ``katib.search.*`` values become
``${trialParameters.x}`` placeholders, everything else is passed verbatim - but
the function runs in a warm per-GPU worker process (kind ``Function``) instead
of a ``bash -c`` heredoc inside a Kubernetes Job. ``resources_per_trial={"gpu": n}``
maps to ``amd.com/gpu``.
"""

from __future__ import annotations

import inspect
import textwrap
import time
from typing import Any, Callable, Dict, List, Optional, Union

from ..api import constants as C
from ..api import models
from ..api.conditions import ExperimentConditions as EC
from ..api.conditions import has_condition
from . import constants

_SHARED = {"manager": None}


def _shared_manager():
    from ..controller.manager import Manager

    if _SHARED["manager"] is None:
        m = Manager()
        m.start()
        _SHARED["manager"] = m
    return _SHARED["manager"]


class KatibClient:
    def __init__(self, namespace: str = "default", manager=None, config_file: Optional[str] = None,
                 host: Optional[str] = None, **_):
        """``manager``: an in-process scheduler; ``host``: URL of a ``katib-amd serve`` daemon
        (also taken from ``$KATIB_AMD_HOST``); neither: a shared in-process scheduler."""
        import os

        self.namespace = namespace
        host = host or os.environ.get("KATIB_AMD_HOST")
        if manager is None and host:
            from .remote import RemoteManager

            manager = RemoteManager(host, namespace)
        if manager is None:
            manager = _shared_manager()
            if config_file:
                from ..controller.config import KatibConfig

                manager.config = KatibConfig.load(config_file)
        self.manager = manager

    # ------------------------------------------------------------------ experiments
    def create_experiment(self, experiment: models.V1beta1Experiment, namespace: Optional[str] = None):
        namespace = namespace or (experiment.metadata.namespace if experiment.metadata else None) or self.namespace
        try:
            out = self.manager.create_experiment(experiment, namespace)
        except Exception as e:
            raise RuntimeError(f"Failed to create Katib Experiment: {namespace}/"
                               f"{experiment.metadata.name if experiment.metadata else ''}: {e}") from e
        print(f"Experiment {namespace}/{out.metadata.name} has been created")
        return out

    def tune(self, name: str, objective: Callable, parameters: Dict[str, Any],
             base_image: str = constants.BASE_IMAGE_PYTORCH, namespace: Optional[str] = None,
             env_per_trial: Optional[Union[Dict[str, str], List]] = None, algorithm_name: str = "random",
             algorithm_settings: Union[dict, List[models.V1beta1AlgorithmSetting], None] = None,
             objective_metric_name: str = None, additional_metric_names: List[str] = [],
             objective_type: str = "maximize", objective_goal: float = None, max_trial_count: int = None,
             parallel_trial_count: int = None, max_failed_trial_count: int = None,
             resources_per_trial: Union[dict, None] = None, retain_trials: bool = False,
             packages_to_install: List[str] = None, pip_index_url: str = "https://pypi.org/simple"):
        namespace = namespace or self.namespace
        exp = models.V1beta1Experiment(
            api_version=f"{constants.KUBEFLOW_GROUP}/{constants.KATIB_VERSION}", kind=constants.EXPERIMENT_KIND,
            metadata=models.V1ObjectMeta(name=name, namespace=namespace), spec=models.V1beta1ExperimentSpec())
        exp.spec.objective = models.V1beta1ObjectiveSpec(type=objective_type,
                                                         objective_metric_name=objective_metric_name,
                                                         additional_metric_names=list(additional_metric_names))
        if objective_goal is not None:
            exp.spec.objective.goal = objective_goal
        if isinstance(algorithm_settings, dict):
            algorithm_settings = [models.V1beta1AlgorithmSetting(name=str(k), value=str(v))
                                  for k, v in algorithm_settings.items()]
        exp.spec.algorithm = models.V1beta1AlgorithmSpec(algorithm_name=algorithm_name,
                                                         algorithm_settings=algorithm_settings)
        if max_trial_count is not None:
            exp.spec.max_trial_count = max_trial_count
        if parallel_trial_count is not None:
            exp.spec.parallel_trial_count = parallel_trial_count
        if max_failed_trial_count is not None:
            exp.spec.max_failed_trial_count = max_failed_trial_count
        validate_objective_function(objective)
        code = textwrap.dedent(inspect.getsource(objective))
        input_params, exp_params, trial_params = {}, [], []
        for p_name, p_value in parameters.items():
            if isinstance(p_value, models.V1beta1ParameterSpec):
                input_params[p_name] = "${trialParameters.%s}" % p_name
                p_value.name = p_name
                exp_params.append(p_value)
                trial_params.append(models.V1beta1TrialParameterSpec(name=p_name, reference=p_name))
            else:
                input_params[p_name] = p_value
        gpus = 0
        if isinstance(resources_per_trial, dict):
            for k in ("gpu", "amd.com/gpu", "nvidia.com/gpu"):
                if k in resources_per_trial:
                    gpus = int(resources_per_trial[k])
        env = []
        if isinstance(env_per_trial, dict):
            env = [{"name": str(k), "value": str(v)} for k, v in env_per_trial.items()]
        elif env_per_trial:
            for x in env_per_trial:
                if isinstance(x, dict):
                    env.append(x)
                elif hasattr(x, "name") and hasattr(x, "value"):
                    env.append({"name": x.name, "value": x.value})
                else:
                    raise ValueError(f"Incorrect value for env_per_trial: {env_per_trial}")
        trial_spec = {
            "apiVersion": "katib-amd.io/v1", "kind": "Function",
            "metadata": {"annotations": {C.ANNOTATION_ISTIO_SIDECAR_INJECT: "false"}},
            "spec": {"source": code, "entry": objective.__name__, "params": input_params, "gpus": gpus,
                     "env": env, "packages": list(packages_to_install or []), "baseImage": base_image},
        }
        exp.spec.parameters = exp_params
        exp.spec.trial_template = models.V1beta1TrialTemplate(
            primary_container_name=constants.DEFAULT_PRIMARY_CONTAINER_NAME, retain=retain_trials,
            trial_parameters=trial_params, trial_spec=trial_spec,
            success_condition=C.DEFAULT_JOB_SUCCESS_CONDITION, failure_condition=C.DEFAULT_JOB_FAILURE_CONDITION)
        return self.create_experiment(exp, namespace)

    def get_experiment(self, name: str, namespace: Optional[str] = None, timeout: int = constants.DEFAULT_TIMEOUT):
        namespace = namespace or self.namespace
        try:
            return self.manager.get_experiment(name, namespace)
        except KeyError as e:
            raise RuntimeError(f"Failed to get Katib Experiment: {namespace}/{name}") from e

    def list_experiments(self, namespace: Optional[str] = None, timeout: int = constants.DEFAULT_TIMEOUT):
        return self.manager.list_experiments(namespace or self.namespace)

    def get_experiment_conditions(self, name: str, namespace: Optional[str] = None, experiment=None,
                                  timeout: int = constants.DEFAULT_TIMEOUT):
        if experiment is None:
            experiment = self.get_experiment(name, namespace, timeout)
        if experiment.status and experiment.status.conditions:
            return experiment.status.conditions
        return []

    def _is(self, cond, name, namespace, experiment):
        return has_condition(experiment or self.get_experiment(name, namespace), cond)

    def is_experiment_created(self, name, namespace=None, experiment=None, timeout=constants.DEFAULT_TIMEOUT):
        return self._is(C.EXPERIMENT_CREATED, name, namespace, experiment)

    def is_experiment_running(self, name, namespace=None, experiment=None, timeout=constants.DEFAULT_TIMEOUT):
        return self._is(C.EXPERIMENT_RUNNING, name, namespace, experiment)

    def is_experiment_restarting(self, name, namespace=None, experiment=None, timeout=constants.DEFAULT_TIMEOUT):
        return self._is(C.EXPERIMENT_RESTARTING, name, namespace, experiment)

    def is_experiment_succeeded(self, name, namespace=None, experiment=None, timeout=constants.DEFAULT_TIMEOUT):
        return self._is(C.EXPERIMENT_SUCCEEDED, name, namespace, experiment)

    def is_experiment_failed(self, name, namespace=None, experiment=None, timeout=constants.DEFAULT_TIMEOUT):
        return self._is(C.EXPERIMENT_FAILED, name, namespace, experiment)

    def wait_for_experiment_condition(self, name: str, namespace: Optional[str] = None,
                                      expected_condition: str = constants.EXPERIMENT_CONDITION_SUCCEEDED,
                                      timeout: int = 600, polling_interval: float = 15,
                                      apiserver_timeout: int = constants.DEFAULT_TIMEOUT):
        namespace = namespace or self.namespace
        deadline = time.time() + timeout
        poll = min(polling_interval, 0.05)  # the scheduler is in-process: poll fast
        while time.time() < deadline:
            e = self.get_experiment(name, namespace)
            if expected_condition == constants.EXPERIMENT_CONDITION_FAILED and EC.is_failed(e):
                return e
            if EC.is_failed(e):
                raise RuntimeError(f"Experiment: {namespace}/{name} is Failed. "
                                   f"Experiment conditions: {e.status.conditions}")
            if has_condition(e, expected_condition):
                return e
            time.sleep(poll)
        raise TimeoutError(f"Timeout waiting for Experiment: {namespace}/{name} to reach {expected_condition} state")

    def edit_experiment_budget(self, name: str, namespace: Optional[str] = None, max_trial_count: int = None,
                               parallel_trial_count: int = None, max_failed_trial_count: int = None,
                               timeout: int = constants.DEFAULT_TIMEOUT):
        namespace = namespace or self.namespace
        if max_trial_count is None and parallel_trial_count is None and max_failed_trial_count is None:
            raise ValueError("Invalid input arguments. You have to set max_trial_count, parallel_trial_count, "
                             "or max_failed_trial_count to modify Experiment Trial budget.")
        e = self.get_experiment(name, namespace)
        if max_trial_count is not None:
            e.spec.max_trial_count = max_trial_count
        if parallel_trial_count is not None:
            e.spec.parallel_trial_count = parallel_trial_count
        if max_failed_trial_count is not None:
            e.spec.max_failed_trial_count = max_failed_trial_count
        try:
            self.manager.update_experiment(e)
        except Exception as ex:
            raise RuntimeError(f"Failed to edit Katib Experiment: {namespace}/{name}: {ex}") from ex
        print(f"Experiment {namespace}/{name} has been updated")

    def delete_experiment(self, name: str, namespace: Optional[str] = None, delete_options=None):
        namespace = namespace or self.namespace
        try:
            self.manager.delete_experiment(name, namespace)
        except KeyError as e:
            raise RuntimeError(f"Failed to delete Katib Experiment: {namespace}/{name}") from e
        print(f"Experiment {namespace}/{name} has been deleted")

    # ------------------------------------------------------------------ suggestions / trials
    def get_suggestion(self, name: str, namespace: Optional[str] = None, timeout: int = constants.DEFAULT_TIMEOUT):
        try:
            return self.manager.get_suggestion(name, namespace or self.namespace)
        except KeyError as e:
            raise RuntimeError(f"Failed to get Katib Suggestion: {name}") from e

    def list_suggestions(self, namespace: Optional[str] = None, timeout: int = constants.DEFAULT_TIMEOUT):
        return self.manager.list_suggestions(namespace or self.namespace)

    def get_trial(self, name: str, namespace: Optional[str] = None, timeout: int = constants.DEFAULT_TIMEOUT):
        try:
            return self.manager.get_trial(name, namespace or self.namespace)
        except KeyError as e:
            raise RuntimeError(f"Failed to get Katib Trial: {name}") from e

    def list_trials(self, experiment_name: str = None, namespace: Optional[str] = None,
                    timeout: int = constants.DEFAULT_TIMEOUT):
        return self.manager.list_trials(experiment_name, namespace or self.namespace)

    def get_success_trial_details(self, experiment_name: str = None, namespace: Optional[str] = None,
                                  timeout: int = constants.DEFAULT_TIMEOUT):
        out = []
        for t in self.list_trials(experiment_name, namespace):
            if t.status and t.status.conditions and has_condition(t, constants.TRIAL_CONDITION_SUCCEEDED):
                out.append({"name": t.metadata.name, "parameter_assignments": t.spec.parameter_assignments,
                            "metrics": t.status.observation.metrics})
        return out

    def get_optimal_hyperparameters(self, name: str, namespace: Optional[str] = None,
                                    timeout: int = constants.DEFAULT_TIMEOUT):
        e = self.get_experiment(name, namespace)
        ot = e.status.current_optimal_trial if e.status else None
        if ot is not None and ot.observation is not None and ot.observation.metrics:
            return ot
        return None

    def get_trial_metrics(self, name: str, namespace: Optional[str] = None,
                          db_manager_address: str = constants.DEFAULT_DB_MANAGER_ADDRESS,
                          timeout: str = constants.DEFAULT_TIMEOUT):
        from ..rpc import api_pb2 as api

        if db_manager_address and db_manager_address != constants.DEFAULT_DB_MANAGER_ADDRESS:
            import grpc

            from ..rpc.client import DBManagerStub

            with grpc.insecure_channel(db_manager_address) as ch:
                rep = DBManagerStub(ch).GetObservationLog(api.GetObservationLogRequest(trial_name=name),
                                                          timeout=timeout)
            return list(rep.observation_log.metric_logs)
        return [api.MetricLog(time_stamp=ts, metric=api.Metric(name=n, value=v))
                for ts, n, v in self.manager.get_observation_log(name)]


def validate_objective_function(objective: Callable):
    """utils/utils.py:76-93"""
    if not callable(objective):
        raise ValueError(f"Objective function must be callable, got function type: {type(objective)}")
    sig = inspect.signature(objective)
    if len(sig.parameters) != 1:
        raise ValueError(f"Objective function must have only one dict argument, got {sig}")
