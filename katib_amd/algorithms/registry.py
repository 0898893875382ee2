"""Algorithm-name -> in-process service registry.

Replaces ``runtime.suggestions[]`` / ``runtime.earlyStoppings[]`` of
``katib-config.yaml`` (reference ``manifests/v1beta1/installs/katib-standalone/katib-config.yaml:1-61``):
an entry names an in-process *service* instead of a container image. The default
mapping is the reference's (random/tpe -> hyperopt, grid/multivariate-tpe ->
optuna, cmaes/sobol -> goptuna, bayesianoptimization -> skopt, ...); any name can
be re-pointed to an alternative service (e.g. ``tpe: optuna``) in the
:class:`katib_amd.controller.config.KatibConfig`.
"""

from __future__ import annotations

from typing import Dict

from .hpo import GoptunaService, HyperoptService, OptunaService, SkoptService
from .hyperband import HyperbandService
from .nas import DartsService, EnasService
from .pbt import PbtService

SERVICES = {
    "hyperopt": HyperoptService,
    "optuna": OptunaService,
    "goptuna": GoptunaService,
    "skopt": SkoptService,
    "hyperband": HyperbandService,
    "pbt": PbtService,
    "enas": EnasService,
    "darts": DartsService,
}

DEFAULT_SUGGESTIONS: Dict[str, str] = {
    "random": "hyperopt",
    "tpe": "hyperopt",
    "grid": "optuna",
    "hyperband": "hyperband",
    "bayesianoptimization": "skopt",
    "cmaes": "goptuna",
    "sobol": "goptuna",
    "multivariate-tpe": "optuna",
    "enas": "enas",
    "darts": "darts",
    "pbt": "pbt",
}

DEFAULT_EARLY_STOPPINGS: Dict[str, str] = {"medianstop": "medianstop"}


def create_service(algorithm_name: str, mapping: Dict[str, str] = None, **kwargs):
    mapping = mapping or DEFAULT_SUGGESTIONS
    if algorithm_name not in mapping:
        raise KeyError(f"unable to get Suggestion config data for algorithm {algorithm_name}")
    svc = mapping[algorithm_name]
    cls = SERVICES[svc]
    accepted = {}
    if cls is PbtService and "data_root" in kwargs:
        accepted["data_root"] = kwargs["data_root"]
    if cls is EnasService and "cache_dir" in kwargs:
        accepted["cache_dir"] = kwargs["cache_dir"]
    return cls(**accepted)


def create_early_stopping(algorithm_name: str, mapping: Dict[str, str] = None, **kwargs):
    from ..earlystopping.medianstop import MedianStopService

    mapping = mapping or DEFAULT_EARLY_STOPPINGS
    if algorithm_name not in mapping:
        raise KeyError(f"unable to get EarlyStopping config data for algorithm {algorithm_name}")
    return MedianStopService(**kwargs)
