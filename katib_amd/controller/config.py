"""KatibConfig for the node-local scheduler.

Reads the reference ``katib-config.yaml`` layout (``pkg/apis/config/v1beta1/types.go:27-126``,
``manifests/v1beta1/installs/katib-standalone/katib-config.yaml``): ``init.controller``
and ``runtime.{suggestions,earlyStoppings,metricsCollectors}``. For a suggestion
entry the ``image`` is replaced by an in-process ``service`` name (if an image
such as ``.../suggestion-hyperopt:...`` is given the service is inferred from it).
The ``amd`` section configures the MI355X node: devices, slots per device, warm
worker pool, state directory.
"""

from __future__ import annotations

import copy
import os
import re
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import yaml

from ..algorithms.registry import DEFAULT_EARLY_STOPPINGS, DEFAULT_SUGGESTIONS, SERVICES


def detect_gpus() -> int:
    """Count visible GPUs without creating a HIP context in the scheduler process."""
    env = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("ROCR_VISIBLE_DEVICES") \
        or os.environ.get("CUDA_VISIBLE_DEVICES")
    if env is not None and env != "":
        return len([x for x in env.split(",") if x.strip() != ""])
    try:
        import torch

        return int(torch.cuda.device_count())  # does not initialise the device on this ROCm build
    except Exception:
        return 0


@dataclass
class AmdConfig:
    num_devices: Optional[int] = None  # None: auto-detect
    slots_per_device: int = 1
    cpu_slots: int = 8  # concurrent CPU-only trials
    state_dir: str = "/tmp/katib-amd"
    warm_workers: bool = True
    worker_python: str = ""
    fault_quarantine_threshold: int = 3
    poll_interval_ms: int = 20
    map_collector_paths: bool = True
    # a Job / LocalProcess trial with amd.com/gpu: N > 1 runs as N rank processes ("ranks", one
    # process per GPU with the torchrun env) or as one process seeing all N GPUs ("single")
    multi_gpu_launch: str = "ranks"
    # cold Python trial processes (`python3 -m module ...` Job commands) forked from a fork server
    # that has already imported torch (controller/zygote.py); KATIB_AMD_ZYGOTE=0 turns it off
    zygote: bool = True


@dataclass
class KatibConfig:
    suggestions: Dict[str, str] = field(default_factory=lambda: dict(DEFAULT_SUGGESTIONS))
    suggestion_settings: Dict[str, Dict] = field(default_factory=dict)
    early_stoppings: Dict[str, str] = field(default_factory=lambda: dict(DEFAULT_EARLY_STOPPINGS))
    metrics_collectors: Dict[str, Dict] = field(default_factory=lambda: {
        "StdOut": {}, "File": {}, "TensorFlowEvent": {}, "PrometheusMetric": {}})
    trial_resources: List[str] = field(default_factory=lambda: ["Job.v1.batch", "LocalProcess.v1.katib-amd.io",
                                                                  "Function.v1.katib-amd.io", "PyTorchJob.v1.kubeflow.org",
                                                                  "TFJob.v1.kubeflow.org", "XGBoostJob.v1.kubeflow.org",
                                                                  "MXJob.v1.kubeflow.org", "MPIJob.v1.kubeflow.org"])
    metrics_addr: str = ":8080"
    healthz_addr: str = ":18080"
    experiment_suggestion_name: str = "default"
    amd: AmdConfig = field(default_factory=AmdConfig)
    raw: Dict = field(default_factory=dict)  # the defaulted katib-config.yaml document

    @staticmethod
    def _service_from_image(image: str) -> Optional[str]:
        m = re.search(r"suggestion-([a-z]+)", image or "")
        if m and m.group(1) in SERVICES:
            return m.group(1)
        return None

    @classmethod
    def from_dict(cls, d: Dict) -> "KatibConfig":
        cfg = cls()
        if not d:
            return cfg
        from ..api import katibconfig as KC

        cfg.raw = KC.set_defaults(copy.deepcopy(d))  # reference defaulting (defaults.go)
        init = (d.get("init") or {}).get("controller") or {}
        if init.get("trialResources"):
            KC.trial_resources_to_gvks(init["trialResources"])
            cfg.trial_resources = list(init["trialResources"])
        cfg.metrics_addr = init.get("metricsAddr", cfg.metrics_addr)
        cfg.healthz_addr = init.get("healthzAddr", cfg.healthz_addr)
        cfg.experiment_suggestion_name = init.get("experimentSuggestionName", cfg.experiment_suggestion_name)
        rt = d.get("runtime") or {}
        if rt.get("suggestions") is not None:
            cfg.suggestions = {}
            for s in rt["suggestions"]:
                svc = s.get("service") or cls._service_from_image(s.get("image", "")) \
                    or DEFAULT_SUGGESTIONS.get(s["algorithmName"])
                if svc is None:
                    raise ValueError("cannot map algorithm %s (image %r) to an in-process service"
                                     % (s["algorithmName"], s.get("image")))
                cfg.suggestions[s["algorithmName"]] = svc
                cfg.suggestion_settings[s["algorithmName"]] = s
        if rt.get("earlyStoppings") is not None:
            cfg.early_stoppings = {e["algorithmName"]: "medianstop" for e in rt["earlyStoppings"]}
        if rt.get("metricsCollectors") is not None:
            cfg.metrics_collectors = {m["kind"]: m for m in rt["metricsCollectors"]}
        amd = d.get("amd") or {}
        for k, v in amd.items():
            if hasattr(cfg.amd, k):
                setattr(cfg.amd, k, v)
        return cfg

    @classmethod
    def load(cls, path: str) -> "KatibConfig":
        with open(path) as f:
            return cls.from_dict(yaml.safe_load(f) or {})

    def devices(self) -> int:
        return self.amd.num_devices if self.amd.num_devices is not None else detect_gpus()
