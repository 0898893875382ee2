"""Node installs: the analog of the reference's ``manifests/v1beta1/installs/*`` kustomize
overlays (katib-standalone, katib-with-kubeflow's MySQL, katib-standalone-postgres) for one
MI355X node without Kubernetes.

``render(profile, prefix)`` writes a self-contained install directory:

* ``katib-config.yaml`` - the reference ``katib-config.yaml`` layout (``init.controller``,
  ``runtime.{suggestions,earlyStoppings,metricsCollectors}``) plus the ``amd`` node section
  (GPUs, slots per GPU, warm workers, state directory), read by ``katib-amd serve --config``;
* ``katib-amd.env`` - the process environment (DB connection variables of the chosen backend,
  ``HSA_ENABLE_IPC_MODE_LEGACY=0`` for RCCL / CUDA-IPC tensor sharing between trial ranks);
* systemd units - ``katib-amd.service`` (scheduler + HTTP API / UI + DBManager gRPC: the
  controller, db-manager and ui Deployments of the reference in one process), and for the
  ``services`` profile the split form: ``katib-amd-db-manager.service``,
  ``katib-amd-suggestion@.service`` (one instance per algorithm, the reference's per-experiment
  suggestion Deployments) and ``katib-amd-earlystopping.service``;
* ``install.sh`` - copies the units into place and enables them.

Profiles: ``standalone`` (native observation store with its journal), ``mysql``,
``postgres`` (the db-manager on that SQL backend, ``db/sql.py``), ``services`` (every
component as its own process, gRPC between them).
"""

from __future__ import annotations

import os
import shlex
import sys
from typing import Dict, List, Optional

import yaml

from ..algorithms.registry import DEFAULT_SUGGESTIONS

PROFILES = ("standalone", "mysql", "postgres", "services")
DB_ENV = {
    "mysql": {"DB_NAME": "mysql", "DB_USER": "root", "DB_PASSWORD": "change-me", "KATIB_MYSQL_DB_HOST": "127.0.0.1",
              "KATIB_MYSQL_DB_PORT": "3306", "KATIB_MYSQL_DB_DATABASE": "katib"},
    "postgres": {"DB_NAME": "postgres", "DB_USER": "katib", "DB_PASSWORD": "change-me",
                 "KATIB_POSTGRESQL_DB_HOST": "127.0.0.1", "KATIB_POSTGRESQL_DB_PORT": "5432",
                 "KATIB_POSTGRESQL_DB_DATABASE": "katib", "KATIB_POSTGRESQL_SSL_MODE": "disable"},
}


def katib_config(state_dir: str, gpus: Optional[int], slots_per_gpu: int) -> Dict:
    """The node's katib-config.yaml document (reference layout + ``amd`` section)."""
    return {
        "apiVersion": "config.kubeflow.org/v1beta1",
        "kind": "KatibConfig",
        "init": {"controller": {
            "experimentSuggestionName": "default",
            "metricsAddr": ":8080",
            "healthzAddr": ":18080",
            "trialResources": ["Job.v1.batch", "LocalProcess.v1.katib-amd.io", "Function.v1.katib-amd.io",
                               "PyTorchJob.v1.kubeflow.org", "TFJob.v1.kubeflow.org", "XGBoostJob.v1.kubeflow.org",
                               "MXJob.v1.kubeflow.org", "MPIJob.v1.kubeflow.org"],
        }},
        "runtime": {
            "suggestions": [{"algorithmName": a, "service": s} for a, s in sorted(DEFAULT_SUGGESTIONS.items())],
            "earlyStoppings": [{"algorithmName": "medianstop", "service": "medianstop"}],
            "metricsCollectors": [{"kind": k} for k in ("StdOut", "File", "TensorFlowEvent", "PrometheusMetric")],
        },
        "amd": {"num_devices": gpus, "slots_per_device": slots_per_gpu, "warm_workers": True,
                "state_dir": state_dir, "multi_gpu_launch": "ranks"},
    }


def _unit(description: str, exec_start: List[str], env_file: str, user: str, after: str = "network-online.target",
          extra: str = "") -> str:
    return "\n".join([
        "[Unit]", "Description=%s" % description, "After=%s" % after, "Wants=network-online.target", "",
        "[Service]", "Type=simple", "User=%s" % user, "EnvironmentFile=%s" % env_file,
        "ExecStart=%s" % " ".join(shlex.quote(a) for a in exec_start),
        "Restart=on-failure", "RestartSec=5", "KillSignal=SIGTERM", "TimeoutStopSec=60", "LimitNOFILE=65536",
        *([extra] if extra else []), "",
        "[Install]", "WantedBy=multi-user.target", ""])


def render(profile: str, prefix: str, python: str = "", user: str = "katib", state_dir: str = "/var/lib/katib-amd",
           gpus: Optional[int] = None, slots_per_gpu: int = 1, api_port: int = 8080,
           grpc_port: int = 6789, listen: str = "127.0.0.1") -> Dict[str, str]:
    """Write the install of ``profile`` under ``prefix``; returns {relative path: content}.

    The HTTP API binds ``listen`` (loopback by default: the API accepts trials whose command
    runs as the service user); the unauthenticated gRPC services always bind loopback. A
    non-loopback ``listen`` makes the API require a bearer token,
    generated into ``api-token`` (mode 0600) and passed with ``--token-file``. The env file (DB
    password) and the token are written 0600 and chowned to the service user by install.sh."""
    if profile not in PROFILES:
        raise ValueError("unknown profile %r (one of %s)" % (profile, ", ".join(PROFILES)))
    python = python or sys.executable
    prefix = os.path.abspath(prefix)
    cfg_path = os.path.join(prefix, "katib-config.yaml")
    env_path = os.path.join(prefix, "katib-amd.env")
    base = [python, "-m", "katib_amd"]
    env = {"HSA_ENABLE_IPC_MODE_LEGACY": "0", "PYTHONUNBUFFERED": "1", "KATIB_AMD_STATE_DIR": state_dir}
    db = profile if profile in DB_ENV else ""
    env.update(DB_ENV.get(db, {}))
    files: Dict[str, str] = {
        "katib-config.yaml": yaml.safe_dump(katib_config(state_dir, gpus, slots_per_gpu), sort_keys=False),
        "katib-amd.env": "".join("%s=%s\n" % kv for kv in sorted(env.items())),
    }
    from ..controller.apiserver import is_loopback

    secret = {"katib-amd.env"}
    serve = base + ["serve", "--address", listen, "--port", str(api_port), "--state-dir", state_dir,
                    "--config", cfg_path]
    if not is_loopback(listen):
        import secrets

        files["api-token"] = secrets.token_hex(32) + "\n"
        secret.add("api-token")
        serve += ["--token-file", os.path.join(prefix, "api-token")]
    # the gRPC services (db-manager, median-stop) carry no authentication: they stay on loopback
    # whatever ``listen`` says; only the token-protected HTTP API follows ``listen``
    bind = "127.0.0.1:%d"
    if gpus is not None:
        serve += ["--gpus", str(gpus)]
    units = []
    if profile == "services":
        db_mgr = base + ["db-manager", "--address", bind % grpc_port, "--journal",
                         os.path.join(state_dir, "observations.journal")]
        files["katib-amd-db-manager.service"] = _unit("Katib (MI355X) DBManager gRPC", db_mgr, env_path, user)
        files["katib-amd-suggestion@.service"] = _unit(
            "Katib (MI355X) suggestion service %i", base + ["suggestion-server", "--algorithm", "%i", "--address",
                                                            "unix:/run/katib-amd/suggestion-%i.sock", "--data-root",
                                                            os.path.join(state_dir, "suggestions", "%i")],
            env_path, user, extra="RuntimeDirectory=katib-amd\nRuntimeDirectoryPreserve=yes")
        files["katib-amd-earlystopping.service"] = _unit(
            "Katib (MI355X) median-stop early stopping", base + ["earlystopping-server", "--address", bind % 6788,
                                                               "--db-manager", "127.0.0.1:%d" % grpc_port],
            env_path, user, after="katib-amd-db-manager.service")
        units += ["katib-amd-db-manager.service", "katib-amd-earlystopping.service"]
        files["katib-amd.service"] = _unit("Katib (MI355X) scheduler, HTTP API and UI", serve, env_path, user,
                                           after="katib-amd-db-manager.service")
    elif db:
        db_mgr = base + ["db-manager", "--address", bind % grpc_port, "--db", db]
        files["katib-amd-db-manager.service"] = _unit("Katib (MI355X) DBManager gRPC on %s" % db, db_mgr, env_path,
                                                      user, after="%s.service" % ("mysqld" if db == "mysql"
                                                                                  else "postgresql"))
        units.append("katib-amd-db-manager.service")
        files["katib-amd.service"] = _unit("Katib (MI355X) scheduler, HTTP API and UI", serve, env_path, user)
    else:
        files["katib-amd.service"] = _unit("Katib (MI355X) scheduler, HTTP API, UI and DBManager gRPC",
                                           serve + ["--grpc", bind % grpc_port], env_path, user)
    units.append("katib-amd.service")
    files["install.sh"] = "\n".join([
        "#!/bin/sh", "# %s install of katib-amd (rendered by 'katib-amd install')" % profile, "set -e",
        "install -d -o %s %s" % (shlex.quote(user), shlex.quote(state_dir)),
        *["chown %s %s && chmod 0600 %s" % (shlex.quote(user), shlex.quote(os.path.join(prefix, f)),
                                             shlex.quote(os.path.join(prefix, f))) for f in sorted(secret)],
        *["install -m 0644 %s /etc/systemd/system/" % shlex.quote(os.path.join(prefix, u))
          for u in sorted(f for f in files if f.endswith(".service"))],
        "systemctl daemon-reload",
        "systemctl enable --now %s" % " ".join(units), ""])
    os.makedirs(prefix, exist_ok=True)
    for name, text in files.items():
        path = os.path.join(prefix, name)
        mode = 0o600 if name in secret else (0o755 if name.endswith(".sh") else 0o644)
        fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, mode)
        with os.fdopen(fd, "w") as f:
            f.write(text)
        os.chmod(path, mode)  # also when the file existed with other permissions
    return files
