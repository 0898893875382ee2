"""``katib-amd`` command line (``python -m katib_amd ...``).

Node daemon and one-shot runs (replacing ``kubectl apply`` + the katib-controller
deployment), plus standalone servers for each reference binary:

* ``run FILE.yaml``         - run the Experiment(s) in FILE to completion in-process, print results
* ``serve``                 - scheduler daemon: HTTP API (:mod:`~katib_amd.controller.apiserver`),
                              DBManager gRPC on the observation store, journal + restore
* ``apply -f FILE`` / ``get`` / ``describe`` / ``delete`` / ``edit-budget`` - talk to a daemon
* ``suggestion-server``     - one algorithm as a gRPC Suggestion service (cmd/suggestion/*/main.py)
* ``earlystopping-server``  - medianstop as a gRPC EarlyStopping service (cmd/earlystopping/medianstop)
* ``db-manager``            - DBManager gRPC server on the native store (cmd/db-manager)
* ``metrics-collector``     - file/StdOut collector (cmd/metricscollector/.../file-metricscollector)
"""

from __future__ import annotations

import argparse
import json
import os
import signal
import sys
import threading
import time

DEFAULT_HOST = "http://127.0.0.1:8080"


# ----------------------------------------------------------------------------- helpers
def _load_file(path):
    from .api.yaml_io import load_documents

    with open(path) as f:
        return load_documents(f.read())


def _summary(e, trials):
    st = e.status
    cond = [c for c in (st.conditions or []) if c.status == "True"]
    out = {
        "name": e.metadata.name, "namespace": e.metadata.namespace,
        "condition": cond[-1].type if cond else "", "reason": cond[-1].reason if cond else "",
        "trials": st.trials or 0, "succeeded": st.trials_succeeded or 0, "failed": st.trials_failed or 0,
        "early_stopped": st.trials_early_stopped or 0, "killed": st.trials_killed or 0,
    }
    best = st.current_optimal_trial
    if best is not None and best.best_trial_name:
        out["optimal_trial"] = {
            "name": best.best_trial_name,
            "parameters": {p.name: p.value for p in best.parameter_assignments or []},
            "metrics": {m.name: {"min": m.min, "max": m.max, "latest": m.latest}
                        for m in (best.observation.metrics if best.observation else []) or []},
        }
    if st.start_time and st.completion_time:
        from .api.models import parse_time

        out["duration_s"] = round((parse_time(st.completion_time) - parse_time(st.start_time)).total_seconds(), 3)
    return out


def _print_table(rows, cols):
    widths = [max(len(c), *(len(str(r.get(c, ""))) for r in rows)) if rows else len(c) for c in cols]
    print("  ".join(c.upper().ljust(w) for c, w in zip(cols, widths)))
    for r in rows:
        print("  ".join(str(r.get(c, "")).ljust(w) for c, w in zip(cols, widths)))


def _wait_signal():
    ev = threading.Event()
    for s in (signal.SIGINT, signal.SIGTERM):
        signal.signal(s, lambda *_: ev.set())
    while not ev.is_set():
        ev.wait(1.0)


# ----------------------------------------------------------------------------- commands
def cmd_run(a):
    from .controller.manager import Manager

    m = Manager(state_dir=a.state_dir, num_devices=a.gpus, journal=bool(a.state_dir))
    if a.slots_per_gpu:
        m.config.amd.slots_per_device = a.slots_per_gpu
        m.slots = m.N.SlotPool(m.n_devices, a.slots_per_gpu)
    exps, cms = _load_file(a.file)
    for cm in cms:
        m.configmaps.put_manifest(cm)
    names = []
    for e in exps:
        if type(e).__name__ != "V1beta1Experiment":
            continue
        m.create_experiment(e, a.namespace)
        names.append(e.metadata.name)
    results = []
    try:
        for n in names:
            done = m.run_until_complete(n, a.namespace, timeout=a.timeout)
            results.append(_summary(done, m.list_trials(n, a.namespace)))
            if not a.json:
                rows = []
                for t in m.list_trials(n, a.namespace):
                    row = {"trial": t.metadata.name, "status": t.status.conditions[-1].type if t.status.conditions
                           else ""}
                    for p in t.spec.parameter_assignments or []:
                        row[p.name] = p.value
                    if t.status.observation:
                        for mt in t.status.observation.metrics or []:
                            row[mt.name] = mt.latest
                    rows.append(row)
                cols = ["trial", "status"] + [p.name for p in done.spec.parameters or []] + \
                    [done.spec.objective.objective_metric_name]
                _print_table(rows, cols)
        if a.trace:
            m.tracer.export(a.trace)
            for r_ in results:
                r_["trace_phase_latencies_s"] = m.tracer.phase_latencies()
    finally:
        m.shutdown()
    print(json.dumps(results if len(results) != 1 else results[0], indent=None if a.json else 2))
    return 0 if all(r["condition"] == "Succeeded" for r in results) else 1


def cmd_serve(a):
    from .controller.apiserver import ApiServer
    from .controller.manager import Manager
    from .rpc.server import make_server

    from .controller.apiserver import is_loopback

    token = None
    if a.token_file:
        with open(a.token_file) as f:
            token = f.read().strip()
    elif os.environ.get("KATIB_AMD_API_TOKEN"):
        token = os.environ["KATIB_AMD_API_TOKEN"]
    api_addr = a.address or "0.0.0.0"  # '' binds every interface
    if not is_loopback(api_addr) and token is None and not a.insecure_listen:
        # the API accepts Job / LocalProcess trials whose command runs as this user: never open
        # it to the network without a token
        print("refusing to listen on %s without --token-file (or --insecure-listen)" % api_addr, file=sys.stderr)
        return 2
    if a.grpc and not _grpc_bind_ok(a.grpc, a.insecure_grpc):
        return 2
    m = Manager(state_dir=a.state_dir, num_devices=a.gpus, journal=True)
    if a.config:
        from .controller.config import KatibConfig

        m.config = KatibConfig.load(a.config)
    restored = m.restore()
    m.start()
    if m.config.amd.zygote:  # the cold-trial fork server warms up with the daemon, not with the first trial
        m.start_zygote(wait=False)
    api = ApiServer(m, a.address, a.port, token=token).start()
    grpc_srv = None
    if a.grpc:
        grpc_srv = make_server(a.grpc, store=m.store)
        grpc_srv.start()
    print(json.dumps({"api": "http://%s:%d" % (a.address, api.port), "grpc": a.grpc or None,
                      "restored": restored, "gpus": m.n_devices}), flush=True)
    _wait_signal()
    api.stop()
    if grpc_srv is not None:
        grpc_srv.stop(0)
    m.shutdown()
    return 0


def _remote(a):
    from .sdk.remote import RemoteManager

    return RemoteManager(a.host, a.namespace)


def cmd_apply(a):
    r = _remote(a)
    exps, cms = _load_file(a.file)
    for cm in cms:
        md = cm.get("metadata", {})
        r.add_configmap(md.get("namespace", a.namespace), md["name"], cm.get("data", {}), md.get("labels"))
    for e in exps:
        try:
            r.create_experiment(e, a.namespace)
            print("experiment.kubeflow.org/%s created" % e.metadata.name)
        except ValueError as err:
            if "already exists" not in str(err):
                raise
            cur = r.get_experiment(e.metadata.name, a.namespace)
            e.metadata = cur.metadata
            r.update_experiment(e)
            print("experiment.kubeflow.org/%s configured" % e.metadata.name)
    return 0


def cmd_get(a):
    r = _remote(a)
    if a.kind in ("experiment", "experiments", "exp"):
        items = [r.get_experiment(a.name, a.namespace)] if a.name else r.list_experiments(a.namespace)
        rows = []
        for e in items:
            s = _summary(e, [])
            rows.append({"name": s["name"], "status": s["condition"], "reason": s["reason"], "trials": s["trials"],
                         "succeeded": s["succeeded"], "optimal": s.get("optimal_trial", {}).get("name", "")})
        _print_table(rows, ["name", "status", "reason", "trials", "succeeded", "optimal"])
    elif a.kind in ("trial", "trials"):
        items = [r.get_trial(a.name, a.namespace)] if a.name else r.list_trials(a.experiment, a.namespace)
        rows = []
        for t in items:
            row = {"name": t.metadata.name, "status": t.status.conditions[-1].type if t.status.conditions else "",
                   "experiment": (t.metadata.labels or {}).get("katib.kubeflow.org/experiment", "")}
            if t.status.observation:
                row["objective"] = ",".join("%s=%s" % (mt.name, mt.latest) for mt in t.status.observation.metrics)
            rows.append(row)
        _print_table(rows, ["name", "experiment", "status", "objective"])
    elif a.kind in ("suggestion", "suggestions"):
        items = [r.get_suggestion(a.name, a.namespace)] if a.name else r.list_suggestions(a.namespace)
        rows = [{"name": s.metadata.name, "algorithm": s.spec.algorithm.algorithm_name, "requests": s.spec.requests,
                 "assigned": s.status.suggestion_count} for s in items]
        _print_table(rows, ["name", "algorithm", "requests", "assigned"])
    else:
        raise SystemExit("unknown kind %s" % a.kind)
    return 0


def cmd_describe(a):
    r = _remote(a)
    e = r.get_experiment(a.name, a.namespace)
    print(json.dumps({"spec": e.to_k8s()["spec"], "summary": _summary(e, [])}, indent=2))
    return 0


def cmd_delete(a):
    _remote(a).delete_experiment(a.name, a.namespace)
    print("experiment.kubeflow.org \"%s\" deleted" % a.name)
    return 0


def cmd_edit_budget(a):
    r = _remote(a)
    e = r.get_experiment(a.name, a.namespace)
    if a.max_trials is not None:
        e.spec.max_trial_count = a.max_trials
    if a.parallel is not None:
        e.spec.parallel_trial_count = a.parallel
    if a.max_failed is not None:
        e.spec.max_failed_trial_count = a.max_failed
    r.update_experiment(e)
    print("experiment.kubeflow.org/%s budget updated" % a.name)
    return 0


def _grpc_bind_ok(address: str, insecure: bool) -> bool:
    """The gRPC services (DBManager, Suggestion, EarlyStopping) have no authentication - the HTTP
    API's bearer token does not cover them - so they bind loopback / unix sockets unless the
    operator explicitly opts in (``--insecure-grpc``, e.g. behind a firewall or an mTLS proxy)."""
    from .controller.apiserver import is_loopback

    if is_loopback(address) or insecure:
        return True
    print("refusing to serve gRPC on %s: the gRPC services are unauthenticated; bind 127.0.0.1 / a unix "
          "socket or pass --insecure-grpc" % address, file=sys.stderr)
    return False


def cmd_suggestion_server(a):
    from .algorithms.registry import create_service
    from .rpc.server import make_server

    if not _grpc_bind_ok(a.address, a.insecure_grpc):
        return 2

    svc = create_service(a.algorithm, data_root=a.data_root)
    srv = make_server(a.address, suggestion_service=svc)
    srv.start()
    print("suggestion service %s listening on %s" % (a.algorithm, a.address), flush=True)
    _wait_signal()
    srv.stop(0)
    return 0


class _GrpcLogSource:
    """Observation logs from a remote DBManager (medianstop outside the scheduler)."""

    def __init__(self, address):
        import grpc

        from .rpc.client import DBManagerStub

        self.stub = DBManagerStub(grpc.insecure_channel(address))

    def get_observation_log(self, trial, metric="", start="", end=""):
        from .rpc import api_pb2 as api

        rep = self.stub.GetObservationLog(api.GetObservationLogRequest(trial_name=trial, metric_name=metric,
                                                                       start_time=start, end_time=end))
        return [(m.time_stamp, m.metric.name, m.metric.value) for m in rep.observation_log.metric_logs]


def cmd_earlystopping_server(a):
    from .earlystopping.medianstop import MedianStopService
    from .rpc.server import make_server

    if not _grpc_bind_ok(a.address, a.insecure_grpc):
        return 2
    marked = []
    svc = MedianStopService(log_source=_GrpcLogSource(a.db_manager) if a.db_manager else None,
                            set_trial_status=lambda n: (marked.append(n), print("early stopped: %s" % n, flush=True)))
    srv = make_server(a.address, early_stopping_service=svc)
    srv.start()
    print("earlystopping service medianstop listening on %s" % a.address, flush=True)
    _wait_signal()
    srv.stop(0)
    return 0


def cmd_db_manager(a):
    from . import native
    from .rpc.server import make_server

    if not _grpc_bind_ok(a.address, a.insecure_grpc):
        return 2
    db = (a.db or os.environ.get("DB_NAME", "")).lower()
    if db not in ("", "native"):
        from .db.sql import new_observation_db

        store = new_observation_db(db, connect_timeout=a.connect_timeout)
        srv = make_server(a.address, store=store)
        srv.start()
        print("db-manager listening on %s (%s backend)" % (a.address, db), flush=True)
        _wait_signal()
        srv.stop(0)
        store.close()
        return 0
    N = native.load()
    store = N.ObservationStore()
    if a.journal:
        if os.path.exists(a.journal):
            store.load_journal(a.journal)
        store.open_journal(a.journal)
    srv = make_server(a.address, store=store)
    srv.start()
    print("db-manager listening on %s (%d trials restored)" % (a.address, len(store.trials())), flush=True)
    _wait_signal()
    srv.stop(0)
    if a.journal:
        store.close_journal()
    return 0


def cmd_metrics_collector(a, rest):
    from .metricscollector.file_collector import collect, parse_args

    return collect(parse_args(rest))


def cmd_install(a):
    from .deploy import render

    files = render(a.profile, a.prefix, python=a.python, user=a.user, state_dir=a.state_dir, gpus=a.gpus,
                   slots_per_gpu=a.slots_per_gpu, listen=a.listen)
    print(json.dumps({"profile": a.profile, "prefix": os.path.abspath(a.prefix), "files": sorted(files)}))
    return 0


def cmd_openapi(a):
    from .api import openapi

    print(openapi.dumps(include_k8s=a.with_k8s))
    return 0


def cmd_inject(a):
    """Print the pod with the metrics collector injected (the /mutate-pod webhook's
    rewrite) for running a trial's pod on a cluster."""
    import yaml

    from .api import katibconfig as KC
    from .controller.inject import mutate_pod

    with open(a.trial) as f:
        trial = yaml.safe_load(f)
    with open(a.pod) as f:
        pod = yaml.safe_load(f)
    kind = (((trial.get("spec") or {}).get("metricsCollector") or {}).get("collector") or {}).get("kind", "StdOut")
    cfg = {}
    if a.config:
        entries = (KC.load_file(a.config).get("runtime") or {}).get("metricsCollectors") or []
        cfg = next((e for e in entries if e.get("kind") == kind), {})
    md = trial.get("metadata") or {}
    exp = (md.get("labels") or {}).get("katib.kubeflow.org/experiment", "")
    sugg = {(md.get("namespace"), exp): a.early_stopping_algorithm} if a.early_stopping_algorithm else None
    print(yaml.safe_dump(mutate_pod(pod, trial, cfg, a.image, sugg, a.db_manager or None), sort_keys=False), end="")
    return 0


def build_parser():
    p = argparse.ArgumentParser(prog="katib-amd", description="Katib-compatible AutoML engine for MI355X nodes")
    sub = p.add_subparsers(dest="cmd", required=True)

    r = sub.add_parser("run", help="run the Experiment(s) in a YAML file to completion")
    r.add_argument("file")
    r.add_argument("--gpus", type=int, default=None, help="GPUs to use (default: all visible)")
    r.add_argument("--slots-per-gpu", type=int, default=0)
    r.add_argument("--state-dir", default=None)
    r.add_argument("--namespace", default="default")
    r.add_argument("--timeout", type=float, default=24 * 3600)
    r.add_argument("--json", action="store_true")
    r.add_argument("--trace", default=None, help="write the trial/suggestion timeline (Chrome trace JSON)")
    r.set_defaults(fn=cmd_run)

    s = sub.add_parser("serve", help="run the scheduler daemon with its HTTP API")
    s.add_argument("--address", default="127.0.0.1")
    s.add_argument("--port", type=int, default=8080)
    s.add_argument("--grpc", default="", help="also serve DBManager gRPC here, e.g. 127.0.0.1:6789")
    s.add_argument("--token-file", default="", help="bearer token required by the HTTP API (needed off loopback)")
    s.add_argument("--insecure-listen", action="store_true",
                   help="allow a non-loopback --address without a token (not recommended)")
    s.add_argument("--insecure-grpc", action="store_true",
                   help="allow a non-loopback --grpc address (the gRPC services have no authentication)")
    s.add_argument("--state-dir", default=None)
    s.add_argument("--gpus", type=int, default=None)
    s.add_argument("--config", default="", help="katib-config.yaml")
    s.set_defaults(fn=cmd_serve)

    for name, fn in (("apply", cmd_apply), ("get", cmd_get), ("describe", cmd_describe), ("delete", cmd_delete),
                     ("edit-budget", cmd_edit_budget)):
        c = sub.add_parser(name)
        c.add_argument("--host", default=os.environ.get("KATIB_AMD_HOST", DEFAULT_HOST))
        c.add_argument("-n", "--namespace", default="default")
        if name == "apply":
            c.add_argument("-f", "--file", required=True)
        elif name == "get":
            c.add_argument("kind")
            c.add_argument("name", nargs="?")
            c.add_argument("-e", "--experiment", default=None)
        else:
            if name != "describe" and name != "delete" and name != "edit-budget":
                c.add_argument("kind")
            c.add_argument("name")
        if name == "edit-budget":
            c.add_argument("--max-trials", type=int)
            c.add_argument("--parallel", type=int)
            c.add_argument("--max-failed", type=int)
        c.set_defaults(fn=fn)

    g = sub.add_parser("suggestion-server", help="serve one algorithm over gRPC (port 6789)")
    g.add_argument("--algorithm", required=True)
    g.add_argument("--address", default="127.0.0.1:6789")
    g.add_argument("--data-root", default="/opt/katib/data")
    g.add_argument("--insecure-grpc", action="store_true", help="allow a non-loopback --address (no auth)")
    g.set_defaults(fn=cmd_suggestion_server)

    es = sub.add_parser("earlystopping-server", help="serve medianstop over gRPC (port 6788)")
    es.add_argument("--address", default="127.0.0.1:6788")
    es.add_argument("--db-manager", default="")
    es.add_argument("--insecure-grpc", action="store_true", help="allow a non-loopback --address (no auth)")
    es.set_defaults(fn=cmd_earlystopping_server)

    d = sub.add_parser("db-manager", help="DBManager gRPC server on the native observation store")
    d.add_argument("--address", default="127.0.0.1:6789")
    d.add_argument("--journal", default="", help="append-only journal file for persistence")
    d.add_argument("--db", default="", help="native (default) | sqlite | mysql | postgres (else $DB_NAME)")
    d.add_argument("--connect-timeout", type=float, default=60.0, help="seconds to wait for the database")
    d.add_argument("--insecure-grpc", action="store_true", help="allow a non-loopback --address (no auth)")
    d.set_defaults(fn=cmd_db_manager)

    sub.add_parser("metrics-collector", help="file/StdOut metrics collector (reference flags)", add_help=False)

    inj = sub.add_parser("inject", help="print a trial pod with the metrics-collector sidecar injected")
    inj.add_argument("--trial", required=True, help="Trial manifest (YAML)")
    inj.add_argument("--pod", required=True, help="Pod manifest (YAML)")
    inj.add_argument("--config", default="", help="katib-config.yaml (metricsCollectors entry for the kind)")
    inj.add_argument("--image", default="", help="collector image (overrides the config)")
    inj.add_argument("--early-stopping-algorithm", default="", help="algorithm serving -s-earlystop")
    inj.add_argument("--db-manager", default="", help="DBManager address (default from KATIB_DB_MANAGER_*)")
    inj.set_defaults(fn=cmd_inject)

    ins = sub.add_parser("install", help="render a node install (katib-config.yaml, env file, systemd units)")
    ins.add_argument("--profile", default="standalone", help="standalone | mysql | postgres | services")
    ins.add_argument("--prefix", required=True, help="output directory")
    ins.add_argument("--python", default="", help="interpreter for the units (default: this one)")
    ins.add_argument("--user", default="katib")
    ins.add_argument("--state-dir", default="/var/lib/katib-amd")
    ins.add_argument("--gpus", type=int, default=None)
    ins.add_argument("--slots-per-gpu", type=int, default=1)
    ins.add_argument("--listen", default="127.0.0.1",
                     help="bind address of the API and gRPC services (non-loopback: a token file is generated)")
    ins.set_defaults(fn=cmd_install)

    oa = sub.add_parser("openapi", help="print the v1beta1 Swagger 2.0 document (reference swagger.json layout)")
    oa.add_argument("--with-k8s", action="store_true", help="also define the v1.ObjectMeta / v1.Time types")
    oa.set_defaults(fn=cmd_openapi)
    return p


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    if argv and argv[0] == "metrics-collector":
        return cmd_metrics_collector(None, argv[1:])
    a = build_parser().parse_args(argv)
    return a.fn(a)


if __name__ == "__main__":
    sys.exit(main())
