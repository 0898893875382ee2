"""Standalone File/StdOut metrics collector (reference
``cmd/metricscollector/v1beta1/file-metricscollector/main.go:102-456``).

The in-process scheduler collects metrics itself (native ``TrialRuntime``); this CLI
is the equivalent for trials run outside it (another host, a batch system): same
flags as the reference sidecar, same parsing (native :class:`MetricsParser`: default
``name=value`` regex, user filters, TEXT/JSON with timestamps), same early-stopping
semantics, and the observation log goes to a DBManager over gRPC
(``ReportObservationLog``).

Instead of sharing a PID namespace with the training container and polling
``/proc`` (``pkg/metricscollector/v1beta1/common/pns.go``), the collector either
launches the training command itself (``-- cmd args...``, stdout redirected into the
metrics file like the injected ``sh -c`` wrapper) or tails a file written by a
process it waits for with ``-pid``.

Early stopping: for each rule ``name;value;comparison;startStep`` the best-so-far
objective (min/max by ``-o-type``) or latest value of other metrics is tracked;
``startStep`` counts reports of that metric; when every rule holds the child gets
SIGTERM, the log is reported and ``SetTrialStatus`` is called on ``-s-earlystop``.
"""

from __future__ import annotations

import argparse
import os
import signal
import subprocess
import sys
import time
from typing import Dict, List, Optional, Tuple


def parse_args(argv):
    p = argparse.ArgumentParser(prog="katib-amd metrics-collector", description=__doc__.split("\n")[0])
    p.add_argument("-t", dest="trial_name", required=True)
    p.add_argument("-m", dest="metric_names", required=True, help="';'-separated, objective first")
    p.add_argument("-o-type", dest="objective_type", default="maximize")
    p.add_argument("-s-db", dest="db_manager", default="katib-db-manager.kubeflow:6789")
    p.add_argument("-path", dest="path", default="/var/log/katib/metrics.log")
    p.add_argument("-f", dest="filters", default="", help="';'-separated metric filter regexes")
    p.add_argument("-format", dest="format", default="TEXT", choices=["TEXT", "JSON"])
    p.add_argument("-w", dest="wait_all", default="true")
    p.add_argument("-stop-rule", dest="stop_rules", action="append", default=[],
                   help="name;value;comparison;startStep")
    p.add_argument("-s-earlystop", dest="earlystop", default="")
    p.add_argument("-pid", dest="pid", type=int, default=0, help="wait for this process instead of launching one")
    p.add_argument("-poll", dest="poll", type=float, default=0.2)
    p.add_argument("cmd", nargs=argparse.REMAINDER, help="-- training command (stdout/stderr -> -path)")
    a = p.parse_args(argv)
    if a.cmd and a.cmd[0] == "--":
        a.cmd = a.cmd[1:]
    return a


class RuleTracker:
    """Early-stopping rule evaluation (file-metricscollector/main.go:143-230)."""

    def __init__(self, rules: List[Tuple[str, float, str, int]], objective: str, objective_type: str):
        self.rules = rules
        self.objective = objective
        self.minimize = objective_type == "minimize"
        self.best: Dict[str, float] = {}
        self.countdown = {r[0]: r[3] for r in rules}
        self.started = {r[0]: r[3] <= 0 for r in rules}

    def observe(self, name: str, value: float) -> None:
        if name == self.objective:
            b = self.best.get(name)
            if b is None or (value < b if self.minimize else value > b):
                self.best[name] = value
        else:
            self.best[name] = value
        if name in self.countdown and not self.started[name]:
            self.countdown[name] -= 1
            if self.countdown[name] == 0:
                self.started[name] = True

    def triggered(self) -> bool:
        if not self.rules:
            return False
        for name, val, cmp_, _ in self.rules:
            if not self.started.get(name) or name not in self.best:
                return False
            v = self.best[name]
            ok = (cmp_ == "less" and v < val) or (cmp_ == "greater" and v > val) or (cmp_ == "equal" and v == val)
            if not ok:
                return False
        return True


def _rules(specs: List[str]):
    out = []
    for s in specs:
        name, value, cmp_, start = s.split(";")
        out.append((name, float(value), cmp_.lower(), int(start or 0)))
    return out


def _alive(pid: int) -> bool:
    try:
        os.kill(pid, 0)
        return True
    except OSError:
        return False


def report(db_address: str, trial: str, logs) -> None:
    import grpc

    from ..rpc import api_pb2 as api
    from ..rpc.client import DBManagerStub

    with grpc.insecure_channel(db_address) as ch:
        DBManagerStub(ch).ReportObservationLog(api.ReportObservationLogRequest(
            trial_name=trial, observation_log=api.ObservationLog(metric_logs=[
                api.MetricLog(time_stamp=t, metric=api.Metric(name=n, value=v)) for t, n, v in logs])),
            timeout=60)


def set_trial_status(address: str, trial: str) -> None:
    import grpc

    from ..rpc import api_pb2 as api
    from ..rpc.client import EarlyStoppingStub

    with grpc.insecure_channel(address) as ch:
        EarlyStoppingStub(ch).SetTrialStatus(api.SetTrialStatusRequest(trial_name=trial), timeout=60)


class CollectError(Exception):
    """errOpenFile / errFileFormat / errParseJson of CollectObservationLog."""


def parse_observation_log(content: str, metrics: List[str], filters: List[str], file_format: str,
                          parser=None) -> List[Tuple[str, str, str]]:
    """Parse a finished metrics file body into (timestamp, name, value) rows; when the
    objective (first metric) never appears the log is one ``unavailable`` row
    (file-metricscollector.go CollectObservationLog)."""
    from .. import native

    if file_format not in ("TEXT", "JSON"):
        raise CollectError("format must be set to TEXT or JSON")
    if parser is None:
        parser = native.load().MetricsParser(list(metrics), list(filters or []), 1 if file_format == "JSON" else 0)
    try:
        logs = parser.parse_content(content)
    except ValueError as e:
        raise CollectError("failed to parse JSON line: %s" % e)
    if metrics and not any(n == metrics[0] for _, n, _ in logs):
        from ..api.models import ZERO_TIME

        logs = [(ZERO_TIME, metrics[0], "unavailable")]
    return logs


def collect_observation_log(path: str, metrics: List[str], filters: List[str],
                            file_format: str) -> List[Tuple[str, str, str]]:
    if file_format not in ("TEXT", "JSON"):
        raise CollectError("format must be set to TEXT or JSON")
    try:
        with open(path, errors="replace") as f:
            content = f.read()
    except OSError as e:
        raise CollectError("failed to open file: %s" % e)
    return parse_observation_log(content, metrics, filters, file_format)


def collect(args, reporter=report, status_setter=set_trial_status) -> int:
    from .. import native

    N = native.load()
    names = [m for m in args.metric_names.split(";") if m]
    filters = [f for f in args.filters.split(";") if f]
    fmt = 1 if args.format == "JSON" else 0
    parser = N.MetricsParser(names, filters, fmt)
    tracker = RuleTracker(_rules(args.stop_rules), names[0], args.objective_type)
    os.makedirs(os.path.dirname(os.path.abspath(args.path)), exist_ok=True)
    child: Optional[subprocess.Popen] = None
    if args.cmd:
        out = open(args.path, "ab")
        child = subprocess.Popen(args.cmd, stdout=out, stderr=subprocess.STDOUT, start_new_session=True)
        pid = child.pid
    else:
        pid = args.pid
    early = False
    pos, buf = 0, b""
    rule_names = [r[0] for r in tracker.rules]

    def running():
        if child is not None:
            return child.poll() is None
        return pid > 0 and _alive(pid)

    while True:
        alive = running()
        if tracker.rules and os.path.exists(args.path):
            with open(args.path, "rb") as f:
                f.seek(pos)
                chunk = f.read()
                pos += len(chunk)
            buf += chunk
            *lines, buf = buf.split(b"\n")
            for ln in lines:
                for name, val in parser.rule_values(ln.decode(errors="replace"), rule_names):
                    tracker.observe(name, val)
            if not early and tracker.triggered():
                early = True
                if child is not None:
                    os.killpg(child.pid, signal.SIGTERM)
                elif pid > 0:
                    os.kill(pid, signal.SIGTERM)
                deadline = time.time() + 60
                while running() and time.time() < deadline:
                    time.sleep(0.1)
                break
        if not alive:
            break
        time.sleep(args.poll)
    code = child.wait() if child is not None else 0
    content = open(args.path, errors="replace").read() if os.path.exists(args.path) else ""
    logs = parse_observation_log(content, names, filters, args.format, parser)
    reporter(args.db_manager, args.trial_name, logs)
    if early and args.earlystop:
        status_setter(args.earlystop, args.trial_name)
    return 0 if early else code


def main(argv=None):
    args = parse_args(sys.argv[1:] if argv is None else argv)
    sys.exit(collect(args))


if __name__ == "__main__":
    main()
