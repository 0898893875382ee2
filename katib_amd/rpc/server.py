"""gRPC servers - wire-compatible with the reference services.

* ``DBManager`` on the native observation store or a SQL backend (``katib_amd.db.sql``)
  (``cmd/db-manager/v1beta1/main.go:37-121``),
* ``Suggestion`` exposing any in-process algorithm service (so external Katib
  controllers or tools can use our algorithms, and ``tools`` written against the
  reference protocol keep working; ``cmd/suggestion/*/main.py``),
* ``EarlyStopping`` (``cmd/earlystopping/medianstop/v1beta1/main.py``),
* ``grpc.health.v1.Health`` reporting SERVING for ``manager.v1beta1.Suggestion``
  (``internal/base_health_service.py``) and the DB (``SELECT 1`` equivalent).

Handlers are registered generically (no protoc-generated servicer base classes).
"""

from __future__ import annotations

from concurrent import futures
from typing import Optional

import grpc

from . import api_pb2 as api

MAX_MSG = 2 ** 31 - 1


def _unary(fn, req_cls, rep_cls):
    return grpc.unary_unary_rpc_method_handler(fn, request_deserializer=req_cls.FromString,
                                               response_serializer=rep_cls.SerializeToString)


class DBManagerServicer:
    def __init__(self, store):
        self.store = store

    def ReportObservationLog(self, request, context):
        logs = [(m.time_stamp, m.metric.name, m.metric.value) for m in request.observation_log.metric_logs]
        try:
            self.store.report(request.trial_name, logs)
        except ValueError as e:
            context.abort(grpc.StatusCode.UNKNOWN, str(e))
        return api.ReportObservationLogReply()

    def GetObservationLog(self, request, context):
        try:
            rows = self.store.get(request.trial_name, request.metric_name, request.start_time, request.end_time)
        except ValueError as e:
            context.abort(grpc.StatusCode.UNKNOWN, str(e))
        return api.GetObservationLogReply(observation_log=api.ObservationLog(metric_logs=[
            api.MetricLog(time_stamp=ts, metric=api.Metric(name=n, value=v)) for ts, n, v in rows]))

    def DeleteObservationLog(self, request, context):
        self.store.remove(request.trial_name)
        return api.DeleteObservationLogReply()


class _ContextAdapter:
    """Lets services written against the reference's ``context.set_code`` API run
    under a real gRPC context."""

    def __init__(self, ctx):
        self.ctx = ctx

    def set_code(self, c):
        self.ctx.set_code(c)

    def set_details(self, d):
        self.ctx.set_details(d)


class SuggestionServicer:
    def __init__(self, service):
        self.service = service

    def GetSuggestions(self, request, context):
        try:
            return self.service.GetSuggestions(request, _ContextAdapter(context))
        except Exception as e:
            context.abort(grpc.StatusCode.INTERNAL, str(e))

    def ValidateAlgorithmSettings(self, request, context):
        return self.service.ValidateAlgorithmSettings(request, _ContextAdapter(context))


class EarlyStoppingServicer:
    def __init__(self, service):
        self.service = service

    def GetEarlyStoppingRules(self, request, context):
        return self.service.GetEarlyStoppingRules(request, _ContextAdapter(context))

    def SetTrialStatus(self, request, context):
        return self.service.SetTrialStatus(request, _ContextAdapter(context))

    def ValidateEarlyStoppingSettings(self, request, context):
        return self.service.ValidateEarlyStoppingSettings(request, _ContextAdapter(context))


class HealthServicer:
    """Health.Check; with a database-backed store the DB is probed with ``SELECT 1``
    (db-manager main.go:70-89) and a failing probe reports NOT_SERVING."""

    def __init__(self, serving=("", "grpc.health.v1.Health", "manager.v1beta1.Suggestion",
                                "manager.v1beta1.DBManager", "manager.v1beta1.EarlyStopping"), store=None):
        self.serving = set(serving)
        self.store = store

    def Check(self, request, context):
        if request.service not in self.serving:
            st = api.HealthCheckResponse.SERVICE_UNKNOWN if hasattr(api.HealthCheckResponse, "SERVICE_UNKNOWN") \
                else api.HealthCheckResponse.UNKNOWN
            return api.HealthCheckResponse(status=st)
        probe = getattr(self.store, "select_one", None)
        if probe is not None:
            try:
                probe()
            except Exception as e:
                if context is not None:
                    context.set_details("Failed to execute `SELECT 1` probe: %s" % e)
                return api.HealthCheckResponse(status=api.HealthCheckResponse.NOT_SERVING)
        return api.HealthCheckResponse(status=api.HealthCheckResponse.SERVING)


def _handler(service_name, servicer):
    methods = {}
    for m, req, rep in api.SERVICES[service_name]:
        req_cls = api.message_factory.GetMessageClass(api.POOL.FindMessageTypeByName(req))
        rep_cls = api.message_factory.GetMessageClass(api.POOL.FindMessageTypeByName(rep))
        methods[m] = _unary(getattr(servicer, m), req_cls, rep_cls)
    return grpc.method_handlers_generic_handler(api.PKG + "." + service_name, methods)


def make_server(address: str = "127.0.0.1:6789", store=None, suggestion_service=None, early_stopping_service=None,
                max_workers: int = 10) -> grpc.Server:
    server = grpc.server(futures.ThreadPoolExecutor(max_workers=max_workers),
                         options=[("grpc.max_send_message_length", MAX_MSG),
                                  ("grpc.max_receive_message_length", MAX_MSG)])
    handlers = []
    if store is not None:
        handlers.append(_handler("DBManager", DBManagerServicer(store)))
    if suggestion_service is not None:
        handlers.append(_handler("Suggestion", SuggestionServicer(suggestion_service)))
    if early_stopping_service is not None:
        handlers.append(_handler("EarlyStopping", EarlyStoppingServicer(early_stopping_service)))
    hs = HealthServicer(store=store)
    handlers.append(grpc.method_handlers_generic_handler("grpc.health.v1.Health", {
        "Check": _unary(hs.Check, api.HealthCheckRequest, api.HealthCheckResponse)}))
    server.add_generic_rpc_handlers(handlers)
    port = server.add_insecure_port(address)
    server.bound_port = port
    return server
