"""gRPC client stubs for the Katib services (no protoc needed)."""

from __future__ import annotations

from . import api_pb2 as api


def _cls(full):
    return api.message_factory.GetMessageClass(api.POOL.FindMessageTypeByName(full))


class _Stub:
    service = ""

    def __init__(self, channel):
        for m, req, rep in api.SERVICES[self.service]:
            setattr(self, m, channel.unary_unary("/%s.%s/%s" % (api.PKG, self.service, m),
                                                 request_serializer=_cls(req).SerializeToString,
                                                 response_deserializer=_cls(rep).FromString))


class DBManagerStub(_Stub):
    service = "DBManager"


class SuggestionStub(_Stub):
    service = "Suggestion"


class EarlyStoppingStub(_Stub):
    service = "EarlyStopping"


class HealthStub:
    def __init__(self, channel):
        self.Check = channel.unary_unary("/grpc.health.v1.Health/Check",
                                         request_serializer=api.HealthCheckRequest.SerializeToString,
                                         response_deserializer=api.HealthCheckResponse.FromString)
