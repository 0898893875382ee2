"""The MySQL and PostgreSQL observation-log backends end to end through ``new_observation_db``
and the gRPC DBManager, with DB-API driver modules (``pymysql`` / ``psycopg2``, not installed
in this image) stood in by an in-memory SQL engine speaking their ``%s`` paramstyle.

What this pins: connection parameters from the reference env vars (``mysql.go:44-57``,
``postgres.go:39-59``), the dialect DDL executing (``CREATE TABLE`` with ``AUTO_INCREMENT`` /
``serial``), multi-row INSERT, filtered SELECT ordered by time, DELETE, and the
``SKIP_DB_INITIALIZATION`` validation query. Server-side typing (MySQL DATETIME(6) rounding,
PostgreSQL TIMESTAMP parsing) is the real servers' and stays parity-unpinned here."""
import sqlite3
import sys
import types

import pytest

from katib_amd.db import sql as S


class _Cursor:
    def __init__(self, cur, log):
        self.cur, self.log = cur, log

    @property
    def description(self):
        return self.cur.description

    def execute(self, q, args=()):
        assert "?" not in q and "$" not in q, "driver received a non-%%s placeholder: %s" % q
        self.log.append(" ".join(q.split()))
        self.cur.execute(q.replace("%s", "?"), tuple(args))

    def fetchall(self):
        return self.cur.fetchall()

    def close(self):
        self.cur.close()


class _Conn:
    def __init__(self, log):
        self.db = sqlite3.connect(":memory:", check_same_thread=False)
        self.log = log

    def cursor(self):
        return _Cursor(self.db.cursor(), self.log)

    def commit(self):
        self.db.commit()

    def close(self):
        self.db.close()


@pytest.fixture
def drivers(monkeypatch):
    seen = {"log": [], "mysql": None, "postgres": None}
    pymysql = types.ModuleType("pymysql")

    def mysql_connect(**kw):
        seen["mysql"] = kw
        return _Conn(seen["log"])

    pymysql.connect = mysql_connect
    psycopg2 = types.ModuleType("psycopg2")

    def pg_connect(dsn):
        seen["postgres"] = dsn
        return _Conn(seen["log"])

    psycopg2.connect = pg_connect
    monkeypatch.setitem(sys.modules, "pymysql", pymysql)
    monkeypatch.setitem(sys.modules, "psycopg2", psycopg2)
    monkeypatch.setattr(S, "CONNECT_INTERVAL_S", 0.0)
    return seen


LOGS = [("2016-12-31T20:02:05.123456Z", "loss", "0.9"), ("2016-12-31T20:02:06.123456Z", "accuracy", "0.5"),
        ("2016-12-31T20:02:07.123456Z", "loss", "0.4"), ("", "loss", "skipped: no timestamp")]


@pytest.mark.parametrize("db", ["mysql", "postgres"])
def test_backend_end_to_end(drivers, monkeypatch, db):
    monkeypatch.setenv("DB_USER", "katib")
    monkeypatch.setenv("DB_PASSWORD", "secret")
    monkeypatch.setenv("KATIB_MYSQL_DB_HOST", "mysql.local")
    monkeypatch.setenv("KATIB_MYSQL_DB_PORT", "3307")
    monkeypatch.setenv("KATIB_POSTGRESQL_DB_HOST", "pg.local")
    monkeypatch.setenv("KATIB_POSTGRESQL_DB_PORT", "5433")
    store = S.new_observation_db(db)
    if db == "mysql":
        assert drivers["mysql"] == {"host": "mysql.local", "port": 3307, "user": "katib", "password": "secret",
                                    "database": "katib", "connect_timeout": 5}
        assert any("AUTO_INCREMENT" in q for q in drivers["log"])
    else:
        assert drivers["postgres"] == ("host=pg.local port=5433 user=katib password=secret dbname=katib "
                                       "sslmode=disable")
        assert any("serial PRIMARY KEY" in q for q in drivers["log"])
    store.report("t1", LOGS)
    store.report("t2", LOGS[:1])
    got = store.get("t1")
    assert [(n, v) for _, n, v in got] == [("loss", "0.9"), ("accuracy", "0.5"), ("loss", "0.4")]
    assert got[0][0] == "2016-12-31T20:02:05.123456Z"
    assert [v for _, _, v in store.get("t1", metric="loss")] == ["0.9", "0.4"]
    # (fractional bounds: the stand-in engine compares the postgres dialect's RFC 3339 text as strings)
    assert [v for _, _, v in store.get("t1", start="2016-12-31T20:02:05.5Z")] == ["0.5", "0.4"]
    assert [v for _, _, v in store.get("t1", end="2016-12-31T20:02:06.5Z")] == ["0.9", "0.5"]
    store.remove("t1")
    assert store.get("t1") == [] and len(store.get("t2")) == 1
    store.close()


def test_skip_db_initialization_runs_the_validation_query(drivers, monkeypatch):
    monkeypatch.setenv("SKIP_DB_INITIALIZATION", "true")
    with pytest.raises(Exception):  # the table does not exist: validation fails instead of creating it
        S.new_observation_db("mysql")
    assert any(q.startswith("SELECT trial_name, id, time, metric_name, value FROM observation_logs")
               for q in drivers["log"])


def test_mysql_behind_grpc_dbmanager(drivers):
    grpc = pytest.importorskip("grpc")
    from katib_amd.rpc import api_pb2 as api
    from katib_amd.rpc.client import DBManagerStub
    from katib_amd.rpc.server import make_server

    store = S.new_observation_db("mysql")
    srv = make_server("127.0.0.1:0", store=store)
    port = srv.bound_port if hasattr(srv, "bound_port") else None
    if port is None:
        pytest.skip("make_server does not expose the bound port")
    srv.start()
    try:
        stub = DBManagerStub(grpc.insecure_channel("127.0.0.1:%d" % port))
        logs = [api.MetricLog(time_stamp=t, metric=api.Metric(name=n, value=v)) for t, n, v in LOGS[:3]]
        stub.ReportObservationLog(api.ReportObservationLogRequest(
            trial_name="g1", observation_log=api.ObservationLog(metric_logs=logs)))
        rep = stub.GetObservationLog(api.GetObservationLogRequest(trial_name="g1", metric_name="loss"))
        assert [m.metric.value for m in rep.observation_log.metric_logs] == ["0.9", "0.4"]
    finally:
        srv.stop(0)
        store.close()
