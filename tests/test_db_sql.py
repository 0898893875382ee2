"""SQL observation-log backends: ports of the reference
``pkg/db/v1beta1/mysql/mysql_test.go``, ``postgres/postgres_test.go`` and
``cmd/db-manager/v1beta1/main_test.go``. A recording DB-API connection stands in
for go-sqlmock (exact SQL text and arguments are checked); the sqlite backend is
exercised end to end, also behind the gRPC DBManager."""
import pytest

from katib_amd.db import sql as S


class RecordingConn:
    """DB-API connection that records statements and replays canned rows."""

    def __init__(self, rows=None):
        self.calls = []
        self.rows = list(rows or [])

    def cursor(self):
        conn = self

        class Cur:
            description = None

            def execute(self, sql, args=()):
                conn.calls.append((" ".join(sql.split()), tuple(args)))
                self.description = [("c",)] if sql.lstrip().upper().startswith("SELECT") else None

            def fetchall(self):
                out, conn.rows = conn.rows, []
                return out

            def close(self):
                pass

        return Cur()

    def commit(self):
        pass

    def close(self):
        pass


LOGS_MYSQL = [("2016-12-31T20:02:05.123456Z", "f1_score", "88.95"), ("2016-12-31T20:02:05.123456Z", "loss", "0.5")]


def test_mysql_init_select_one(monkeypatch):
    monkeypatch.delenv(S.SKIP_DB_INIT_ENV, raising=False)
    c = RecordingConn()
    db = S.SQLObservationDB(c, S.MySQLDialect())
    db.db_init()
    db.select_one()
    assert c.calls[0][0].startswith("CREATE TABLE IF NOT EXISTS observation_logs")
    assert "id INT AUTO_INCREMENT PRIMARY KEY" in c.calls[0][0] and "time DATETIME(6)" in c.calls[0][0]
    assert c.calls[1] == ("SELECT 1", ())


def test_skip_db_initialization_validates_table(monkeypatch):
    monkeypatch.setenv(S.SKIP_DB_INIT_ENV, "true")
    c = RecordingConn()
    S.SQLObservationDB(c, S.PostgresDialect()).db_init()
    assert c.calls == [(S.VALIDATE_TABLE, ())]


def test_mysql_register_observation_log():
    c = RecordingConn()
    S.SQLObservationDB(c, S.MySQLDialect()).report("test1_trial1", LOGS_MYSQL)
    assert c.calls == [("INSERT INTO observation_logs (trial_name, time, metric_name, value) VALUES "
                        "(?, ?, ?, ?),(?, ?, ?, ?)",
                        ("test1_trial1", "2016-12-31 20:02:05.123456", "f1_score", "88.95",
                         "test1_trial1", "2016-12-31 20:02:05.123456", "loss", "0.5"))]


def test_mysql_get_observation_log():
    c = RecordingConn(rows=[("2016-12-31 21:02:05.123456", "loss", "0.9"), ("2016-12-31 22:02:05.123456", "loss", "0.9")])
    out = S.SQLObservationDB(c, S.MySQLDialect()).get("test1_trial1", "loss", "2016-12-31T21:01:05.123456Z",
                                                      "2016-12-31T22:10:20.123456Z")
    assert c.calls == [("SELECT time, metric_name, value FROM observation_logs WHERE trial_name = ? AND "
                        "metric_name = ? AND time >= ? AND time <= ? ORDER BY time",
                        ("test1_trial1", "loss", "2016-12-31 21:01:05.123456", "2016-12-31 22:10:20.123456"))]
    assert out == [("2016-12-31T21:02:05.123456Z", "loss", "0.9"), ("2016-12-31T22:02:05.123456Z", "loss", "0.9")]


def test_mysql_delete_observation_log():
    c = RecordingConn()
    S.SQLObservationDB(c, S.MySQLDialect()).remove("test1_trial1")
    assert c.calls == [("DELETE FROM observation_logs WHERE trial_name = ?", ("test1_trial1",))]


def test_mysql_dsn(monkeypatch):
    for k in (S.DB_USER_ENV, S.DB_PASSWORD_ENV, S.MYSQL_HOST_ENV, S.MYSQL_PORT_ENV, S.MYSQL_DATABASE_ENV):
        monkeypatch.delenv(k, raising=False)
    assert S.mysql_dsn() == "root:@tcp(katib-mysql:3306)/katib?timeout=5s"


def test_postgres_register_get_delete():
    c = RecordingConn()
    db = S.SQLObservationDB(c, S.PostgresDialect())
    db.report("test1_trial1", [("2016-12-31T20:01:05.123456Z", "f1_score", "88.95"),
                               ("2016-12-31T20:02:05.123456Z", "loss", "0.5")])
    assert c.calls[-1] == ("INSERT INTO observation_logs (trial_name, time, metric_name, value) VALUES "
                           "($1, $2, $3, $4),($5, $6, $7, $8)",
                           ("test1_trial1", "2016-12-31T20:01:05.123456Z", "f1_score", "88.95",
                            "test1_trial1", "2016-12-31T20:02:05.123456Z", "loss", "0.5"))
    c.rows = [("2016-12-31T20:01:05.123456Z", "loss", "0.9"), ("2016-12-31T20:02:05.123456Z", "loss", "0.9")]
    out = db.get("test1_trial1", "loss", "2016-12-31T20:01:05.123456Z", "2016-12-31T20:02:05.123456Z")
    assert c.calls[-1] == ("SELECT time, metric_name, value FROM observation_logs WHERE trial_name = $1 AND "
                           "metric_name = $2 AND time >= $3 AND time <= $4 ORDER BY time",
                           ("test1_trial1", "loss", "2016-12-31T20:01:05.123456Z", "2016-12-31T20:02:05.123456Z"))
    assert len(out) == 2
    db.remove("test1_trial1")
    assert c.calls[-1] == ("DELETE FROM observation_logs WHERE trial_name = $1", ("test1_trial1",))


@pytest.mark.parametrize("env,want", [
    ({}, "host=katib-postgres port=5432 user=katib password= dbname=katib sslmode=disable"),
    ({S.DB_USER_ENV: "testUser"}, "host=katib-postgres port=5432 user=testUser password= dbname=katib sslmode=disable"),
    ({S.PG_HOST_ENV: "testHost"}, "host=testHost port=5432 user=katib password= dbname=katib sslmode=disable"),
    ({S.PG_PORT_ENV: "1234"}, "host=katib-postgres port=1234 user=katib password= dbname=katib sslmode=disable"),
    ({S.PG_DATABASE_ENV: "testDB"}, "host=katib-postgres port=5432 user=katib password= dbname=testDB sslmode=disable"),
    ({S.DB_PASSWORD_ENV: "testPassword"},
     "host=katib-postgres port=5432 user=katib password=testPassword dbname=katib sslmode=disable"),
    ({S.PG_SSL_MODE_ENV: "require"}, "host=katib-postgres port=5432 user=katib password= dbname=katib sslmode=require"),
])
def test_postgres_dsn(monkeypatch, env, want):
    for k in (S.DB_USER_ENV, S.DB_PASSWORD_ENV, S.PG_HOST_ENV, S.PG_PORT_ENV, S.PG_DATABASE_ENV, S.PG_SSL_MODE_ENV):
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    assert S.postgres_dsn() == want


def test_time_encodings():
    t, ns = S.parse_rfc3339("2019-02-03T04:05:06+09:00")
    assert S.format_rfc3339_nano(t, ns) == "2019-02-02T19:05:06Z"
    assert S.MySQLDialect().to_db_time("2016-12-31T20:02:05.1Z") == "2016-12-31 20:02:05.1"
    assert S.MySQLDialect().from_db_time("2016-12-31 20:02:05") == "2016-12-31T20:02:05Z"
    with pytest.raises(ValueError, match="Error parsing start time"):
        S.insert_statement(S.MySQLDialect(), "t", [("yesterday", "m", "1")])


def test_rows_without_timestamp_are_skipped():
    sql, args = S.insert_statement(S.MySQLDialect(), "t", [("", "m", "1"), ("2016-12-31T20:02:05Z", "m", "2")])
    assert sql.endswith("VALUES (?, ?, ?, ?)") and args == ["t", "2016-12-31 20:02:05", "m", "2"]


def test_sqlite_end_to_end(tmp_path, monkeypatch):
    monkeypatch.setenv(S.SQLITE_PATH_ENV, str(tmp_path / "k.db"))
    monkeypatch.delenv(S.SKIP_DB_INIT_ENV, raising=False)
    db = S.new_observation_db("sqlite")
    db.select_one()
    db.report("t1", [("2021-01-01T00:00:02Z", "loss", "0.2"), ("2021-01-01T00:00:01.5Z", "loss", "0.5"),
                     ("2021-01-01T00:00:03+01:00", "acc", "0.9"), ("2021-01-01T00:00:10.000001Z", "loss", "0.1")])
    db.report("t2", [("2021-01-01T00:00:01Z", "loss", "9")])
    assert db.get("t1", "loss") == [("2021-01-01T00:00:01.5Z", "loss", "0.5"), ("2021-01-01T00:00:02Z", "loss", "0.2"),
                                    ("2021-01-01T00:00:10.000001Z", "loss", "0.1")]
    assert [r[1] for r in db.get("t1")] == ["acc", "loss", "loss", "loss"]  # 23:00:03 UTC of the previous day first
    assert db.get("t1", "loss", "2021-01-01T00:00:02Z", "2021-01-01T00:00:09Z") == [
        ("2021-01-01T00:00:02Z", "loss", "0.2")]
    db.remove("t1")
    assert db.get("t1") == [] and len(db.get("t2")) == 1
    db.close()
    db2 = S.new_observation_db("sqlite")  # persisted
    assert db2.get("t2") == [("2021-01-01T00:00:01Z", "loss", "9")]


def test_missing_driver_and_invalid_name():
    with pytest.raises(S.DBError, match="Invalid DB Name"):
        S.new_observation_db("oracle")
    try:
        import pymysql  # noqa: F401
    except ImportError:
        with pytest.raises(S.DBError, match="pymysql"):
            S.new_observation_db("mysql", connect_timeout=0)


def test_open_with_retry_times_out():
    clock = iter(range(100))
    calls = []

    def opener():
        calls.append(1)
        raise ConnectionRefusedError("no server")

    with pytest.raises(S.DBError, match="Timeout waiting for DB conn"):
        S.open_with_retry(opener, interval=5, timeout=3, sleep=lambda s: None, clock=lambda: next(clock))
    assert len(calls) >= 2


def test_db_manager_grpc_on_sqlite(tmp_path, monkeypatch):
    """main_test.go: Report / Get / Delete / Check through the gRPC facade."""
    import grpc

    from katib_amd.rpc import api_pb2 as api
    from katib_amd.rpc.client import DBManagerStub, HealthStub
    from katib_amd.rpc.server import make_server

    monkeypatch.setenv(S.SQLITE_PATH_ENV, str(tmp_path / "g.db"))
    db = S.new_observation_db("sqlite")
    srv = make_server("127.0.0.1:0", store=db)
    srv.start()
    try:
        with grpc.insecure_channel("127.0.0.1:%d" % srv.bound_port) as ch:
            stub = DBManagerStub(ch)
            logs = [api.MetricLog(time_stamp="2019-02-03T04:05:06+09:00", metric=api.Metric(name=n, value=v))
                    for n, v in (("f1_score", "88.95"), ("loss", "0.5"), ("precision", "88.7"), ("recall", "89.2"))]
            stub.ReportObservationLog(api.ReportObservationLogRequest(
                trial_name="test1-trial1", observation_log=api.ObservationLog(metric_logs=logs)), timeout=10)
            rep = stub.GetObservationLog(api.GetObservationLogRequest(
                trial_name="test1-trial1", start_time="2019-02-03T03:05:06+09:00", end_time="2019-02-03T05:05:06+09:00"),
                timeout=10)
            assert len(rep.observation_log.metric_logs) == 4
            stub.DeleteObservationLog(api.DeleteObservationLogRequest(trial_name="test1-trial1"), timeout=10)
            rep = stub.GetObservationLog(api.GetObservationLogRequest(trial_name="test1-trial1"), timeout=10)
            assert len(rep.observation_log.metric_logs) == 0
            h = HealthStub(ch)
            ok = h.Check(api.HealthCheckRequest(service="grpc.health.v1.Health"), timeout=10)
            assert ok.status == api.HealthCheckResponse.SERVING
            bad = h.Check(api.HealthCheckRequest(service="grpc.health.v1.1.Health"), timeout=10)
            assert bad.status != api.HealthCheckResponse.SERVING
            db.close()  # a dead database reports NOT_SERVING
            down = h.Check(api.HealthCheckRequest(service="grpc.health.v1.Health"), timeout=10)
            assert down.status == api.HealthCheckResponse.NOT_SERVING
    finally:
        srv.stop(0)
