"""SQL observation-log backends for the DBManager
(reference ``pkg/db/v1beta1/{mysql,postgres,common}`` and ``cmd/db-manager/v1beta1/main.go``).

The scheduler's own store is the native in-memory :class:`ObservationStore` (with
its append-only journal). These backends exist for deployments that keep metrics
in an external database shared with other tools: same schema, the same SQL text
and the same time encodings as the reference, so an existing Katib database can
be pointed at unchanged.

* ``mysql``   - ``?`` placeholders, ``DATETIME(6)`` stored as
  ``YYYY-MM-DD HH:MM:SS[.ffffff]`` (Go layout ``2006-01-02 15:04:05.999999``);
* ``postgres`` - ``$n`` placeholders, times stored as RFC 3339 (nano) text;
* ``sqlite``  - Python's built-in sqlite3 (single-node deployments, tests).

Backends expose the store interface the gRPC DBManager servicer uses
(``report / get / remove``) plus ``db_init`` and ``select_one``. Drivers for MySQL
and PostgreSQL (``pymysql``, ``psycopg2``) are optional and imported lazily: a
missing driver is reported when that backend is requested.
"""

from __future__ import annotations

import datetime as _dt
import os
import re
import sqlite3
import threading
import time
from typing import Callable, List, Optional, Sequence, Tuple

DB_USER_ENV, DB_NAME_ENV, DB_PASSWORD_ENV = "DB_USER", "DB_NAME", "DB_PASSWORD"
MYSQL_HOST_ENV, MYSQL_PORT_ENV, MYSQL_DATABASE_ENV = "KATIB_MYSQL_DB_HOST", "KATIB_MYSQL_DB_PORT", \
    "KATIB_MYSQL_DB_DATABASE"
PG_HOST_ENV, PG_PORT_ENV, PG_DATABASE_ENV, PG_SSL_MODE_ENV = "KATIB_POSTGRESQL_DB_HOST", "KATIB_POSTGRESQL_DB_PORT", \
    "KATIB_POSTGRESQL_DB_DATABASE", "KATIB_POSTGRESQL_SSL_MODE"
SKIP_DB_INIT_ENV = "SKIP_DB_INITIALIZATION"
SQLITE_PATH_ENV = "KATIB_SQLITE_DB_PATH"
CONNECT_INTERVAL_S = 5.0

CREATE_TABLE = {
    "mysql": """CREATE TABLE IF NOT EXISTS observation_logs
        (trial_name VARCHAR(255) NOT NULL,
        id INT AUTO_INCREMENT PRIMARY KEY,
        time DATETIME(6),
        metric_name VARCHAR(255) NOT NULL,
        value TEXT NOT NULL)""",
    "postgres": """CREATE TABLE IF NOT EXISTS observation_logs
        (trial_name VARCHAR(255) NOT NULL,
        id serial PRIMARY KEY,
        time TIMESTAMP(6),
        metric_name VARCHAR(255) NOT NULL,
        value TEXT NOT NULL)""",
    "sqlite": """CREATE TABLE IF NOT EXISTS observation_logs
        (trial_name VARCHAR(255) NOT NULL,
        id INTEGER PRIMARY KEY AUTOINCREMENT,
        time TEXT,
        metric_name VARCHAR(255) NOT NULL,
        value TEXT NOT NULL)""",
}
VALIDATE_TABLE = "SELECT trial_name, id, time, metric_name, value FROM observation_logs LIMIT 1"

_RFC3339 = re.compile(r"^(\d{4})-(\d{2})-(\d{2})[Tt ](\d{2}):(\d{2}):(\d{2})(?:\.(\d+))?(Z|z|[+-]\d{2}:\d{2})$")


class DBError(RuntimeError):
    pass


def parse_rfc3339(s: str) -> Tuple[_dt.datetime, int]:
    """time.Parse(time.RFC3339Nano): (UTC datetime at second resolution, nanoseconds)."""
    m = _RFC3339.match(s or "")
    if not m:
        raise ValueError("cannot parse %r as RFC3339" % s)
    y, mo, d, h, mi, se, frac, tz = m.groups()
    ns = int((frac or "").ljust(9, "0")[:9]) if frac else 0
    t = _dt.datetime(int(y), int(mo), int(d), int(h), int(mi), int(se), tzinfo=_dt.timezone.utc)
    if tz not in ("Z", "z"):
        sign = 1 if tz[0] == "+" else -1
        t -= sign * _dt.timedelta(hours=int(tz[1:3]), minutes=int(tz[4:6]))
    return t, ns


def _frac(ns: int, digits: int) -> str:
    """Go's .999... layout: up to ``digits`` fractional digits, trailing zeros dropped."""
    f = ("%09d" % ns)[:digits].rstrip("0")
    return "." + f if f else ""


def format_rfc3339_nano(t: _dt.datetime, ns: int) -> str:
    return t.strftime("%Y-%m-%dT%H:%M:%S") + _frac(ns, 9) + "Z"


def format_mysql_time(t: _dt.datetime, ns: int) -> str:
    return t.strftime("%Y-%m-%d %H:%M:%S") + _frac(ns, 6)


def parse_mysql_time(s) -> Tuple[_dt.datetime, int]:
    if isinstance(s, _dt.datetime):  # drivers may return datetime objects
        t = s if s.tzinfo else s.replace(tzinfo=_dt.timezone.utc)
        return t.replace(microsecond=0), s.microsecond * 1000
    m = re.match(r"^(\d{4}-\d{2}-\d{2} \d{2}:\d{2}:\d{2})(?:\.(\d{1,9}))?$", str(s))
    if not m:
        raise ValueError("cannot parse %r as a MySQL DATETIME" % s)
    t = _dt.datetime.strptime(m.group(1), "%Y-%m-%d %H:%M:%S").replace(tzinfo=_dt.timezone.utc)
    return t, int((m.group(2) or "").ljust(9, "0")) if m.group(2) else 0


class Dialect:
    name = ""
    fixed_width_time = False

    def placeholder(self, i: int) -> str:  # 1-based
        return "?"

    def to_db_time(self, ts: str) -> str:
        t, ns = parse_rfc3339(ts)
        return format_rfc3339_nano(t, ns)

    def from_db_time(self, v) -> str:
        if isinstance(v, _dt.datetime):
            t = v if v.tzinfo else v.replace(tzinfo=_dt.timezone.utc)
            return format_rfc3339_nano(t.astimezone(_dt.timezone.utc).replace(microsecond=0), v.microsecond * 1000)
        t, ns = parse_rfc3339(v)
        return format_rfc3339_nano(t, ns)


class MySQLDialect(Dialect):
    name = "mysql"

    def to_db_time(self, ts: str) -> str:
        t, ns = parse_rfc3339(ts)
        return format_mysql_time(t, ns)

    def from_db_time(self, v) -> str:
        t, ns = parse_mysql_time(v)
        return format_rfc3339_nano(t, ns)


class PostgresDialect(Dialect):
    name = "postgres"

    def placeholder(self, i: int) -> str:
        return "$%d" % i


class SQLiteDialect(Dialect):
    """Fixed-width microsecond text so that ``ORDER BY time`` and range filters compare
    chronologically as strings."""
    name = "sqlite"

    def to_db_time(self, ts: str) -> str:
        t, ns = parse_rfc3339(ts)
        return t.strftime("%Y-%m-%d %H:%M:%S") + ".%06d" % (ns // 1000)

    def from_db_time(self, v) -> str:
        t, ns = parse_mysql_time(v)
        return format_rfc3339_nano(t, ns)


DIALECTS = {"mysql": MySQLDialect, "postgres": PostgresDialect, "sqlite": SQLiteDialect}


def insert_statement(dialect: Dialect, trial: str, logs: Sequence[Tuple[str, str, str]]) -> Tuple[str, list]:
    """RegisterObservationLog's multi-row INSERT (mysql.go:67-102, postgres.go:69-109);
    rows without a timestamp are skipped."""
    sql = "INSERT INTO observation_logs (trial_name, time, metric_name, value) VALUES "
    vals: list = []
    groups = []
    i = 1
    for ts, name, value in logs:
        if not ts:
            continue
        try:
            t = dialect.to_db_time(ts)
        except ValueError as e:
            raise ValueError("Error parsing start time %s: %s" % (ts, e))
        groups.append("(%s, %s, %s, %s)" % tuple(dialect.placeholder(i + k) for k in range(4)))
        vals += [trial, t, name, value]
        i += 4
    return sql + ",".join(groups), vals


def select_statement(dialect: Dialect, trial: str, metric: str = "", start: str = "",
                     end: str = "") -> Tuple[str, list]:
    """GetObservationLog's filtered SELECT (mysql.go:109-135, postgres.go:111-146)."""
    args = [trial]
    q = "SELECT time, metric_name, value FROM observation_logs WHERE trial_name = %s" % dialect.placeholder(1)
    if metric:
        args.append(metric)
        q += " AND metric_name = %s" % dialect.placeholder(len(args))
    for ts, op, what in ((start, ">=", "start"), (end, "<=", "completion")):
        if ts:
            try:
                args.append(dialect.to_db_time(ts))
            except ValueError as e:
                raise ValueError("Error parsing %s time %s: %s" % (what, ts, e))
            q += " AND time %s %s" % (op, dialect.placeholder(len(args)))
    return q + " ORDER BY time", args


def delete_statement(dialect: Dialect, trial: str) -> Tuple[str, list]:
    return "DELETE FROM observation_logs WHERE trial_name = %s" % dialect.placeholder(1), [trial]


class SQLObservationDB:
    """KatibDBInterface (pkg/db/v1beta1/common/kdb.go) over a DB-API 2.0 connection."""

    def __init__(self, conn, dialect: Dialect):
        self.conn = conn
        self.dialect = dialect
        self._lock = threading.Lock()  # DB-API connections are not shared across threads safely

    def _exec(self, sql: str, args: Sequence = ()):
        with self._lock:
            cur = self.conn.cursor()
            try:
                cur.execute(sql, tuple(args))
                rows = cur.fetchall() if cur.description else []
            finally:
                cur.close()
            commit = getattr(self.conn, "commit", None)
            if commit is not None:
                commit()
            return rows

    def db_init(self):
        if os.environ.get(SKIP_DB_INIT_ENV, "false") == "false":
            self._exec(CREATE_TABLE[self.dialect.name])
        else:
            self._exec(VALIDATE_TABLE)

    def select_one(self):
        try:
            self._exec("SELECT 1")
        except Exception as e:
            raise DBError("Error `SELECT 1` probing: %s" % e)

    # store interface used by the DBManager servicer and the scheduler -------------
    def report(self, trial: str, logs: Sequence[Tuple[str, str, str]]):
        sql, args = insert_statement(self.dialect, trial, logs)
        if not args:
            return
        try:
            self._exec(sql, args)
        except ValueError:
            raise
        except Exception as e:
            raise DBError("Execute SQL INSERT failed: %s" % e)

    def get(self, trial: str, metric: str = "", start: str = "", end: str = "") -> List[Tuple[str, str, str]]:
        sql, args = select_statement(self.dialect, trial, metric, start, end)
        try:
            rows = self._exec(sql, args)
        except Exception as e:
            raise DBError("Failed to get ObservationLogs %s" % e)
        out = []
        for t, name, value in rows:
            try:
                out.append((self.dialect.from_db_time(t), name, value))
            except ValueError:
                continue  # the reference logs and skips unparsable rows
        return out

    def remove(self, trial: str):
        sql, args = delete_statement(self.dialect, trial)
        self._exec(sql, args)

    def close(self):
        self.conn.close()


class _QmarkCursor:
    """Adapts ``?``/``$n`` SQL to drivers whose paramstyle is ``%s`` (pymysql, psycopg2)."""

    def __init__(self, cur):
        self.cur = cur

    @property
    def description(self):
        return self.cur.description

    def execute(self, sql, args=()):
        return self.cur.execute(re.sub(r"\?|\$\d+", "%s", sql), args)

    def fetchall(self):
        return self.cur.fetchall()

    def close(self):
        self.cur.close()


class _FormatParamConn:
    def __init__(self, conn):
        self.conn = conn

    def cursor(self):
        return _QmarkCursor(self.conn.cursor())

    def commit(self):
        self.conn.commit()

    def close(self):
        self.conn.close()


def mysql_dsn() -> str:
    """getDbName (mysql.go:44-57)."""
    e = os.environ.get
    return "%s:%s@tcp(%s:%s)/%s?timeout=5s" % (e(DB_USER_ENV, "root"), e(DB_PASSWORD_ENV, ""),
                                               e(MYSQL_HOST_ENV, "katib-mysql"), e(MYSQL_PORT_ENV, "3306"),
                                               e(MYSQL_DATABASE_ENV, "katib"))


def postgres_dsn() -> str:
    """getDbName (postgres.go:39-59)."""
    e = os.environ.get
    return "host=%s port=%s user=%s password=%s dbname=%s sslmode=%s" % (
        e(PG_HOST_ENV, "katib-postgres"), e(PG_PORT_ENV, "5432"), e(DB_USER_ENV, "katib"), e(DB_PASSWORD_ENV, ""),
        e(PG_DATABASE_ENV, "katib"), e(PG_SSL_MODE_ENV, "disable"))


def _open_mysql():
    try:
        import pymysql
    except ImportError:
        raise DBError("DB_NAME=mysql needs the 'pymysql' driver, which is not installed")
    e = os.environ.get
    return _FormatParamConn(pymysql.connect(host=e(MYSQL_HOST_ENV, "katib-mysql"),
                                            port=int(e(MYSQL_PORT_ENV, "3306")), user=e(DB_USER_ENV, "root"),
                                            password=e(DB_PASSWORD_ENV, ""), database=e(MYSQL_DATABASE_ENV, "katib"),
                                            connect_timeout=5))


def _open_postgres():
    try:
        import psycopg2
    except ImportError:
        raise DBError("DB_NAME=postgres needs the 'psycopg2' driver, which is not installed")
    return _FormatParamConn(psycopg2.connect(postgres_dsn()))


def _open_sqlite():
    path = os.environ.get(SQLITE_PATH_ENV, "katib.db")
    return sqlite3.connect(path, check_same_thread=False)


def open_with_retry(opener: Callable, interval: float = CONNECT_INTERVAL_S, timeout: float = 60.0,
                    sleep: Callable[[float], None] = time.sleep, clock: Callable[[], float] = time.monotonic):
    """OpenSQLConn (common/connection.go:27-48): try every ``interval`` seconds until
    ``timeout``; a missing driver fails at once."""
    deadline = clock() + timeout
    last = None
    while True:
        sleep(interval)
        try:
            conn = opener()
            cur = conn.cursor()
            cur.execute("SELECT 1")
            cur.close()
            return conn
        except DBError:
            raise
        except Exception as e:  # connection refused, auth, ... -> retry
            last = e
        if clock() >= deadline:
            raise DBError("Timeout waiting for DB conn successfully opened. (last error: %s)" % last)


def new_observation_db(db_name: Optional[str] = None, connect_timeout: float = 60.0, interval: float = 0.0):
    """NewKatibDBInterface (pkg/db/v1beta1/db.go): ``mysql``, ``postgres`` or ``sqlite``;
    ``native`` (or empty) returns the in-memory native store."""
    name = (db_name if db_name is not None else os.environ.get(DB_NAME_ENV, "")).lower()
    if name in ("", "native"):
        from .. import native

        return native.load().ObservationStore()
    openers = {"mysql": _open_mysql, "postgres": _open_postgres, "sqlite": _open_sqlite}
    if name not in openers:
        raise DBError("Invalid DB Name: %s" % name)
    conn = open_with_retry(openers[name], interval=interval if name == "sqlite" else CONNECT_INTERVAL_S,
                           timeout=connect_timeout)
    db = SQLObservationDB(conn, DIALECTS[name]())
    db.db_init()
    return db
