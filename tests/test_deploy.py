"""Node installs (``katib-amd install``, the analog of the reference's
``manifests/v1beta1/installs/*``): every profile renders a katib-config.yaml the scheduler
loads, an env file with the backend's DB variables, and systemd units whose ExecStart lines
are valid katib-amd command lines."""
import shlex

import pytest

from katib_amd import cli
from katib_amd.algorithms.registry import DEFAULT_SUGGESTIONS
from katib_amd.controller.config import KatibConfig
from katib_amd.deploy import PROFILES, render


def _exec_args(unit_text):
    line = [ln for ln in unit_text.splitlines() if ln.startswith("ExecStart=")][0]
    argv = shlex.split(line[len("ExecStart="):])
    i = argv.index("katib_amd")
    return argv[i + 1:]


@pytest.mark.parametrize("profile", PROFILES)
def test_profile_renders_loadable_config_and_valid_units(tmp_path, profile):
    files = render(profile, str(tmp_path), python="/usr/bin/python3", gpus=8, slots_per_gpu=2)
    cfg = KatibConfig.load(str(tmp_path / "katib-config.yaml"))
    assert cfg.amd.num_devices == 8 and cfg.amd.slots_per_device == 2
    assert set(DEFAULT_SUGGESTIONS) <= set(cfg.suggestions)
    assert "medianstop" in cfg.early_stoppings and "PrometheusMetric" in cfg.metrics_collectors
    env = dict(ln.split("=", 1) for ln in (tmp_path / "katib-amd.env").read_text().splitlines())
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    if profile in ("mysql", "postgres"):
        assert env["DB_NAME"] == profile
    parser = cli.build_parser()
    units = sorted(f for f in files if f.endswith(".service"))
    assert "katib-amd.service" in units
    for u in units:
        args = [a.replace("%i", "tpe") for a in _exec_args(files[u])]
        ns = parser.parse_args(args)  # a valid command line of this CLI
        if ns.cmd == "serve":
            assert ns.config == str(tmp_path / "katib-config.yaml") and ns.gpus == 8
            assert bool(ns.grpc) == (profile == "standalone")
        if ns.cmd == "db-manager" and profile in ("mysql", "postgres"):
            assert ns.db == profile
    install = (tmp_path / "install.sh").read_text()
    assert "systemctl enable --now" in install and "katib-amd.service" in install


def test_cli_install_and_unknown_profile(tmp_path, capsys):
    assert cli.main(["install", "--profile", "services", "--prefix", str(tmp_path / "svc")]) == 0
    out = capsys.readouterr().out
    assert "katib-amd-suggestion@.service" in out
    with pytest.raises(ValueError):
        render("kubernetes", str(tmp_path / "x"))


def _binds(files):
    out = []
    for u in sorted(f for f in files if f.endswith(".service")):
        a = _exec_args(files[u])
        for flag in ("--address", "--grpc"):
            if flag in a:
                out.append(a[a.index(flag) + 1])
    return out


@pytest.mark.parametrize("profile", PROFILES)
def test_default_install_binds_loopback_and_hides_secrets(tmp_path, profile):
    """the rendered services listen on loopback only; the env file (DB password)
    is 0600 and install.sh chowns it to the service user."""
    import os
    import stat

    files = render(profile, str(tmp_path), python="/usr/bin/python3")
    for b in _binds(files):
        assert b.startswith("127.0.0.1") or b.startswith("unix:"), (profile, b)
    assert stat.S_IMODE(os.stat(tmp_path / "katib-amd.env").st_mode) == 0o600
    assert "chmod 0600" in files["install.sh"] and "katib-amd.env" in files["install.sh"]
    assert "api-token" not in files


def test_non_loopback_install_requires_token(tmp_path):
    import os
    import stat

    files = render("standalone", str(tmp_path), python="/usr/bin/python3", listen="0.0.0.0")
    a = _exec_args(files["katib-amd.service"])
    assert a[a.index("--address") + 1] == "0.0.0.0"
    tok = a[a.index("--token-file") + 1]
    assert os.path.basename(tok) == "api-token" and len((tmp_path / "api-token").read_text().strip()) == 64
    assert stat.S_IMODE(os.stat(tmp_path / "api-token").st_mode) == 0o600


def test_serve_refuses_open_bind_without_token(tmp_path, capsys):
    rc = cli.main(["serve", "--address", "0.0.0.0", "--port", "0", "--state-dir", str(tmp_path)])
    assert rc == 2 and "refusing to listen" in capsys.readouterr().err


def test_api_token_enforced(tmp_path):
    import json
    import urllib.error
    import urllib.request

    from katib_amd.controller.apiserver import ApiServer
    from katib_amd.controller.manager import Manager
    from katib_amd.sdk.remote import RemoteManager

    m = Manager(state_dir=str(tmp_path), num_devices=0, journal=False)
    api = ApiServer(m, "127.0.0.1", 0, token="s3cret").start()
    try:
        base = "http://127.0.0.1:%d" % api.port
        assert urllib.request.urlopen(base + "/healthz").read() == b"ok"  # probes stay open
        with pytest.raises(urllib.error.HTTPError) as ei:
            urllib.request.urlopen(base + "/apis/kubeflow.org/v1beta1/namespaces/default/experiments")
        assert ei.value.code == 401
        r = RemoteManager(base, token="s3cret")
        assert r.list_experiments("default") == []
        with pytest.raises(Exception):
            RemoteManager(base, token="wrong").list_experiments("default")
    finally:
        api.stop()
        m.shutdown()


def test_grpc_stays_loopback_and_empty_address_is_exposed(tmp_path, capsys):
    """the bearer token protects only the HTTP API, so a non-loopback install keeps the
    gRPC services on loopback, ``serve --grpc`` / the standalone gRPC servers refuse a
    non-loopback bind without --insecure-grpc, and ``--address ''`` (every interface) counts as
    exposed."""
    files = render("services", str(tmp_path), python="/usr/bin/python3", listen="0.0.0.0")
    binds = _binds({k: v for k, v in files.items() if k != "katib-amd.service"})
    assert binds and all(b.startswith("127.0.0.1") or b.startswith("unix:") for b in binds), binds
    rc = cli.main(["serve", "--address", "", "--port", "0", "--state-dir", str(tmp_path)])
    assert rc == 2 and "refusing to listen" in capsys.readouterr().err
    tok = tmp_path / "tok"
    tok.write_text("abc\n")
    rc = cli.main(["serve", "--address", "127.0.0.1", "--port", "0", "--state-dir", str(tmp_path),
                   "--token-file", str(tok), "--grpc", "0.0.0.0:0"])
    assert rc == 2 and "unauthenticated" in capsys.readouterr().err
    for argv in (["db-manager", "--address", "0.0.0.0:0"], ["suggestion-server", "--algorithm", "random",
                                                            "--address", "10.1.2.3:0"],
                 ["earlystopping-server", "--address", "[::]:0"]):
        assert cli.main(argv) == 2, argv
        assert "unauthenticated" in capsys.readouterr().err


def test_ui_token_cookie(tmp_path):
    """The browser UI cannot send a bearer header: ``/?token=<token>`` sets an HttpOnly cookie that
    authorises the later UI requests; a wrong token gets 401."""
    import urllib.error
    import urllib.request

    from katib_amd.controller.apiserver import ApiServer
    from katib_amd.controller.manager import Manager

    m = Manager(state_dir=str(tmp_path), num_devices=0, journal=False)
    api = ApiServer(m, "127.0.0.1", 0, token="s3cret").start()
    try:
        base = "http://127.0.0.1:%d" % api.port
        with pytest.raises(urllib.error.HTTPError) as ei:
            urllib.request.urlopen(base + "/katib/fetch_experiments?namespace=default")
        assert ei.value.code == 401
        with pytest.raises(urllib.error.HTTPError):
            urllib.request.urlopen(base + "/?token=wrong")
        import http.client

        # the token query is answered with a 303 to "/" that sets the cookie (the token
        # leaves the URL at once) and no-referrer; elsewhere it is refused
        conn = http.client.HTTPConnection("127.0.0.1", api.port)
        conn.request("GET", "/?token=s3cret")
        r = conn.getresponse()
        r.read()
        assert r.status == 303 and r.headers["Location"] == "/"
        assert r.headers["Referrer-Policy"] == "no-referrer"
        cookie = r.headers["Set-Cookie"]
        assert cookie.startswith("katib_amd_token=s3cret") and "HttpOnly" in cookie
        conn.request("GET", "/katib/fetch_experiments?namespace=default&token=s3cret")
        r = conn.getresponse()
        r.read()
        assert r.status == 401
        conn.close()
        req = urllib.request.Request(base + "/katib/fetch_experiments?namespace=default",
                                     headers={"Cookie": cookie.split(";")[0]})
        assert urllib.request.urlopen(req).status == 200
    finally:
        api.stop()
        m.shutdown()
