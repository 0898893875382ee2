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
