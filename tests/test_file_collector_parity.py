"""Port of TestCollectObservationLog (reference
``pkg/metricscollector/v1beta1/file-metricscollector/file-metricscollector_test.go``):
same file bodies, filters and expected observation logs, run through the native
:class:`MetricsParser` via :func:`collect_observation_log`."""
import pytest

from katib_amd.metricscollector.file_collector import CollectError, collect_observation_log

Z = "0001-01-01T00:00:00Z"
FILTER = r"{metricName: ([\w|-]+), metricValue: ((-?\d+)(\.\d+)?)}"
UNAVAILABLE = "unavailable"

CASES = {
    "Positive case for logs in JSON format": dict(
        file="good.json",
        data='{"checkpoint_path": "", "global_step": "0", "loss": "0.22082142531871796", "timestamp": 1638422847.28721, "trial": "0"}\n'  # noqa: E501
             '{"acc": "0.9349666833877563", "checkpoint_path": "", "global_step": "0", "timestamp": 1638422847.287801, "trial": "0"}\n'  # noqa: E501
             '{"checkpoint_path": "", "global_step": "1", "loss": "0.1414974331855774", "timestamp": "2021-12-02T14:27:50.000035161Z", "trial": "0"}\n'  # noqa: E501
             '{"acc": "0.9586416482925415", "checkpoint_path": "", "global_step": "1", "timestamp": "2021-12-02T14:27:50.000037459Z", "trial": "0"}\n'  # noqa: E501
             '{"checkpoint_path": "", "global_step": "2", "loss": "0.10683439671993256", "trial": "0"}',
        metrics=["acc", "loss"], fmt="JSON",
        want=[("2021-12-02T05:27:27.000028721Z", "loss", "0.22082142531871796"),
              ("2021-12-02T05:27:27.000287801Z", "acc", "0.9349666833877563"),
              ("2021-12-02T14:27:50.000035161Z", "loss", "0.1414974331855774"),
              ("2021-12-02T14:27:50.000037459Z", "acc", "0.9586416482925415"),
              (Z, "loss", "0.10683439671993256")]),
    "Positive case for logs in TEXT format": dict(
        file="good.log",
        data="2024-03-04T17:55:08Z INFO     {metricName: accuracy, metricValue: 0.8078};{metricName: loss, metricValue: 0.5183}\n"  # noqa: E501
             "2024-03-04T17:55:08Z INFO     {metricName: accuracy, metricValue: 0.6752}\n"
             "2024-03-04T17:55:08Z INFO     {metricName: loss, metricValue: 0.3634}\n"
             "2024-03-04T17:55:08Z INFO     {metricName: accuracy, metricValue: 100}\n"
             "2024-03-04T17:55:08Z INFO     {metricName: accuracy, metricValue: 888.333}\n"
             "2024-03-04T17:55:08Z INFO     {metricName: accuracy, metricValue: -0.4759}\n"
             "{metricName: loss, metricValue: 0.8671}",
        metrics=["accuracy", "loss"], filters=[FILTER], fmt="TEXT",
        want=[("2024-03-04T17:55:08Z", "accuracy", "0.8078"), ("2024-03-04T17:55:08Z", "loss", "0.5183"),
              ("2024-03-04T17:55:08Z", "accuracy", "0.6752"), ("2024-03-04T17:55:08Z", "loss", "0.3634"),
              ("2024-03-04T17:55:08Z", "accuracy", "100"), ("2024-03-04T17:55:08Z", "accuracy", "888.333"),
              ("2024-03-04T17:55:08Z", "accuracy", "-0.4759"), (Z, "loss", "0.8671")]),
    "Invalid case for logs in TEXT format": dict(
        file="invalid-value.log",
        data="2024-03-04T17:55:08Z INFO     {metricName: accuracy, metricValue: .333}\n"
             "2024-03-04T17:55:08Z INFO     {metricName: accuracy, metricValue: -.333}\n"
             "2024-03-04T17:55:08Z INFO     {metricName: accuracy, metricValue: - 345.333}\n"
             "2024-03-04T17:55:08Z INFO     {metricName: accuracy, metricValue: 888.}",
        metrics=["accuracy", "loss"], filters=[FILTER], fmt="TEXT",
        want=[(Z, "accuracy", UNAVAILABLE)]),
    "Invalid file name": dict(file="invalid", fmt="JSON", error="failed to open file"),
    "Invalid file format": dict(file="good.log", data="x=1", fmt="invalid", error="format must be set"),
    "Invalid formatted file for logs in JSON format": dict(
        file="invalid-format.json",
        data='"checkpoint_path": "", "global_step": "0", "loss": "0.22082142531871796", "timestamp": 1638422847.28721, "trial": "0"\n'  # noqa: E501
             '{"acc": "0.9349666833877563", "checkpoint_path": "", "global_step": "0", "timestamp": 1638422847.287801, "trial": "0',  # noqa: E501
        fmt="JSON", error="failed to parse JSON"),
    "Invalid formatted file for logs in TEXT format": dict(
        file="invalid-format.log",
        data="2024-03-04T17:55:08Z INFO     {metricName: accuracy, metricValue: 0.6752\n"
             "2024-03-04T17:55:08Z INFO     {metricName: loss, metricValue: 0.3634}",
        metrics=["accuracy", "loss"], filters=[FILTER], fmt="TEXT",
        want=[(Z, "accuracy", UNAVAILABLE)]),
    "Invalid timestamp for logs in JSON format": dict(
        file="invalid-timestamp.json",
        data='{"checkpoint_path": "", "global_step": "0", "loss": "0.22082142531871796", "timestamp": "invalid", "trial": "0"}\n'  # noqa: E501
             '{"acc": "0.9349666833877563", "checkpoint_path": "", "global_step": "0", "timestamp": 1638422847, "trial": "0"}',  # noqa: E501
        metrics=["acc", "loss"], fmt="JSON",
        want=[(Z, "loss", "0.22082142531871796"), ("2021-12-02T05:27:27Z", "acc", "0.9349666833877563")]),
    "Invalid timestamp for logs in TEXT format": dict(
        file="invalid-timestamp.log",
        data="2024-03-04T17:55:08Z INFO     {metricName: accuracy, metricValue: 0.6752}\n"
             "invalid INFO     {metricName: loss, metricValue: 0.3634}",
        metrics=["accuracy", "loss"], filters=[FILTER], fmt="TEXT",
        want=[("2024-03-04T17:55:08Z", "accuracy", "0.6752"), (Z, "loss", "0.3634")]),
    "Missing objective metric in JSON training logs": dict(
        file="missing-objective-metric.json",
        data='{"checkpoint_path": "", "global_step": "0", "loss": "0.22082142531871796", "timestamp": 1638422847.28721, "trial": "0"}\n'  # noqa: E501
             '{"checkpoint_path": "", "global_step": "1", "loss": "0.1414974331855774", "timestamp": "2021-12-02T14:27:50.000035161+09:00", "trial": "0"}\n'  # noqa: E501
             '{"checkpoint_path": "", "global_step": "2", "loss": "0.10683439671993256", "trial": "0"}',
        metrics=["acc", "loss"], fmt="JSON",
        want=[(Z, "acc", UNAVAILABLE)]),
    "Missing objective metric in TEXT training logs": dict(
        file="missing-objective-metric.log",
        data="2024-03-04T17:55:08Z INFO     {metricName: loss, metricValue: 0.3634}\n"
             "2024-03-04T17:55:08Z INFO     {metricName: loss, metricValue: 0.8671}",
        metrics=["accuracy", "loss"], fmt="TEXT",
        want=[(Z, "accuracy", UNAVAILABLE)]),
}


@pytest.mark.parametrize("name", list(CASES))
def test_collect_observation_log(name, tmp_path):
    c = CASES[name]
    if c.get("data") is not None:
        (tmp_path / c["file"]).write_text(c["data"])
    args = (str(tmp_path / c["file"]), c.get("metrics", []), c.get("filters", []), c["fmt"])
    if "error" in c:
        with pytest.raises(CollectError, match=c["error"]):
            collect_observation_log(*args)
    else:
        assert [tuple(r) for r in collect_observation_log(*args)] == c["want"]
