"""Native runtime: metrics parser (reference file-metricscollector semantics), observation
store (db-manager semantics), samplers."""
import os
import re

import numpy as np
import pytest

from katib_amd import native

N = native.load()
DEFAULT = r"([\w|-]+)\s*=\s*([+-]?\d*(\.\d+)?([Ee][+-]?\d+)?)"


@pytest.mark.parametrize("line", [
    "loss=0.3", "accuracy=.98", "Score=-7.53e-05", "Score=-7.53e+05", "Score=1E0", "Score=1.23E10",
    "epoch 1: loss = 0.25, accuracy=0.91 lr=1e-3", "a|b-c=5e+", "x==3", "name=abc val=1.5.6",
    "  spaced  =  42  ", "a=1b=2", "-=3", "|=|4", "weird=1e", "k=+.5e-3x",
])
def test_default_filter_matches_regex_semantics(line):
    # Python's re has the same leftmost-first semantics as RE2 for this pattern
    want = [(m.group(1), m.group(2)) for m in re.finditer(DEFAULT, line)]
    assert N.default_filter_scan(line) == want


def test_text_parse_timestamp_and_filtering():
    p = N.MetricsParser(["loss", "accuracy"], [], 0)
    assert p.parse_line("2021-01-01T00:00:00.5Z loss=0.3, accuracy=0.9") == [
        ("2021-01-01T00:00:00.5Z", "loss", "0.3"), ("2021-01-01T00:00:00.5Z", "accuracy", "0.9")]
    assert p.parse_line("no metrics here") == []
    assert p.parse_line("val_loss=3") == []  # name must equal a metric exactly
    z = "0001-01-01T00:00:00Z"
    assert p.parse_line("loss=0.1") == [(z, "loss", "0.1")]


def test_custom_filter():
    p = N.MetricsParser(["Best-Genotype"], [r"([\w-]+)=(Genotype.*)"], 0)
    out = p.parse_line("Best-Genotype=Genotype(normal=[[('a',0)]],normal_concat=range(2,5))")
    assert out[0][1] == "Best-Genotype" and out[0][2].startswith("Genotype(")


def test_unavailable_when_objective_missing():
    p = N.MetricsParser(["acc", "loss"], [], 0)
    assert p.parse_content("loss=0.1\nloss=0.2\n") == [("0001-01-01T00:00:00Z", "acc", "unavailable")]


def test_json_format():
    p = N.MetricsParser(["loss", "acc"], [], 1)
    # only string values are taken (file-metricscollector.go:162), float timestamps quirk
    out = p.parse_line('{"loss": "0.5", "acc": 0.9, "timestamp": 1614066000.5}')
    assert out == [("2021-02-23T07:40:00.000000005Z", "loss", "0.5")]
    out = p.parse_line('{"loss": "0.4", "timestamp": "2021-02-23T07:40:00Z"}')
    assert out == [("2021-02-23T07:40:00Z", "loss", "0.4")]
    with pytest.raises(ValueError):
        p.parse_line("{not json")


def test_rule_values():
    p = N.MetricsParser(["loss"], [], 0)
    assert p.rule_values("loss=0.5 acc=1", ["loss", "acc"]) == [("loss", 0.5), ("acc", 1.0)]
    assert p.rule_values("nothing", ["loss"]) == []


def test_store_semantics(tmp_path):
    s = N.ObservationStore()
    s.report("t1", [("2021-01-01T00:00:02Z", "loss", "0.2"), ("2021-01-01T00:00:01Z", "loss", "0.5"),
                    ("2021-01-01T00:00:03Z", "loss", "0.3"), ("2021-01-01T00:00:03Z", "acc", "x"),
                    ("", "skipped", "1")])
    rows = s.get("t1")
    assert [r[2] for r in rows] == ["0.5", "0.2", "0.3", "x"]
    assert s.get("t1", "loss", "2021-01-01T00:00:02Z", "") == [("2021-01-01T00:00:02Z", "loss", "0.2"),
                                                                ("2021-01-01T00:00:03Z", "loss", "0.3")]
    assert s.get("t1", "loss", "", "2021-01-01T00:00:01Z") == [("2021-01-01T00:00:01Z", "loss", "0.5")]
    assert s.get("missing") == []
    # getMetrics: min/max/latest; the reference "else if" means one value updates min OR max
    red = dict((r[0], r[1:]) for r in s.reduce("t1", ["loss", "acc", "none"]))
    assert red["loss"] == ("0.2", "0.5", "0.3")
    assert red["acc"] == ("unavailable", "unavailable", "x")
    assert red["none"] == ("unavailable",) * 3
    with pytest.raises(ValueError):
        s.report("t2", [("yesterday", "loss", "1")])
    s.remove("t1")
    assert s.size("t1") == 0


def test_store_reduce_else_if_quirk():
    s = N.ObservationStore()
    s.report("t", [("2021-01-01T00:00:01Z", "m", "5"), ("2021-01-01T00:00:02Z", "m", "3"),
                   ("2021-01-01T00:00:03Z", "m", "9")])
    (name, mn, mx, lt), = s.reduce("t", ["m"])
    assert (mn, mx, lt) == ("3", "9", "9")


def test_store_journal(tmp_path):
    path = str(tmp_path / "j.jsonl")
    s = N.ObservationStore()
    s.open_journal(path)
    s.report("a", [("2021-01-01T00:00:01Z", "m", "1")])
    s.report("b", [("2021-01-01T00:00:01Z", "m", "2")])
    s.remove("a")
    s.close_journal()
    s2 = N.ObservationStore()
    s2.load_journal(path)
    assert s2.trials() == ["b"] and s2.get("b")[0][2] == "2"


def test_rfc3339():
    assert N.parse_rfc3339("2021-01-01T00:00:00Z") == (1609459200, 0)
    assert N.parse_rfc3339("2021-01-01T01:00:00+01:00") == (1609459200, 0)
    assert N.parse_rfc3339("2021-02-30T00:00:00Z") is None
    assert N.format_rfc3339_nano(1609459200, 500000000) == "2021-01-01T00:00:00.5Z"


def test_sobol_matches_scipy():
    from scipy.stats import qmc

    from katib_amd.algorithms.samplers import sobol_table

    poly, vinit = sobol_table()
    e = N.SobolEngine(7, poly[:7].tolist(), vinit[:7].tolist())
    a = np.array(e.points(0, 256))
    b = qmc.Sobol(7, scramble=False).random(256)
    assert np.abs(a - b).max() == 0.0


def test_cmaes_converges():
    c = N.CmaEs([0.5, 0.5, 0.5], 0.3, [0, 0, 0], [1, 1, 1], 7, 0)
    for _ in range(60):
        xs = [c.ask() for _ in range(c.popsize)]
        c.tell(xs, [sum((x[i] - t) ** 2 for i, t in enumerate((0.2, 0.7, 0.4))) for x in xs])
    assert np.allclose(c.mean, [0.2, 0.7, 0.4], atol=1e-3)
    with pytest.raises(ValueError):
        c.tell([[0.1, 0.1, 0.1]], [1.0])


def test_tpe_prefers_good_region():
    rng = np.random.RandomState(0)
    xs = rng.uniform(0, 1, (60, 1)).tolist()
    losses = [abs(x[0] - 0.8) for x in xs]
    picks = [N.tpe_sample([{"kind": 0, "low": 0, "high": 1}], xs, losses, {}, s)[0] for s in range(20)]
    assert abs(np.median(picks) - 0.8) < 0.15
    pm = [N.tpe_sample([{"kind": 0, "low": 0, "high": 1}], xs, losses, {"multivariate": True,
                                                                         "gamma_mode": 1, "gamma": 0.1}, s)[0]
          for s in range(20)]
    assert abs(np.median(pm) - 0.8) < 0.2


def test_slot_pool():
    p = N.SlotPool(4, 1)
    a = p.acquire(2)
    b = p.acquire(2)
    assert sorted(a + b) == [0, 1, 2, 3] and p.acquire(1) == []
    p.release(a)
    assert p.free_slots() == 2
    p.record_fault(0, 1)
    assert p.quarantined() == [0] and p.capacity() == 3


def test_template_render():
    assert N.render_template("x=${trialParameters.lr} y=${trialParameters.lr}", {"lr": "0.1"}) == "x=0.1 y=0.1"
    assert N.unresolved_placeholders("${trialParameters.a} and ${trialParameters.b}") == [
        "${trialParameters.a}", "${trialParameters.b}"]


@pytest.mark.parametrize("re2,ecma,icase", [
    (r"{metricName: ([\w|-]+), metricValue: ((-?\d+)(\.\d+)?)}",
     r"\{metricName: ([\w|-]+), metricValue: ((-?\d+)(\.\d+)?)\}", False),
    (r"(?P<name>\w+)=(\d+)", r"(\w+)=(\d+)", False),
    (r"a{2,3}b{4}c{5,}", r"a{2,3}b{4}c{5,}", False),
    (r"x{a}", r"x\{a\}", False),
    (r"(?i)loss=(\d)", r"loss=(\d)", True),
    (r"[]a](x)", r"[\]a](x)", False),
    (r"\Qa.b\E(\d)", r"a\.b(\d)", False),
    (r"\A(\w+)=(\d)\z", r"^(\w+)=(\d)$", False),
])
def test_re2_filter_translation(re2, ecma, icase):
    """Go RE2 filter syntax the reference accepts (literal braces, named groups, \\Q..\\E)."""
    assert N.re2_to_ecmascript(re2) == (ecma, icase)


def test_brace_filter_parses():
    p = N.MetricsParser(["accuracy"], [r"{metricName: ([\w|-]+), metricValue: ((-?\d+)(\.\d+)?)}"], 0)
    assert p.parse_line("{metricName: accuracy, metricValue: 0.5}") == [("0001-01-01T00:00:00Z", "accuracy", "0.5")]
