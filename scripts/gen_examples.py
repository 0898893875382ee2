#!/usr/bin/env python3
"""Regenerates the CPU example catalogue (examples/{hp-tuning,early-stopping,metrics-collector,
resume-experiment,trial-template}) that mirrors the reference examples/v1beta1 set."""
import os, yaml
R = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples")
QUAD = "a=${trialParameters.a}; b=${trialParameters.b}; print('result=%s' % (4*a - b*b))"
PARAMS = [{"name": "a", "parameterType": "double", "feasibleSpace": {"min": "0", "max": "2"}},
          {"name": "b", "parameterType": "double", "feasibleSpace": {"min": "-1", "max": "1"}}]

def exp(name, algo, settings=None, params=None, command=None, parallel=3, max_trials=12, extra=None,
        objective=None, tp=None, metadata_env=None):
    params = params or PARAMS
    names = [p["name"] for p in params]
    container = {"name": "training-container", "image": "python:3.10",
                 "command": command or ["python3", "-c", QUAD]}
    if metadata_env:
        container["env"] = metadata_env
    spec = {
        "objective": objective or {"type": "maximize", "goal": 7.99, "objectiveMetricName": "result"},
        "algorithm": {"algorithmName": algo, **({"algorithmSettings": settings} if settings else {})},
        "parallelTrialCount": parallel, "maxTrialCount": max_trials, "maxFailedTrialCount": 3,
        "parameters": params,
        "trialTemplate": {
            "primaryContainerName": "training-container",
            "trialParameters": tp or [{"name": n, "reference": n} for n in names],
            "trialSpec": {"apiVersion": "batch/v1", "kind": "Job",
                          "spec": {"template": {"spec": {"containers": [container], "restartPolicy": "Never"}}}},
        },
    }
    if extra:
        spec.update(extra)
    return {"apiVersion": "kubeflow.org/v1beta1", "kind": "Experiment",
            "metadata": {"namespace": "kubeflow", "name": name}, "spec": spec}

def write(sub, fname, ref, doc, note="", trial=None):
    os.makedirs(os.path.join(R, sub), exist_ok=True)
    head = "# Counterpart of the reference's examples/v1beta1/%s.\n" % ref
    head += "# CPU-only trial: %s%s.\n" % (trial or "F(a, b) = 4a - b^2 (maximum 8 at a=2, b=0)", note)
    with open(os.path.join(R, sub, fname), "w") as f:
        f.write(head + yaml.safe_dump(doc, sort_keys=False))

# hp-tuning: one per algorithm (settings as in the reference examples)
write("hp-tuning", "random.yaml", "hp-tuning/random.yaml",
      exp("random", "random", [{"name": "random_state", "value": "10"}]))
write("hp-tuning", "tpe.yaml", "hp-tuning/tpe.yaml",
      exp("tpe", "tpe", [{"name": "random_state", "value": "10"}, {"name": "gamma", "value": "0.25"},
                         {"name": "prior_weight", "value": "1.0"}, {"name": "n_EI_candidates", "value": "24"}]))
write("hp-tuning", "multivariate-tpe.yaml", "hp-tuning/multivariate-tpe.yaml",
      exp("multivariate-tpe", "multivariate-tpe", [{"name": "n_startup_trials", "value": "5"},
                                                    {"name": "n_ei_candidates", "value": "24"},
                                                    {"name": "random_state", "value": "10"}]))
write("hp-tuning", "cma-es.yaml", "hp-tuning/cma-es.yaml",
      exp("cmaes", "cmaes", [{"name": "random_state", "value": "10"}, {"name": "sigma", "value": "0.5"}]))
write("hp-tuning", "sobol.yaml", "hp-tuning/sobol.yaml", exp("sobol", "sobol"))
write("hp-tuning", "bayesian-optimization.yaml", "hp-tuning/bayesian-optimization.yaml",
      exp("bayesian-optimization", "bayesianoptimization",
          [{"name": "random_state", "value": "10"}, {"name": "n_initial_points", "value": "4"},
           {"name": "base_estimator", "value": "GP"}, {"name": "acq_func", "value": "gp_hedge"}]))
write("hp-tuning", "grid.yaml", "hp-tuning/grid.yaml",
      exp("grid", "grid", params=[
          {"name": "a", "parameterType": "double", "feasibleSpace": {"min": "0", "max": "2", "step": "0.5"}},
          {"name": "b", "parameterType": "int", "feasibleSpace": {"min": "-1", "max": "1"}}], max_trials=15))
hb_code = ("import sys; a=${trialParameters.a}; b=${trialParameters.b}; e=int(${trialParameters.epochs})\n"
           "for s in range(e): print('result=%s' % ((4*a - b*b) * (s + 1) / e))")
write("hp-tuning", "hyperband.yaml", "hp-tuning/hyperband.yaml",
      exp("hyperband", "hyperband", [{"name": "resource_name", "value": "epochs"}, {"name": "eta", "value": "3"},
                                      {"name": "r_l", "value": "9"}],
          params=PARAMS + [{"name": "epochs", "parameterType": "int", "feasibleSpace": {"min": "1", "max": "9"}}],
          command=["python3", "-c", hb_code], parallel=9, max_trials=20,
          objective={"type": "maximize", "objectiveMetricName": "result"}),
      note="; the resource parameter scales the reported objective")

# early stopping: median stop (TEXT and JSON formats)
ms_code = ("import time; a=${trialParameters.a}; b=${trialParameters.b}\n"
           "for s in range(8):\n    print('result=%s' % ((4*a - b*b) * (s + 1) / 8), flush=True); time.sleep(0.02)")
ms = {"earlyStopping": {"algorithmName": "medianstop", "algorithmSettings": [
    {"name": "min_trials_required", "value": "2"}, {"name": "start_step", "value": "2"}]}}
write("early-stopping", "median-stop.yaml", "early-stopping/median-stop.yaml",
      exp("median-stop", "random", [{"name": "random_state", "value": "10"}], command=["python3", "-u", "-c", ms_code],
          parallel=2, max_trials=8, extra=ms, objective={"type": "maximize", "objectiveMetricName": "result"}))
msj_code = ("import json, time; a=${trialParameters.a}; b=${trialParameters.b}\n"
            "for s in range(8):\n"
            "    with open('/tmp/katib-median-stop-${trialSpec.Name}.json', 'a') as f:\n"
            "        f.write(json.dumps({'result': str((4*a - b*b) * (s + 1) / 8), 'step': str(s)}) + '\\n')\n"
            "    time.sleep(0.02)")
write("early-stopping", "median-stop-with-json-format.yaml", "early-stopping/median-stop-with-json-format.yaml",
      exp("median-stop-with-json-format", "random", [{"name": "random_state", "value": "10"}],
          command=["python3", "-u", "-c", msj_code], parallel=2, max_trials=8,
          extra={**ms, "metricsCollectorSpec": {"collector": {"kind": "File"}, "source": {"fileSystemPath": {
              "path": "/tmp/katib-median-stop-${trialSpec.Name}.json", "kind": "File", "format": "JSON"}}}},
          objective={"type": "maximize", "objectiveMetricName": "result"}))

# metrics collectors
file_code = ("a=${trialParameters.a}; b=${trialParameters.b}\n"
             "with open('/tmp/katib-file-${trialSpec.Name}.log', 'w') as f:\n"
             "    f.write('result=%s\\naccuracy=%s\\n' % (4*a - b*b, a / 2))")
write("metrics-collector", "file-metrics-collector.yaml", "metrics-collector/file-metrics-collector.yaml",
      exp("file-metrics-collector", "random", [{"name": "random_state", "value": "10"}],
          command=["python3", "-c", file_code], max_trials=6,
          extra={"metricsCollectorSpec": {"collector": {"kind": "File"}, "source": {
              "fileSystemPath": {"path": "/tmp/katib-file-${trialSpec.Name}.log", "kind": "File"},
              "filter": {"metricsFormat": ["([\\w|-]+)\\s*=\\s*([+-]?\\d*(\\.\\d+)?([Ee][+-]?\\d+)?)"]}}}},
          objective={"type": "maximize", "goal": 7.99, "objectiveMetricName": "result",
                     "additionalMetricNames": ["accuracy"]}))
json_code = ("import json; a=${trialParameters.a}; b=${trialParameters.b}\n"
             "with open('/tmp/katib-json-${trialSpec.Name}.json', 'w') as f:\n"
             "    f.write(json.dumps({'result': str(4*a - b*b), 'accuracy': str(a / 2)}) + '\\n')")
write("metrics-collector", "file-metrics-collector-with-json-format.yaml",
      "metrics-collector/file-metrics-collector-with-json-format.yaml",
      exp("file-metrics-collector-json", "random", [{"name": "random_state", "value": "10"}],
          command=["python3", "-c", json_code], max_trials=6,
          extra={"metricsCollectorSpec": {"collector": {"kind": "File"}, "source": {"fileSystemPath": {
              "path": "/tmp/katib-json-${trialSpec.Name}.json", "kind": "File", "format": "JSON"}}}},
          objective={"type": "maximize", "goal": 7.99, "objectiveMetricName": "result",
                     "additionalMetricNames": ["accuracy"]}))
write("metrics-collector", "custom-metrics-collector.yaml", "metrics-collector/custom-metrics-collector.yaml",
      exp("custom-metrics-collector", "random", [{"name": "random_state", "value": "10"}],
          command=["python3", "-c", "a=${trialParameters.a}; b=${trialParameters.b}; "
                   "print('epoch 1: result is %s' % (4*a - b*b))"], max_trials=6,
          extra={"metricsCollectorSpec": {"collector": {"kind": "StdOut"}, "source": {"filter": {
              "metricsFormat": ["(result) is ([+-]?\\d+(\\.\\d+)?([Ee][+-]?\\d+)?)"]}}}}),
      note="; a custom metricsFormat regex on stdout (no sidecar image to run)")
strat_code = ("a=${trialParameters.a}; b=${trialParameters.b}\n"
              "for s in range(4): print('loss=%s\\naccuracy=%s' % ((a - 1.5)**2 + b*b + 1.0/(s+1), a/2 - 0.1*s))")
write("metrics-collector", "metrics-collection-strategy.yaml", "metrics-collector/metrics-collection-strategy.yaml",
      exp("metrics-collection-strategy", "tpe", [{"name": "random_state", "value": "10"}],
          command=["python3", "-c", strat_code], max_trials=6,
          objective={"type": "minimize", "objectiveMetricName": "loss", "additionalMetricNames": ["accuracy"],
                     "metricStrategies": [{"name": "accuracy", "value": "max"}, {"name": "loss", "value": "min"}]}),
      trial="over steps s=0..3 it prints loss = (a-1.5)^2 + b^2 + 1/(s+1) and accuracy = a/2 - 0.1 s; "
            "the strategies keep min(loss) and max(accuracy)")

# resume policies
write("resume-experiment", "long-running-resume.yaml", "resume-experiment/long-running-resume.yaml",
      exp("long-running-resume", "random", [{"name": "random_state", "value": "10"}], max_trials=6,
          extra={"resumePolicy": "LongRunning"}, objective={"type": "maximize", "objectiveMetricName": "result"}),
      note="; raise maxTrialCount after completion to resume")
write("resume-experiment", "from-volume-resume.yaml", "resume-experiment/from-volume-resume.yaml",
      exp("from-volume-resume", "random", [{"name": "random_state", "value": "10"}], max_trials=6,
          extra={"resumePolicy": "FromVolume"}, objective={"type": "maximize", "objectiveMetricName": "result"}),
      note="; suggestion state persists in the state directory")

# trial template: metadata substitution
md = exp("trial-metadata-substitution", "random", [{"name": "random_state", "value": "10"}],
         command=["python3", "-c", "import os; a=${trialParameters.a}; b=${trialParameters.b}; "
                  "assert os.environ['TRIAL_NAME'] and os.environ['TRIAL_KIND'] == 'Job'; "
                  "assert os.environ['TRIAL_API_VERSION'] == 'batch/v1'; "
                  "assert os.environ['TRIAL_LABEL'] == 'custom-label'; "
                  "assert os.environ['TRIAL_ANNOTATION'] == 'custom-annotation'; "
                  "print('result=%s' % (4*a - b*b))"],
         max_trials=4,
         tp=[{"name": "a", "reference": "a"}, {"name": "b", "reference": "b"},
             {"name": "trialName", "reference": "${trialSpec.Name}"},
             {"name": "trialNamespace", "reference": "${trialSpec.Namespace}"},
             {"name": "trialKind", "reference": "${trialSpec.Kind}"},
             {"name": "trialAPIVersion", "reference": "${trialSpec.APIVersion}"},
             {"name": "trialLabelCustom", "reference": "${trialSpec.Labels[custom-key]}"},
             {"name": "trialAnnotationCustom", "reference": "${trialSpec.Annotations[custom-key]}"}],
         metadata_env=[{"name": "TRIAL_NAME", "value": "${trialParameters.trialName}"},
                       {"name": "TRIAL_NAMESPACE", "value": "${trialParameters.trialNamespace}"},
                       {"name": "TRIAL_KIND", "value": "${trialParameters.trialKind}"},
                       {"name": "TRIAL_API_VERSION", "value": "${trialParameters.trialAPIVersion}"},
                       {"name": "TRIAL_LABEL", "value": "${trialParameters.trialLabelCustom}"},
                       {"name": "TRIAL_ANNOTATION", "value": "${trialParameters.trialAnnotationCustom}"}],
         objective={"type": "maximize", "objectiveMetricName": "result"})
ts = md["spec"]["trialTemplate"]["trialSpec"]
ts_new = {"apiVersion": ts["apiVersion"], "kind": ts["kind"],
          "metadata": {"labels": {"custom-key": "custom-label"}, "annotations": {"custom-key": "custom-annotation"}},
          "spec": ts["spec"]}
md["spec"]["trialTemplate"]["trialSpec"] = ts_new
write("trial-template", "trial-metadata-substitution.yaml", "trial-template/trial-metadata-substitution.yaml", md)
