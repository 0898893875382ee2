"""katib_amd - a Katib-compatible AutoML engine built for AMD MI355X nodes.

Hyperparameter tuning (random, grid, TPE, multivariate-TPE, CMA-ES, Sobol,
Bayesian optimisation, HyperBand, PBT), early stopping (median stop) and neural
architecture search (DARTS, ENAS) with the Katib v1beta1 Experiment API, run by
an in-process trial scheduler that pins ``parallelTrialCount`` trials onto the
node's GPUs. See README.md / SURVEY.md.
"""

__version__ = "0.1.0"


def report(**metrics):
    """Emit metrics from a trial in the default collector format (``name=value``)."""
    print(" ".join("%s=%s" % (k, v) for k, v in metrics.items()), flush=True)
