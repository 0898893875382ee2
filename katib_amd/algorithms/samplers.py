"""Search samplers shared by the HPO suggestion services.

The heavy numerical cores are native (``katib_amd._native``: Sobol, CMA-ES, TPE);
this module adapts them to Katib parameter specs and implements the ask/tell
bookkeeping that the reference gets from hyperopt / optuna / goptuna / skopt:

================  ===================================================  =====================
sampler           behaviour                                             reference analogue
================  ===================================================  =====================
RandomSampler     independent uniform draws (INT/DOUBLE honour step)    hyperopt.rand, optuna
                                                                        RandomSampler, goptuna
TpeSampler        univariate Parzen/EI (hyperopt) or optuna-style;      hyperopt.tpe,
                  ``multivariate`` = joint kernels + constant liar      optuna TPESampler
CmaEsSampler      generation-tagged CMA-ES asks, tell when a full       goptuna cmaes,
                  population of the generation completed; IPOP/BIPOP    optuna CmaEsSampler
SobolSampler      i-th point of a Joe-Kuo Sobol sequence                goptuna sobol
GridSampler       shuffled walk over the full cartesian grid            optuna GridSampler
BayesOptSampler   GP / RF / ET / GBRT surrogate, EI/PI/LCB/gp_hedge,    skopt.Optimizer
                  sampling or L-BFGS acquisition optimiser,
                  constant-liar (cl_min) batches, log-uniform DOUBLE
================  ===================================================  =====================
"""

from __future__ import annotations

import itertools
import math
import os
from typing import Dict, List, Optional

import numpy as np

from .internal import (AlgorithmError, CATEGORICAL, DISCRETE, DOUBLE, INTEGER, MAX_GOAL, Param, SearchSpace)


def _native():
    from .. import native

    return native.load()


# ------------------------------------------------------------------------------- study
class Study:
    """Observation history + outstanding asks for one experiment."""

    def __init__(self, space: SearchSpace):
        self.space = space
        self.observations: List[Dict] = []  # {"params": {name: typed}, "loss": float, "name": str}
        self.pending: Dict[str, List[Dict]] = {}  # assignment key -> [params]
        self.recorded: set = set()
        self.n_asked = 0

    @staticmethod
    def key(assign: Dict[str, str]) -> str:
        return ",".join(f"{k}:{assign[k]}" for k in sorted(assign))

    def typed(self, assign: Dict[str, str]) -> Dict:
        out = {}
        for p in self.space.params:
            v = assign.get(p.name)
            if v is None:
                continue
            if p.type == INTEGER:
                out[p.name] = int(float(v))
            elif p.type == DOUBLE:
                out[p.name] = float(v)
            else:
                out[p.name] = str(v)
        return out

    def register_ask(self, params: Dict):
        from .internal import format_value

        k = self.key({n: format_value(v) for n, v in params.items() if not n.startswith("__")})
        self.pending.setdefault(k, []).append(params)
        self.n_asked += 1

    def tell(self, name: str, assign: Dict[str, str], loss: float) -> Optional[Dict]:
        """Record a completed trial once. Returns the matching asked params (or the
        trial's own parsed params when the trial was not produced by this study)."""
        if name in self.recorded:
            return None
        self.recorded.add(name)
        k = self.key(assign)
        lst = self.pending.get(k)
        params = lst.pop(0) if lst else self.typed(assign)
        self.observations.append({"params": params, "loss": loss, "name": name})
        return params

    def running_params(self) -> List[Dict]:
        return [p for lst in self.pending.values() for p in lst]


class Sampler:
    def __init__(self, space: SearchSpace, seed: Optional[int] = None):
        self.space = space
        self.rng = np.random.RandomState(seed)
        self.seed = seed

    def sample(self, study: Study, request_size: int) -> Dict:
        raise NotImplementedError

    def on_tell(self, study: Study, params: Dict, loss: float):
        pass

    def random_params(self) -> Dict:
        return {p.name: p.sample_uniform(self.rng) for p in self.space.params}


class RandomSampler(Sampler):
    def sample(self, study, request_size):
        return self.random_params()


# ------------------------------------------------------------------------------- TPE
class TpeSampler(Sampler):
    """mode="hyperopt": gamma 0.25 (ceil(gamma*sqrt(n)) below), prior_weight 1,
    24 EI candidates, startup = size of the current request (base_service.py:213-231).
    mode="optuna": gamma 0.1 (min(ceil(0.1 n), 25)), 10 startup trials, constant liar."""

    def __init__(self, space, seed=None, mode="hyperopt", gamma=None, prior_weight=1.0, n_ei_candidates=24,
                 n_startup_trials=None, multivariate=False, constant_liar=False):
        super().__init__(space, seed)
        self.mode = mode
        self.gamma = gamma if gamma is not None else (0.25 if mode == "hyperopt" else 0.1)
        self.prior_weight = prior_weight
        self.n_ei = n_ei_candidates
        self.n_startup = n_startup_trials
        self.multivariate = multivariate
        self.constant_liar = constant_liar
        self._draws = 0

    def _dims(self):
        dims = []
        for p in self.space.params:
            if p.type in (CATEGORICAL, DISCRETE):
                dims.append({"kind": 1, "n_choices": len(p.list)})
            elif p.type == INTEGER:
                dims.append({"kind": 0, "low": p.min, "high": p.max, "q": float(p.step or 1)})
            else:
                dims.append({"kind": 0, "low": p.min, "high": p.max, "q": float(p.step or 0)})
        return dims

    def _vec(self, params):
        return [p.to_internal(str(params[p.name])) if p.type in (CATEGORICAL, DISCRETE) else float(params[p.name])
                for p in self.space.params]

    def sample(self, study, request_size):
        startup = self.n_startup
        if startup is None:
            startup = request_size if self.mode == "hyperopt" else 10
        obs = study.observations
        if len(obs) < max(startup, 1):
            return self.random_params()
        xs = [self._vec(o["params"]) for o in obs]
        losses = [o["loss"] for o in obs]
        if self.constant_liar:
            worst = max(losses)
            for rp in study.running_params():
                xs.append(self._vec(rp))
                losses.append(worst)
        self._draws += 1
        seed = int(self.rng.randint(0, 2**31 - 1))
        x = _native().tpe_sample(self._dims(), xs, losses,
                                 {"gamma": self.gamma, "gamma_mode": 0 if self.mode == "hyperopt" else 1,
                                  "prior_weight": self.prior_weight, "n_ei_candidates": self.n_ei,
                                  "multivariate": self.multivariate}, seed)
        return {p.name: p.from_internal(v) for p, v in zip(self.space.params, x)}


# ------------------------------------------------------------------------------- CMA-ES
class CmaEsSampler(Sampler):
    """Relative CMA-ES over INT/DOUBLE dims (categoricals are drawn at random, as
    goptuna's independent fallback does). Each ask is tagged with the optimizer
    generation; once ``popsize`` trials of the current generation completed the
    generation is told (goptuna/cmaes/sampler.go semantics). ``restart_strategy``
    ipop doubles the population on stagnation; bipop alternates large/small."""

    def __init__(self, space, seed=None, sigma0=None, restart_strategy=None, popsize=None, inc_popsize=2):
        super().__init__(space, seed)
        self.num_params = [p for p in space.params if p.is_numeric]
        if len(self.num_params) < 1:
            raise AlgorithmError("cmaes only supports two or more dimensional continuous search space.")
        self.lo = [p.min for p in self.num_params]
        self.hi = [p.max for p in self.num_params]
        self.sigma0 = sigma0 if sigma0 else min(h - l for l, h in zip(self.lo, self.hi)) / 6.0
        self.restart = restart_strategy if restart_strategy not in ("none", "None", "") else None
        self.inc_popsize = inc_popsize
        self.base_popsize = popsize or 0
        self.n_restarts = 0
        self._small_budget = 0
        self._large_budget = 0
        self._make(self.base_popsize)
        self.tags: Dict[int, int] = {}  # id(params) -> generation
        self.gen_solutions: List = []

    def _make(self, popsize, sigma=None, mean=None):
        if mean is None:
            mean = [l + (h - l) / 2.0 for l, h in zip(self.lo, self.hi)]
        seed = int(self.rng.randint(0, 2**31 - 1))
        self.opt = _native().CmaEs(mean, sigma or self.sigma0, self.lo, self.hi, seed, popsize)
        self.gen_solutions = []

    def sample(self, study, request_size):
        x = self.opt.ask()
        params = {}
        xi = iter(x)
        for p in self.space.params:
            if p.is_numeric:
                params[p.name] = p.from_internal(next(xi))
            else:
                params[p.name] = p.sample_uniform(self.rng)
        params["__cma_gen__"] = self.opt.generation
        params["__cma_x__"] = list(x)
        return params

    def on_tell(self, study, params, loss):
        gen = params.get("__cma_gen__")
        if gen is None:
            return
        if gen != self.opt.generation:
            return  # stale generation result: dropped (it cannot be told any more)
        self.gen_solutions.append((params["__cma_x__"], loss))
        if len(self.gen_solutions) >= self.opt.popsize:
            sol = self.gen_solutions[: self.opt.popsize]
            self.opt.tell([s[0] for s in sol], [s[1] for s in sol])
            self.gen_solutions = self.gen_solutions[self.opt.popsize:]
            if self.restart and self.opt.should_stop():
                self._do_restart()

    def _do_restart(self):
        self.n_restarts += 1
        pop = self.opt.popsize
        if self.restart == "ipop":
            self._make(pop * self.inc_popsize)
        else:  # bipop: alternate a doubled regime and a small-population regime
            large = (self.base_popsize or pop) * (self.inc_popsize ** self.n_restarts)
            if self._small_budget < self._large_budget:
                small = max(2, int(pop * (0.5 * (large / pop)) ** (self.rng.uniform() ** 2)))
                self._make(small, sigma=self.sigma0 * 10 ** (-2 * self.rng.uniform()))
                self._small_budget += small
            else:
                self._make(large)
                self._large_budget += large


# ------------------------------------------------------------------------------- Sobol
_SOBOL_TABLE = None


def sobol_table():
    global _SOBOL_TABLE
    if _SOBOL_TABLE is None:
        import scipy.stats

        path = os.path.join(os.path.dirname(scipy.stats.__file__), "_sobol_direction_numbers.npz")
        z = np.load(path)  # allow_pickle=False (default): plain integer arrays
        _SOBOL_TABLE = (z["poly"].astype(np.int64), z["vinit"].astype(np.int64))
    return _SOBOL_TABLE


class SobolSampler(Sampler):
    def __init__(self, space, seed=None):
        super().__init__(space, seed)
        poly, vinit = sobol_table()
        d = max(1, len(space.params))
        self.engine = _native().SobolEngine(d, poly[:d].tolist(), vinit[:d].tolist())

    def sample(self, study, request_size):
        u = self.engine.point(study.n_asked)
        params = {}
        for p, x in zip(self.space.params, u):
            if p.is_numeric:
                params[p.name] = p.from_internal(p.min + x * (p.max - p.min))
            else:
                params[p.name] = p.list[min(int(x * len(p.list)), len(p.list) - 1)]
        return params


# ------------------------------------------------------------------------------- grid
class GridSampler(Sampler):
    def __init__(self, space, seed=None):
        super().__init__(space, seed)
        combos = space.combinations()
        self.names = list(combos)
        self.grid = list(itertools.product(*combos.values()))
        order = np.arange(len(self.grid))
        self.rng.shuffle(order)
        self.order = list(order)
        self.pos = 0

    def __len__(self):
        return len(self.grid)

    def exhausted(self) -> bool:
        return self.pos >= len(self.order)

    def sample(self, study, request_size):
        if self.exhausted():
            # every point has been proposed: re-visit (optuna warns and re-samples)
            self.pos = 0
        g = self.grid[self.order[self.pos]]
        self.pos += 1
        return dict(zip(self.names, g))


# ------------------------------------------------------------------------------- Bayesian optimisation
class BayesOptSampler(Sampler):
    """skopt.Optimizer equivalent. DOUBLE dims use a log-uniform prior, exactly as the
    reference (``skopt/base_service.py:57-58``) -- they are modelled in log space."""

    ACQS = ("gp_hedge", "LCB", "EI", "PI", "EIps", "PIps")

    def __init__(self, space, seed=None, base_estimator="GP", n_initial_points=10, acq_func="gp_hedge",
                 acq_optimizer="auto", n_candidates=4000, xi=0.01, kappa=1.96):
        super().__init__(space, seed)
        self.base_estimator = base_estimator
        self.n_initial = n_initial_points
        self.acq_func = acq_func
        self.acq_optimizer = acq_optimizer
        self.n_candidates = n_candidates
        self.xi, self.kappa = xi, kappa
        self.gains = np.zeros(3)
        self._batch = []

    # unit-cube encoding (categoricals one-hot)
    def _encode(self, params: Dict) -> np.ndarray:
        out = []
        for p in self.space.params:
            v = params[p.name]
            if p.type == DOUBLE:
                if p.min > 0:
                    lo, hi = math.log(p.min), math.log(p.max)
                    out.append((math.log(max(float(v), p.min)) - lo) / max(hi - lo, 1e-12))
                else:
                    out.append((float(v) - p.min) / max(p.max - p.min, 1e-12))
            elif p.type == INTEGER:
                out.append((float(v) - p.min) / max(p.max - p.min, 1e-12))
            else:
                oh = [0.0] * len(p.list)
                if str(v) in p.list:
                    oh[p.list.index(str(v))] = 1.0
                out.extend(oh)
        return np.asarray(out, dtype=np.float64)

    def _random_encoded(self, n):
        cols = []
        for p in self.space.params:
            if p.type in (CATEGORICAL, DISCRETE):
                idx = self.rng.randint(0, len(p.list), size=n)
                cols.append(np.eye(len(p.list))[idx])
            else:
                cols.append(self.rng.uniform(0, 1, size=(n, 1)))
        return np.concatenate(cols, axis=1)

    def _decode(self, z: np.ndarray) -> Dict:
        out, i = {}, 0
        for p in self.space.params:
            if p.type == DOUBLE:
                u = float(np.clip(z[i], 0, 1))
                if p.min > 0:
                    lo, hi = math.log(p.min), math.log(p.max)
                    out[p.name] = p.from_internal(math.exp(lo + u * (hi - lo)))
                else:
                    out[p.name] = p.from_internal(p.min + u * (p.max - p.min))
                i += 1
            elif p.type == INTEGER:
                out[p.name] = p.from_internal(p.min + float(np.clip(z[i], 0, 1)) * (p.max - p.min))
                i += 1
            else:
                k = len(p.list)
                out[p.name] = p.list[int(np.argmax(z[i:i + k]))]
                i += k
        return out

    def _fit(self, X, y):
        from sklearn.ensemble import ExtraTreesRegressor, GradientBoostingRegressor, RandomForestRegressor
        from sklearn.gaussian_process import GaussianProcessRegressor
        from sklearn.gaussian_process.kernels import ConstantKernel, Matern, WhiteKernel

        seed = int(self.rng.randint(0, 2**31 - 1))
        be = self.base_estimator
        if be == "GP":
            k = ConstantKernel(1.0, (0.01, 1000.0)) * Matern(length_scale=np.ones(X.shape[1]),
                                                            length_scale_bounds=(0.01, 100.0), nu=2.5) \
                + WhiteKernel(1e-5, (1e-9, 1e-1))
            m = GaussianProcessRegressor(kernel=k, normalize_y=True, n_restarts_optimizer=2, random_state=seed)
            m.fit(X, y)
            return lambda Z: m.predict(Z, return_std=True)
        if be in ("RF", "ET"):
            cls = RandomForestRegressor if be == "RF" else ExtraTreesRegressor
            m = cls(n_estimators=100, min_samples_leaf=3, random_state=seed)
            m.fit(X, y)

            def pred(Z):
                allp = np.stack([t.predict(Z) for t in m.estimators_])
                return allp.mean(0), allp.std(0) + 1e-9
            return pred
        if be == "GBRT":
            models = []
            for a in (0.16, 0.5, 0.84):
                g = GradientBoostingRegressor(loss="quantile", alpha=a, n_estimators=100, random_state=seed)
                g.fit(X, y)
                models.append(g)

            def pred(Z):
                lo, mid, hi = (g.predict(Z) for g in models)
                return mid, np.maximum((hi - lo) / 2.0, 1e-9)
            return pred
        raise AlgorithmError(f"base_estimator {be} is not supported in Bayesian optimization")

    @staticmethod
    def _acq(kind, mu, sd, ybest, xi, kappa):
        from scipy.stats import norm

        sd = np.maximum(sd, 1e-12)
        if kind in ("EI", "EIps"):
            imp = ybest - mu - xi
            z = imp / sd
            return imp * norm.cdf(z) + sd * norm.pdf(z)
        if kind in ("PI", "PIps"):
            return norm.cdf((ybest - mu - xi) / sd)
        return -(mu - kappa * sd)  # LCB (maximise the negative bound)

    def _propose(self, X, y):
        pred = self._fit(X, y)
        cands = self._random_encoded(self.n_candidates)
        mu, sd = pred(cands)
        ybest = float(np.min(y))
        kinds = ["EI", "PI", "LCB"]
        if self.acq_func == "gp_hedge":
            probs = np.exp(self.gains - self.gains.max())
            probs /= probs.sum()
            scores = [self._acq(k, mu, sd, ybest, self.xi, self.kappa) for k in kinds]
            picks = [int(np.argmax(s)) for s in scores]
            chosen = int(self.rng.choice(3, p=probs))
            idx = picks[chosen]
            # update gains with the (negated) predicted value at each candidate
            self.gains -= np.array([mu[i] for i in picks])
        else:
            s = self._acq(self.acq_func, mu, sd, ybest, self.xi, self.kappa)
            idx = int(np.argmax(s))
        best = cands[idx]
        numeric_only = all(p.type in (DOUBLE, INTEGER) for p in self.space.params)
        if self.acq_optimizer == "lbfgs" or (self.acq_optimizer == "auto" and numeric_only
                                             and self.base_estimator == "GP"):
            from scipy.optimize import minimize

            kind = "EI" if self.acq_func in ("gp_hedge", "EIps") else self.acq_func
            f = lambda z: -float(self._acq(kind, *pred(z[None, :]), ybest, self.xi, self.kappa)[0])
            try:
                r = minimize(f, best, method="L-BFGS-B", bounds=[(0, 1)] * len(best), options={"maxiter": 50})
                if r.success and f(r.x) <= f(best):
                    best = r.x
            except Exception:
                pass
        return best

    def sample(self, study, request_size):
        obs = study.observations
        if len(obs) < self.n_initial or len(obs) < 2:
            return self.random_params()
        X = np.stack([self._encode(o["params"]) for o in obs])
        y = np.asarray([o["loss"] for o in obs], dtype=np.float64)
        # constant liar (cl_min) for the points already proposed but not evaluated
        pend = study.running_params()
        if pend:
            X = np.concatenate([X, np.stack([self._encode(p) for p in pend])])
            y = np.concatenate([y, np.full(len(pend), y.min())])
        return self._decode(self._propose(X, y))
