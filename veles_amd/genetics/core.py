"""Genetic algorithm core: chromosomes, population, selection, crossover and
mutation operators.

Reference behaviour (veles/genetics/core.py:122-830): chromosomes carry a
numeric vector inside per-gene [min, max] bounds (optionally a binary /
Gray-coded form); the population keeps the best ``size`` after each
evaluation round, breeds children by the crossing pipeline (uniform,
arithmetic, geometric; pointed for binary codes) from parents chosen by
roulette / random / tournament selection, and appends mutated copies
(binary_point, altering, gaussian, uniform).  Written fresh here with one
numpy generator per population so a search is reproducible from its seed.
"""
from __future__ import annotations

import numpy

from veles_amd.utils.logger import Logger

__all__ = ["Chromosome", "Population", "gray_encode", "gray_decode",
           "num_to_bin", "bin_to_num", "schwefel"]


def schwefel(values):
    """The Schwefel benchmark (a standard GA test function, maximised as
    its negative)."""
    v = numpy.asarray(values, dtype=numpy.float64)
    return -(418.9829 * len(v) - numpy.sum(v * numpy.sin(
        numpy.sqrt(numpy.abs(v)))))


def gray_encode(n):
    return n ^ (n >> 1)


def gray_decode(g):
    n = 0
    while g:
        n ^= g
        g >>= 1
    return n


def num_to_bin(values, mins, maxs, bits, gray=False):
    """Quantise each gene to ``bits`` bits -> one '0'/'1' string."""
    out = []
    q = (1 << bits) - 1
    for v, lo, hi in zip(values, mins, maxs):
        k = int(round((v - lo) / (hi - lo) * q)) if hi > lo else 0
        k = min(max(k, 0), q)
        if gray:
            k = gray_encode(k)
        out.append(format(k, "0%db" % bits))
    return "".join(out)


def bin_to_num(binary, mins, maxs, bits, gray=False):
    q = (1 << bits) - 1
    vals = []
    for i, (lo, hi) in enumerate(zip(mins, maxs)):
        k = int(binary[i * bits:(i + 1) * bits], 2)
        if gray:
            k = gray_decode(k)
        vals.append(lo + (hi - lo) * k / q)
    return vals


class Chromosome(object):
    def __init__(self, population, numeric):
        self.population = population
        self.numeric = list(numeric)
        self.fitness = None
        self.config = None
        self.snapshot = None
        self.fix()

    @property
    def size(self):
        return len(self.numeric)

    @property
    def binary(self):
        p = self.population
        return num_to_bin(self.numeric, p.min_values, p.max_values, p.bits,
                          p.code == "gray")

    @binary.setter
    def binary(self, value):
        p = self.population
        self.numeric = bin_to_num(value, p.min_values, p.max_values, p.bits,
                                  p.code == "gray")
        self.fix()

    def fix(self):
        """Clamp into bounds; integer genes are rounded."""
        p = self.population
        for i, v in enumerate(self.numeric):
            v = min(max(float(v), p.min_values[i]), p.max_values[i])
            if p.is_int[i]:
                v = int(round(v))
            self.numeric[i] = v

    def copy(self):
        c = Chromosome(self.population, self.numeric)
        return c

    # -- mutations ----------------------------------------------------------
    def mutate(self, name, n_points, probability):
        getattr(self, "mutation_" + name)(max(n_points, 1), probability)
        self.fitness = None
        self.fix()

    def _points(self, n):
        rs = self.population.rand
        return rs.choice(self.size, size=min(n, self.size), replace=False)

    def mutation_gaussian(self, n_points, probability):
        p, rs = self.population, self.population.rand
        for i in self._points(n_points):
            if rs.rand() < probability:
                span = p.max_values[i] - p.min_values[i]
                self.numeric[i] += rs.normal(0.0, span / 6.0)

    def mutation_uniform(self, n_points, probability):
        p, rs = self.population, self.population.rand
        for i in self._points(n_points):
            if rs.rand() < probability:
                self.numeric[i] = rs.uniform(p.min_values[i],
                                             p.max_values[i])

    def mutation_altering(self, n_points, probability):
        """Swap two genes' relative positions inside their ranges."""
        p, rs = self.population, self.population.rand
        if self.size < 2 or rs.rand() >= probability:
            return
        i, j = rs.choice(self.size, 2, replace=False)
        rel = [(self.numeric[k] - p.min_values[k]) /
               max(p.max_values[k] - p.min_values[k], 1e-30) for k in (i, j)]
        self.numeric[i] = p.min_values[i] + rel[1] * (
            p.max_values[i] - p.min_values[i])
        self.numeric[j] = p.min_values[j] + rel[0] * (
            p.max_values[j] - p.min_values[j])

    def mutation_binary_point(self, n_points, probability):
        rs = self.population.rand
        b = list(self.binary)
        for i in rs.choice(len(b), size=min(n_points, len(b)),
                           replace=False):
            if rs.rand() < probability:
                b[i] = "1" if b[i] == "0" else "0"
        self.binary = "".join(b)

    def __repr__(self):
        return "Chromosome(%s, fitness=%s)" % (
            ", ".join("%.6g" % v for v in self.numeric), self.fitness)


class Population(Logger):
    """``size`` chromosomes over per-gene bounds; ``update()`` makes the
    next generation once every chromosome has a fitness."""

    def __init__(self, min_values, max_values, size, seed=1234,
                 max_generations=20, code="float", bits=16,
                 selection="roulette", is_int=None, initial=None):
        super().__init__()
        if len(min_values) != len(max_values):
            raise ValueError("min_values / max_values lengths differ")
        if size < 2:
            raise ValueError("population size must be >= 2")
        self.min_values = [float(v) for v in min_values]
        self.max_values = [float(v) for v in max_values]
        self.is_int = list(is_int or [False] * len(min_values))
        self.size = int(size)
        self.rand = numpy.random.RandomState(seed)
        self.code = code
        self.bits = bits
        self.selection = selection
        self.max_generations = max_generations
        self.generation = 0
        self.roulette_select_size = 0.75
        self.random_select_size = 0.5
        self.tournament_size = 0.5
        self.tournament_select_size = 0.1
        self.crossing = {"pointed": (0.2, 1.0), "uniform": (0.15, 0.9),
                         "arithmetic": (0.15, 0.9), "geometric": (0.2, 0.9)}
        self.pipeline = ["uniform", "arithmetic", "geometric"]
        if code in ("binary", "gray"):
            self.pipeline = ["pointed", "uniform"]
        self.mutations = {
            "binary_point": {"use": code in ("binary", "gray"),
                             "chromosomes": 0.2, "points": 0.06,
                             "probability": 0.35},
            "gaussian": {"use": True, "chromosomes": 0.35, "points": 0.05,
                         "probability": 0.7},
            "uniform": {"use": True, "chromosomes": 0.35, "points": 0.05,
                        "probability": 0.7},
            "altering": {"use": False, "chromosomes": 0.1, "points": 0,
                         "probability": 0.35}}
        self.chromosomes = []
        self.history = []
        self.best = None
        if initial is not None:
            self.chromosomes.append(Chromosome(self, initial))
        while len(self.chromosomes) < self.size:
            self.chromosomes.append(Chromosome(self, [
                self.rand.uniform(lo, hi) for lo, hi in
                zip(self.min_values, self.max_values)]))

    # -- access -------------------------------------------------------------
    def __len__(self):
        return len(self.chromosomes)

    def __iter__(self):
        return iter(self.chromosomes)

    def __getitem__(self, i):
        return self.chromosomes[i]

    @property
    def pending(self):
        return [c for c in self.chromosomes if c.fitness is None]

    @property
    def done(self):
        return self.generation >= self.max_generations

    # -- selection ----------------------------------------------------------
    def _sorted(self):
        return sorted(self.chromosomes, key=lambda c: -c.fitness)

    def select(self):
        return getattr(self, "select_" + self.selection)()

    def select_roulette(self):
        chromos = self._sorted()
        fit = numpy.array([c.fitness for c in chromos], dtype=numpy.float64)
        ok = numpy.isfinite(fit)
        if not ok.any():
            fit = numpy.zeros_like(fit)
        else:  # failed evaluations (-inf) get the lowest weight
            fit = numpy.where(ok, fit, fit[ok].min() - 1.0)
        w = fit - fit.min() + 1e-12
        w /= w.sum()
        n = max(2, int(len(chromos) * self.roulette_select_size))
        idx = self.rand.choice(len(chromos), size=n, p=w)
        return [chromos[i] for i in idx]

    def select_random(self):
        n = max(2, int(len(self.chromosomes) * self.random_select_size))
        idx = self.rand.choice(len(self.chromosomes), size=n)
        return [self.chromosomes[i] for i in idx]

    def select_tournament(self):
        n = max(2, int(len(self.chromosomes) * self.tournament_size))
        k = max(2, int(len(self.chromosomes) * self.tournament_select_size))
        out = []
        for _ in range(n):
            grp = self.rand.choice(len(self.chromosomes), size=k)
            out.append(max((self.chromosomes[i] for i in grp),
                           key=lambda c: c.fitness))
        return out

    # -- crossover ----------------------------------------------------------
    def _pairs(self, parents, share):
        n = max(1, int(self.size * share))
        for _ in range(n):
            i, j = self.rand.choice(len(parents), 2)
            yield parents[i], parents[j]

    def cross_uniform(self, a, b, probability):
        child = [x if self.rand.rand() < 0.5 else y
                 for x, y in zip(a.numeric, b.numeric)]
        return child if self.rand.rand() < probability else None

    def cross_arithmetic(self, a, b, probability):
        if self.rand.rand() >= probability:
            return None
        t = self.rand.rand()
        return [t * x + (1 - t) * y for x, y in zip(a.numeric, b.numeric)]

    def cross_geometric(self, a, b, probability):
        if self.rand.rand() >= probability:
            return None
        out = []
        for x, y, lo in zip(a.numeric, b.numeric, self.min_values):
            # geometric mean in the shifted positive domain
            sx, sy = x - lo + 1e-12, y - lo + 1e-12
            out.append(lo + numpy.sqrt(sx * sy))
        return out

    def cross_pointed(self, a, b, probability):
        if self.rand.rand() >= probability:
            return None
        ba, bb = a.binary, b.binary
        npts = max(1, int(len(ba) * 0.08))
        pts = sorted(self.rand.choice(len(ba), size=npts, replace=False))
        out, src, last = [], 0, 0
        for p in list(pts) + [len(ba)]:
            out.append((ba, bb)[src][last:p])
            src ^= 1
            last = p
        c = Chromosome(self, a.numeric)
        c.binary = "".join(out)
        return c.numeric

    # -- generation step ----------------------------------------------------
    def update(self):
        """All chromosomes evaluated -> keep the best ``size``, breed and
        mutate.  Returns False once ``max_generations`` is reached."""
        if self.pending:
            raise RuntimeError("%d chromosomes are not evaluated" %
                               len(self.pending))
        ranked = self._sorted()
        self.chromosomes = ranked[:self.size]
        fits = [c.fitness for c in self.chromosomes]
        self.best = self.chromosomes[0]
        self.history.append({"generation": self.generation,
                             "best": fits[0], "average": float(
                                 numpy.mean(fits)),
                             "worst": fits[-1],
                             "median": fits[len(fits) // 2],
                             "best_values": list(self.best.numeric)})
        self.info("Generation %d: best %.6g average %.6g",
                  self.generation, fits[0], numpy.mean(fits))
        self.generation += 1
        if self.done:
            return False
        parents = self.select()
        children = []
        for name in self.pipeline:
            share, prob = self.crossing[name]
            op = getattr(self, "cross_" + name)
            for a, b in self._pairs(parents, share):
                ch = op(a, b, prob)
                if ch is not None:
                    children.append(Chromosome(self, ch))
        base = len(self.chromosomes)
        for name, mp in self.mutations.items():
            if not mp["use"]:
                continue
            for i in self.rand.choice(base, size=min(base, max(1, int(
                    base * mp["chromosomes"]))), replace=False):
                m = self.chromosomes[i].copy()
                m.mutate(name, int(m.size * mp["points"]) or 1,
                         mp["probability"])
                children.append(m)
        self.chromosomes.extend(children)
        return True

    def optimize(self, fitness_fn, evaluate_many=None):
        """Run to completion with a local fitness function (or a batch
        evaluator ``evaluate_many(chromosomes)`` that sets ``fitness``)."""
        while True:
            todo = self.pending
            if evaluate_many is not None:
                evaluate_many(todo)
            else:
                for c in todo:
                    c.fitness = float(fitness_fn(c.numeric))
            if not self.update():
                return self.best
