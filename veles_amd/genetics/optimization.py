"""``--optimize N[:G]``: genetic search over the ``Range`` leaves of the
config tree, every chromosome evaluated by a full child training run.

Reference: veles/genetics/optimization_workflow.py:70-339 (GeneticsOptimizer:
chromosomes -> config values -> ``python -m veles ... --result-file`` per
evaluation, fitness = the child's ``EvaluationFitness``; the best config is
written to ``<workflow>_best_config.py``).  The evaluations of a generation
run concurrently on the job farm, one child per GPU
(veles_amd/parallel/jobfarm.py).
"""
from __future__ import annotations

import json
import os

from veles_amd.genetics.config import Range, find_tuneables
from veles_amd.genetics.core import Population
from veles_amd.parallel.jobfarm import Job, JobFarm, veles_argv
from veles_amd.utils.config import Config, root
from veles_amd.utils.logger import Logger

__all__ = ["GeneticsOptimizer", "run_optimization", "path_expr",
           "parse_optimize"]


def parse_optimize(spec):
    """"N[:G]" -> (population size, generations)."""
    parts = str(spec).split(":")
    size = int(parts[0])
    gens = int(parts[1]) if len(parts) > 1 and parts[1] else 10
    return size, gens


def path_expr(path, base=None):
    """("a", "layers", 0, "<-", "lr") -> "root.a.layers[0]['<-']['lr']"."""
    node = root if base is None else base
    expr = "root"
    for k in path:
        if isinstance(node, Config):
            expr += "." + str(k)
            node = getattr(node, k)
        else:
            expr += "[%r]" % (k,)
            node = node[k]
    return expr


class GeneticsOptimizer(Logger):
    def __init__(self, size, generations, evaluate_many, seed=1234,
                 selection="roulette"):
        super().__init__()
        self.tuneables = [(p, t) for p, t in find_tuneables(root)
                          if isinstance(t, Range)]
        if not self.tuneables:
            raise ValueError("--optimize needs Range(...) values in the "
                             "config")
        self.exprs = [path_expr(p) for p, _ in self.tuneables]
        ts = [t for _, t in self.tuneables]
        self.population = Population(
            [t.min_value for t in ts], [t.max_value for t in ts], size,
            seed=seed, max_generations=generations, selection=selection,
            is_int=[t.is_int for t in ts], initial=[t.default for t in ts])
        self.evaluate_many = evaluate_many

    def overrides(self, chromo):
        return ["%s=%r" % (e, v) for e, v in zip(self.exprs, chromo.numeric)]

    def run(self):
        best = self.population.optimize(None, self._evaluate)
        return best

    def _evaluate(self, chromos):
        self.evaluate_many(chromos, [self.overrides(c) for c in chromos])


def _child_argv(main):
    argv = list(main.argv)
    if "--optimize" in argv:
        i = argv.index("--optimize")
        del argv[i:i + 2]
    argv = [a for a in argv if not a.startswith("--optimize=")]
    if "--result-file" in argv:
        i = argv.index("--result-file")
        del argv[i:i + 2]
    return argv


def run_optimization(main, module, args):
    size, gens = parse_optimize(args.optimize)
    base = _child_argv(main)
    farm = JobFarm(timeout=None)
    log = Logger()

    def evaluate_many(chromos, overrides):
        jobs = [Job(veles_argv(*(base + ["--random-seed", "1234"] + ov)),
                    tag="chromosome %d" % i)
                for i, ov in enumerate(overrides)]
        for c, job in zip(chromos, farm.map(jobs)):
            r = job.result or {}
            c.fitness = float(r.get("EvaluationFitness", float("-inf")))
            c.config = overrides[chromos.index(c)]
            c.snapshot = r.get("Snapshot")
            log.info("%s -> fitness %s", c, c.fitness)

    opt = GeneticsOptimizer(size, gens, evaluate_many)
    best = opt.run()
    lines = opt.overrides(best)
    wf_base = os.path.splitext(args.workflow)[0]
    cfg = args.config
    if cfg == "-":
        cfg = wf_base + "_config.py"
    out_cfg = wf_base + "_best_config.py"
    with open(out_cfg, "w") as f:
        if cfg and os.path.exists(cfg):
            with open(cfg) as src:
                f.write(src.read())
        f.write("\n# best chromosome of the genetic search (fitness %r)\n" %
                best.fitness)
        for ln in lines:
            f.write(ln + "\n")
    log.info("Best config written to %s", out_cfg)
    result = {"EvaluationFitness": best.fitness,
              "best": dict(zip(opt.exprs, best.numeric)),
              "best_config": out_cfg,
              "generations": opt.population.history}
    if args.result_file:
        with open(args.result_file, "w") as f:
            json.dump(result, f, indent=2, default=str)
    return 0
