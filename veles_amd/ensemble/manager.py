"""``--ensemble-train N:ratio`` / ``--ensemble-test file``.

Reference: veles/ensemble/{base_workflow,model_workflow,test_workflow}.py —
train N models, each on a random ``train_ratio`` share of the TRAIN set with
its own seed, record each model's results and snapshot in one JSON file;
``--ensemble-test`` re-runs every member in ``--test`` mode from its
snapshot and stores its ``Output`` / ``Labels`` next to it (the input of
``EnsembleLoader``, veles_amd/loader/ensemble.py).  Members train
concurrently on the job farm, one per GPU.
"""
from __future__ import annotations

import json
import os

from veles_amd.parallel.jobfarm import Job, JobFarm, veles_argv
from veles_amd.utils.logger import Logger

__all__ = ["run_ensemble", "parse_ensemble_train"]


def parse_ensemble_train(spec):
    n, _, ratio = str(spec).partition(":")
    n, ratio = int(n), float(ratio or 1.0)
    if n < 1 or not 0 < ratio <= 1:
        raise ValueError("--ensemble-train N:ratio with N >= 1, 0 < ratio "
                         "<= 1 (got %r)" % spec)
    return n, ratio


def _strip(argv, *flags):
    argv = list(argv)
    for f in flags:
        while f in argv:
            i = argv.index(f)
            del argv[i:i + 2]
    return argv


def _ensemble_file(args):
    if args.result_file:
        return args.result_file
    return os.path.splitext(args.workflow)[0] + "_ensemble.json"


def run_ensemble(main, module, args):
    log = Logger()
    farm = JobFarm()
    base = _strip(main.argv, "--ensemble-train", "--ensemble-test",
                  "--result-file", "--train-ratio", "--random-seed", "-r")
    if args.ensemble_train:
        n, ratio = parse_ensemble_train(args.ensemble_train)
        jobs = []
        for i in range(n):
            jobs.append(Job(veles_argv(*(
                ["--train-ratio", str(ratio), "--random-seed",
                 str(1000 + 7919 * i)] + base +
                ["root.common.ensemble.model_index=%d" % i,
                 "root.common.ensemble.size=%d" % n])),
                tag="model %d" % i))
        models = []
        for i, job in enumerate(farm.map(jobs)):
            r = job.result
            if r is None:
                log.error("model %d failed", i)
                continue
            r["id"] = i
            r["train_ratio"] = ratio
            models.append(r)
        out = {"size": n, "train_ratio": ratio, "models": models,
               "workflow": args.workflow, "config": args.config}
        path = _ensemble_file(args)
        with open(path, "w") as f:
            json.dump(out, f, indent=1, default=str)
        log.info("Ensemble of %d/%d models written to %s", len(models), n,
                 path)
        return 0 if models else 1
    # --ensemble-test: evaluate every member from its snapshot
    with open(args.ensemble_test) as f:
        ens = json.load(f)
    jobs = []
    for m in ens["models"]:
        snap = m.get("Snapshot")
        if not snap:
            raise ValueError("model %s has no snapshot" % m.get("id"))
        jobs.append(Job(veles_argv(*(["--test", "--snapshot", snap] + base)),
                        tag="model %s" % m.get("id")))
    for m, job in zip(ens["models"], farm.map(jobs)):
        r = job.result or {}
        m["Output"] = r.get("Output")
        m["Labels"] = r.get("Labels")
        m["test"] = {k: v for k, v in r.items()
                     if k not in ("Output", "Labels")}
    path = args.result_file or args.ensemble_test
    with open(path, "w") as f:
        json.dump(ens, f, indent=1, default=str)
    log.info("Ensemble test results written to %s", path)
    return 0
