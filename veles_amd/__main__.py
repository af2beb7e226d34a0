"""``python -m veles_amd [opts] workflow.py config.py [root.x=y ...]``.

Reference: veles/__main__.py:136-864 (``Main``: argv parsing, logging, RNG
seeding, workflow import, config application, ``root.x=y`` overrides,
``--dry-run``, snapshot resume, special modes) and the user workflow
contract ``run(load, main)`` (samples/ + docs)."""
from __future__ import annotations

import logging
import os
import runpy
import sys

__all__ = ["Main", "main"]


_LAUNCH_FLAGS = ("--gpus", "--nnodes", "--node-rank", "--master-addr",
                 "--master-port")


def _strip_launch_flags(argv):
    """The command line each spawned rank gets: the launcher's own flags
    (``--gpus`` and the multi-node rendezvous) removed, both the
    ``--flag value`` and ``--flag=value`` forms."""
    out = []
    skip = False
    for a in argv:
        if skip:
            skip = False
            continue
        if a in _LAUNCH_FLAGS:
            skip = True
            continue
        if a.split("=", 1)[0] in _LAUNCH_FLAGS and "=" in a:
            continue
        out.append(a)
    return out


def _html_help(parser):
    """``--html-help`` (reference cmdline.py:139-151): the argparse help as
    a standalone HTML page, one table row per option."""
    import html
    rows = []
    for act in parser._actions:
        flags = ", ".join(act.option_strings) or act.dest
        rows.append("<tr><td><code>%s</code></td><td>%s</td></tr>" % (
            html.escape(flags), html.escape(act.help or "")))
    return ("<!DOCTYPE html><html><head><meta charset=\"utf-8\">"
            "<title>veles_amd command line</title></head><body>"
            "<h1>python -m veles_amd</h1><pre>%s</pre><table>%s</table>"
            "</body></html>" % (html.escape(parser.format_usage()),
                                "".join(rows)))


class Main(object):
    def __init__(self, argv=None):
        self.argv = sys.argv[1:] if argv is None else list(argv)
        self.workflow = None
        self.launcher = None

    # -- helpers ------------------------------------------------------------
    def _setup_logging(self, args):
        from veles_amd.utils.logger import (setup_logging,
                                            redirect_all_logging_to_file)
        lvl = getattr(logging, args.verbosity.upper())
        setup_logging(lvl)
        for name in filter(None, args.debug.split(",")):
            logging.getLogger(name).setLevel(logging.DEBUG)
        if args.log_file:
            path = args.log_file
            if args.log_file_pid:
                b, e = os.path.splitext(path)
                path = "%s.%d%s" % (b, os.getpid(), e)
            redirect_all_logging_to_file(path)

    def _seed(self, spec):
        from veles_amd.prng import random_generator
        import numpy
        import torch
        if spec in ("", None):
            seeds = [1234]
        elif spec == "-":
            seeds = [int.from_bytes(os.urandom(4), "little")]
        else:
            seeds = []
            for part in spec.split(","):
                if ":" in part and os.path.exists(part.split(":")[0]):
                    fn, cnt = part.split(":")[:2]
                    dt = part.split(":")[2] if part.count(":") > 1 else \
                        "uint32"
                    g = random_generator.RandomGenerator("file")
                    g.seed(fn, dtype=dt, count=int(cnt))
                    seeds.append(g.randint(0, 2 ** 31))
                else:
                    seeds.append(int(part, 0))
        for i, s in enumerate(seeds):
            random_generator.get(i).seed(s)
        numpy.random.seed(seeds[0] & 0xFFFFFFFF)
        torch.manual_seed(seeds[0])
        self.seeds = seeds

    @staticmethod
    def _import_workflow(path):
        from veles_amd.utils.import_file import import_file
        return import_file(path)

    @staticmethod
    def _apply_config(path, overrides):
        from veles_amd.utils.config import root
        if path:
            runpy.run_path(path, init_globals={"root": root})
        for stmt in overrides:
            if "=" not in stmt:
                raise ValueError("override %r is not root.x=y" % stmt)
            exec(stmt, {"root": root})

    # -- the run(load, main) contract ---------------------------------------
    def _load(self, workflow_class, **kwargs):
        from veles_amd.launcher import Launcher
        args = self.args
        self.launcher = Launcher(
            backend="cpu" if args.backend == "numpy" else args.backend,
            device_id=args.device or None,
            result_file=args.result_file or None, testing=args.test,
            trace_events=args.trace_events or None, log_id=args.log_id,
            snapshot_file=args.snapshot or None)
        if args.snapshot:
            from veles_amd.snapshotter import SnapshotterToFile
            wf = SnapshotterToFile.import_(args.snapshot)
            wf.workflow = self.launcher
            self.launcher.add_ref(wf)
            if args.test and hasattr(wf, "switch_to_testing"):
                wf.switch_to_testing()
            restored = True
        else:
            if args.test:
                kwargs.setdefault("testing", True)
            wf = workflow_class(self.launcher, **kwargs)
            restored = False
        self.workflow = wf
        return wf, restored

    def _main(self, **kwargs):
        args = self.args
        if args.dry_run == "load":
            return
        if args.job_timeout > 0:
            from veles_amd.utils.config import root
            root.common.engine.dp.timeout_s = max(60, int(args.job_timeout *
                                                         60))
        dev = self.launcher.initialize()
        kwargs.setdefault("device", dev)
        self.workflow.initialize(**kwargs)
        if args.workflow_graph:
            self.workflow.generate_graph(args.workflow_graph)
        if args.dry_run == "init":
            return
        if args.fault_inject_prob > 0:
            from veles_amd.parallel.faults import FaultInjector
            FaultInjector(self.workflow, args.fault_inject_prob).install()
        wd = None
        if args.job_timeout > 0:
            from veles_amd.parallel.faults import Watchdog
            wd = Watchdog(args.job_timeout * 60.0).install(self.workflow)
        self.launcher.run()
        if wd is not None:
            wd.stop()
        self.launcher.finish()
        if args.dump_unit_attributes != "no":
            for u in self.workflow:
                print(u.name, {k: v for k, v in u.__dict__.items()
                               if not k.startswith("_")})

    def run(self):
        from veles_amd import __version__
        from veles_amd.cmdline import make_parser
        from veles_amd.utils.config import root
        args = make_parser().parse_intermixed_args(self.argv)
        self.args = args
        if args.version:
            print("veles_amd", __version__)
            return 0
        if args.html_help:
            print(_html_help(make_parser()))
            return 0
        if args.gpus and int(os.environ.get("WORLD_SIZE", "1")) == 1:
            from veles_amd.parallel.launch import spawn_ranks
            argv = _strip_launch_flags(self.argv)
            return spawn_ranks(args.gpus, [sys.executable, "-m", "veles_amd"]
                               + argv, respawn=args.respawn,
                               shrink=args.respawn_shrink,
                               nnodes=args.nnodes, node_rank=args.node_rank,
                               master_addr=args.master_addr,
                               master_port=args.master_port)
        self._setup_logging(args)
        if not args.workflow:
            make_parser().print_help()
            return 1
        self._seed(args.random_seed)
        root.common.engine.backend = "cpu" if args.backend == "numpy" \
            else args.backend
        if args.force_cpu:
            root.common.engine.force_cpu = tuple(args.force_cpu.split(","))
        root.common.engine.sync_run = args.sync_run
        if args.no_graphics_client or args.matplotlib_backend == "":
            root.common.disable.plotting = True
        elif args.matplotlib_backend:
            root.common.plotting.backend = args.matplotlib_backend
        root.common.loader.train_ratio = args.train_ratio
        module = self._import_workflow(args.workflow)
        cfg = args.config
        if cfg == "-":
            cfg = os.path.splitext(args.workflow)[0] + "_config.py"
        self._apply_config(cfg, args.config_list)
        if args.dump_config:
            root.print_()
        if args.optimize:
            from veles_amd.genetics.optimization import run_optimization
            return run_optimization(self, module, args)
        if args.ensemble_train or args.ensemble_test:
            from veles_amd.ensemble.manager import run_ensemble
            return run_ensemble(self, module, args)
        from veles_amd.genetics.config import fix_config
        fix_config(root)
        module.run(self._load, self._main)
        return 0


def main(argv=None):
    return Main(argv).run()


if __name__ == "__main__":
    sys.exit(main() or 0)
