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


def daemonize(log_path=None):
    """``-b/--background`` (reference __main__.py:372-378): detach from the
    terminal by a double fork + setsid, BEFORE anything touches the GPU
    (a process that initialised HIP must never fork).  Returns True in the
    detached grandchild (which continues the run, stdio on ``log_path`` or
    /dev/null) and False in the original process (which should exit 0)."""
    if os.fork() > 0:
        return False
    os.setsid()
    if os.fork() > 0:
        os._exit(0)
    sys.stdout.flush()
    sys.stderr.flush()
    fd_in = os.open(os.devnull, os.O_RDONLY)
    fd_out = os.open(log_path, os.O_WRONLY | os.O_CREAT | os.O_APPEND,
                     0o644) if log_path else os.open(os.devnull, os.O_WRONLY)
    os.dup2(fd_in, 0)
    os.dup2(fd_out, 1)
    os.dup2(fd_out, 2)
    return True


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
            from veles_amd.snapshotter import import_snapshot
            wf = import_snapshot(args.snapshot)
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
        """The second half of the run(load, main) contract.  ``--dry-run``
        (reference cmdline.py:172-177, __main__.py:628-656): ``init`` stops
        before the workflow is initialised, ``exec`` before it runs;
        ``--visualize`` initialises, writes the workflow graph and renders
        every plotter once instead of running."""
        args = self.args
        if args.dry_run in ("load", "init"):
            self.stopped_before = "initialize"
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
        if args.manhole:
            from veles_amd.interaction import install_manhole
            self.manhole_path = install_manhole(self.workflow)
            logging.getLogger("Main").info(
                "manhole: kill -USR2 %d, then nc -U %s", os.getpid(),
                self.manhole_path)
        if args.dump_unit_attributes != "no":
            self._dump_unit_attributes(args.dump_unit_attributes == "all")
        if args.dry_run == "exec":
            self.stopped_before = "run"
            return
        if args.visualize:
            self.visualized = self._visualize()
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
        if args.pdb_on_finish:
            self._pdb_on_finish()

    def _dump_unit_attributes(self, arrays):
        """``--dump-unit-attributes pretty|all`` after initialisation
        (reference __main__.py:665-685)."""
        for u in self.workflow:
            attrs = {}
            for k, v in sorted(u.__dict__.items()):
                if k.startswith("_"):
                    continue
                if not arrays and hasattr(v, "__len__") and \
                        not isinstance(v, (str, bytes)):
                    try:
                        n = len(v)
                    except Exception:  # noqa: BLE001
                        n = 0
                    if n > 32:
                        v = "<%s of length %d>" % (type(v).__name__, n)
                attrs[k] = v
            print(u.name, attrs)

    def _visualize(self):
        """``--visualize``: the workflow graph (DOT) and one rendering of
        every plotter unit, without running the model; returns the files."""
        from veles_amd.plotter import Plotter
        files = []
        dot = self.args.workflow_graph or "%s.dot" % self.workflow.name
        self.workflow.generate_graph(dot, with_data_links=True)
        files.append(dot)
        for u in self.workflow:
            if isinstance(u, Plotter) and not u.disabled:
                try:
                    u.collect()
                    u.render()
                    files.extend(u.files)
                except Exception as e:  # noqa: BLE001 - nothing to draw yet
                    logging.getLogger("Main").warning(
                        "--visualize: %s not rendered (%s)", u.name, e)
        for f in files:
            print("visualize:", f)
        return files

    def _pdb_on_finish(self):
        """``--pdb-on-finish`` (reference launcher.py:688-690): a debugger
        prompt with the finished workflow in scope (only on a terminal)."""
        if not sys.stdin.isatty():
            logging.getLogger("Main").warning(
                "--pdb-on-finish: stdin is not a terminal, no debugger")
            return
        import pdb
        workflow = self.workflow  # noqa: F841 - in the debugger's scope
        pdb.set_trace()

    def run(self):
        from veles_amd import __version__
        from veles_amd.cmdline import make_parser
        from veles_amd.utils.config import root
        args = make_parser().parse_intermixed_args(self.argv)
        self.args = args
        self.stopped_before = None
        if args.background and not daemonize(args.log_file or None):
            return 0   # the original process; the daemon carries on
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
        if args.debug_pickle:
            from veles_amd.utils.pickle2 import setup_pickle_debug
            setup_pickle_debug()
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
        if args.dry_run == "load":
            # stop before the workflow is created (module and config only)
            self.stopped_before = "load"
            return 0
        from veles_amd.genetics.config import fix_config
        fix_config(root)
        module.run(self._load, self._main)
        return 0


def main(argv=None):
    return Main(argv).run()


if __name__ == "__main__":
    sys.exit(main() or 0)
