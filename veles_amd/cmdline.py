"""Command-line surface (reference: veles/cmdline.py:61-278; SURVEY
Appendix A).  Positional ``workflow config [root.x=y ...]``; every class may
contribute flags through ``init_parser`` (CommandLineArgumentsRegistry)."""
from __future__ import annotations

import argparse

__all__ = ["CommandLineArgumentsRegistry", "make_parser", "kwargs_to_argv"]


class CommandLineArgumentsRegistry(type):
    classes = []

    def __init__(cls, name, bases, clsdict):
        super().__init__(name, bases, clsdict)
        if "init_parser" in clsdict:
            CommandLineArgumentsRegistry.classes.append(cls)


def make_parser():
    p = argparse.ArgumentParser(
        prog="python -m veles_amd",
        description="veles_amd: MI355X-native dataflow deep-learning engine")
    p.add_argument("workflow", nargs="?", help="workflow module (.py)")
    p.add_argument("config", nargs="?", default="",
                   help="config module (.py); '-' = <workflow>_config.py")
    p.add_argument("config_list", nargs="*",
                   help="root.x.y=value overrides (Python expressions)")
    p.add_argument("--no-logo", action="store_true")
    p.add_argument("--version", action="store_true")
    p.add_argument("-v", "--verbosity", default="info",
                   choices=["debug", "info", "warning", "error"])
    p.add_argument("--debug", default="",
                   help="comma-separated class names logged at DEBUG")
    p.add_argument("--debug-pickle", action="store_true",
                   help="name the attribute that fails to (un)pickle; on a "
                        "terminal, open the post-mortem debugger there")
    p.add_argument("-r", "--random-seed", default="",
                   help="seed[,seed...] | file:count[:dtype] | -")
    p.add_argument("-w", "--snapshot", default="",
                   help="resume from a snapshot file")
    p.add_argument("--dump-config", action="store_true")
    p.add_argument("--dry-run", default="no",
                   choices=["load", "init", "exec", "no"],
                   help="load: stop before creating the workflow; init: "
                        "before initialising it; exec: before running it")
    p.add_argument("--visualize", action="store_true",
                   help="initialise, then write the workflow graph and "
                        "render every plotter once instead of running")
    p.add_argument("--workflow-graph", default="")
    p.add_argument("--dump-unit-attributes", default="no",
                   choices=["no", "pretty", "all"])
    p.add_argument("--optimize", default="",
                   help="N[:G] genetic hyper-parameter search")
    p.add_argument("--ensemble-train", default="", help="N:ratio")
    p.add_argument("--ensemble-test", default="", help="ensemble file")
    p.add_argument("-b", "--background", action="store_true",
                   help="run detached as a daemon (forks before any GPU "
                        "call; output to --log-file)")
    p.add_argument("-t", "--test", action="store_true",
                   help="test (inference) mode")
    p.add_argument("-p", "--matplotlib-backend", default=None,
                   help="plot backend; '' disables every plotter")
    p.add_argument("--no-graphics-client", action="store_true",
                   help="disable every plotter")
    p.add_argument("--html-help", action="store_true",
                   help="print this help as an HTML page and exit")
    p.add_argument("--pdb-on-finish", action="store_true",
                   help="open pdb with the finished workflow in scope")
    p.add_argument("-s", "--stealth", action="store_true")
    p.add_argument("-f", "--log-file", default="")
    p.add_argument("--log-file-pid", action="store_true")
    p.add_argument("-i", "--log-id", default="")
    p.add_argument("--result-file", default="")
    p.add_argument("-a", "--backend", default="auto",
                   choices=["auto", "hip", "cpu", "numpy"])
    p.add_argument("-d", "--device", default="",
                   help="device id(s) / spec, e.g. 0 or 0-7 or 0,2x2")
    p.add_argument("--gpus", default="",
                   help="spawn one data-parallel rank per listed GPU")
    p.add_argument("--nnodes", type=int, default=1,
                   help="nodes in a multi-node --gpus job (each node runs "
                        "the same command with its own --node-rank)")
    p.add_argument("--node-rank", type=int, default=0)
    p.add_argument("--master-addr", default=None,
                   help="rendezvous host of global rank 0 (multi-node)")
    p.add_argument("--master-port", type=int, default=None)
    p.add_argument("--force-cpu", default="",
                   help="comma-separated units pinned to the CPU")
    p.add_argument("--sync-run", action="store_true")
    p.add_argument("--fault-inject-prob", type=float, default=0.0)
    p.add_argument("--respawn", type=int, default=0,
                   help="restart failed rank groups N times from the "
                        "latest snapshot")
    p.add_argument("--job-timeout", type=float, default=0.0,
                   help="minutes a training step (or a collective) may "
                        "take before the rank aborts for a respawn")
    p.add_argument("--respawn-shrink", action="store_true",
                   help="on respawn, drop the failed ranks' GPUs and keep "
                        "the global batch by gradient accumulation")
    p.add_argument("--trace-events", default="",
                   help="write a Chrome-trace JSON of unit events here")
    p.add_argument("--train-ratio", type=float, default=1.0)
    p.add_argument("--manhole", action="store_true",
                   help="on SIGUSR2 serve a Python console into the "
                        "workflow on /tmp/veles_amd_manhole_<pid>.sock")
    for cls in CommandLineArgumentsRegistry.classes:
        try:
            cls.init_parser(p)
        except argparse.ArgumentError:
            pass
    return p


def kwargs_to_argv(**kwargs):
    """``veles(workflow, config, foo_bar=1)`` -> argv (reference
    cmdline.py:252-278)."""
    argv = []
    for k, v in kwargs.items():
        flag = "--" + k.replace("_", "-")
        if v is True:
            argv.append(flag)
        elif v is False or v is None:
            continue
        else:
            argv.extend([flag, str(v)])
    return argv
