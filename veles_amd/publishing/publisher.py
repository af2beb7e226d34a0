"""Publisher: a Markdown report of a finished run (reference
veles/publishing/publisher.py:57-271 + markdown_backend.py).

Gathered: workflow name / checksum / device, the config tree, the results
(``gather_results``), per-unit timing statistics, the unit graph (DOT),
loader class statistics, plots written by the plotting units, and the
kernel library build info.  PDF / Confluence backends of the reference are
out of scope (no weasyprint / network); HTML is Markdown rendered by any
viewer.
"""
from __future__ import annotations

import datetime
import json
import os

from veles_amd.units import Unit
from veles_amd.utils.config import get, root
from veles_amd.utils.json_encoders import NumpyJSONEncoder

__all__ = ["Publisher"]


class Publisher(Unit):
    MAPPING = "publisher"

    def __init__(self, workflow, **kwargs):
        kwargs.setdefault("view_group", "SERVICE")
        super().__init__(workflow, **kwargs)
        self.output = kwargs.get("output", "report.md")
        self.backends = kwargs.get("backends", {"markdown": {}})
        self.plotters = list(kwargs.get("plotters", []))

    def run(self):
        if get(root.common.disable.publishing, False):
            return
        self.publish()

    def gather_info(self):
        wf = self.workflow
        info = {"name": getattr(wf, "name", type(wf).__name__),
                "class": type(wf).__name__,
                "checksum": getattr(wf, "checksum", ""),
                "device": str(getattr(wf, "device", None)),
                "date": datetime.datetime.now().isoformat(timespec="seconds"),
                "results": {}, "stats": [], "plots": [], "loader": {}}
        try:
            info["results"] = wf.gather_results()
        except Exception as e:  # results are optional in a report
            info["results"] = {"error": str(e)}
        for u in wf:
            t = getattr(u, "total_run_time", None)
            n = getattr(u, "_run_calls", None)
            if t:
                info["stats"].append((u.name, t, n))
        info["stats"].sort(key=lambda r: -r[1])
        ld = getattr(wf, "loader", None)
        if ld is not None:
            info["loader"] = {
                "class": type(ld).__name__,
                "class_lengths": list(getattr(ld, "class_lengths", [])),
                "minibatch_size": getattr(ld, "max_minibatch_size", None),
                "normalization": getattr(ld, "normalization_type", None)}
        for p in self.plotters + [u for u in wf if hasattr(u, "files") and
                                  u not in self.plotters]:
            info["plots"].extend(getattr(p, "files", []))
        try:
            g = wf.generate_graph(None, write_on_disk=False)
            if isinstance(g, (tuple, list)):
                g = next((x for x in g if isinstance(x, str) and
                          x.startswith("digraph")), None)
            info["graph"] = g
        except Exception:
            info["graph"] = None
        try:
            info["config"] = root.__content__ and json.loads(json.dumps(
                {k: v for k, v in root.__content__.items()
                 if k != "common"}, cls=NumpyJSONEncoder, default=str))
        except Exception:
            info["config"] = None
        return info

    def render_markdown(self, info):
        out = ["# %s" % info["name"], "",
               "* workflow class: `%s`" % info["class"],
               "* checksum: `%s`" % info["checksum"],
               "* device: `%s`" % info["device"],
               "* date: %s" % info["date"], ""]
        if info["loader"]:
            out += ["## Data", ""] + ["* %s: %s" % kv for kv in
                                      info["loader"].items()] + [""]
        out += ["## Results", "", "| metric | value |", "|---|---|"]
        for k, v in sorted(info["results"].items()):
            if k in ("Output", "Epoch history"):
                continue
            out.append("| %s | %s |" % (k, json.dumps(
                v, cls=NumpyJSONEncoder, default=str)[:200]))
        hist = info["results"].get("Epoch history")
        if hist:
            keys = sorted({k for h in hist for k in h})
            out += ["", "### Epoch history", "",
                    "| " + " | ".join(keys) + " |",
                    "|" + "---|" * len(keys)]
            for h in hist:
                out.append("| " + " | ".join(
                    "%.4g" % h[k] if isinstance(h.get(k), float)
                    else str(h.get(k, "")) for k in keys) + " |")
        if info["stats"]:
            out += ["", "## Unit run time", "", "| unit | seconds | calls |",
                    "|---|---|---|"]
            out += ["| %s | %.4f | %s |" % r for r in info["stats"][:30]]
        if info["plots"]:
            out += ["", "## Plots", ""]
            base = os.path.dirname(os.path.abspath(self.output))
            for p in info["plots"]:
                rel = os.path.relpath(p, base)
                out.append("![%s](%s)" % (os.path.basename(p), rel)
                           if p.endswith((".png", ".svg", ".jpg")) else
                           "* [%s](%s)" % (os.path.basename(p), rel))
        if info.get("config"):
            out += ["", "## Configuration", "", "```json",
                    json.dumps(info["config"], indent=1)[:20000], "```"]
        if info.get("graph"):
            out += ["", "## Workflow graph (DOT)", "", "```dot",
                    info["graph"], "```"]
        return "\n".join(out) + "\n"

    def publish(self):
        info = self.gather_info()
        text = self.render_markdown(info)
        d = os.path.dirname(os.path.abspath(self.output))
        os.makedirs(d, exist_ok=True)
        with open(self.output, "w") as f:
            f.write(text)
        self.info("Report written to %s", self.output)
        return self.output
