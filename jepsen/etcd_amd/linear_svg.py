"""linear.svg for an invalid key: the picture jepsen's checker/linearizable
writes next to a failed analysis (register.clj:110-111 builds that checker;
jepsen 0.3.x calls knossos.linear.report/render-analysis! on an invalid
result, into the key's store directory).  knossos is not in this container,
so this is a host-side restatement of the same figure for the Python mirror
(checker.RegisterChecker(timeline_dir=...)); the Clojure shim calls knossos's
own renderer.  Not byte-identical (parity unpinned); never on the verdict path.

The figure, as knossos draws it: one row per process; every op that matters
to the failure — the last :ok before it (:previous-ok), the ops still pending
in the reported configuration, the failing op, and every op on a final path —
as a bar from its invocation to its completion on a compressed time axis
(distinct call/return indices only); then each final path (:final-paths,
at most 10) as a line through the ops it tries to linearize, in order, each
step labelled with the model it reaches, the inconsistent last step in red.
"""
import html
import os

from .abi import LC_INF

_ROW = 34      # px per process row
_STEP = 26     # px per distinct time point
_LEFT = 90     # process labels
_TOP = 40
_PATH_DY = 9   # vertical offset between successive final paths


def _fmt(v):
    if v is None:
        return "nil"
    if isinstance(v, (list, tuple)):
        return "[" + " ".join(_fmt(x) for x in v) + "]"
    if isinstance(v, str):
        return ":" + v
    return str(v)


def _model_text(m):
    if m is None:
        return ""
    if "inconsistent" in m:
        return str(m["inconsistent"])
    return "{:version %s, :value %s}" % (_fmt(m.get("version")), _fmt(m.get("value")))


def _op_label(op):
    f = op.get("f", "")
    f = f[1:] if isinstance(f, str) and f.startswith(":") else f
    return "%s %s" % (f, _fmt(op.get("value")))


def render(done, analysis, title=""):
    """SVG text.  done: the key's completed ops (history.complete records, as
    diagnostics.invalid_analysis takes them); analysis: the key's :linear map
    (op, previous-ok, configs, final-paths)."""
    # op maps in the analysis are the records' own invoke/completion dicts
    by_id = {}
    for i, r in enumerate(done):
        for k in ("invoke", "completion"):
            if r.get(k) is not None:
                by_id[id(r[k])] = i
    want = []

    def add(op):
        i = by_id.get(id(op)) if op is not None else None
        if i is not None and i not in want:
            want.append(i)

    add(analysis.get("previous-ok"))
    for cfg in analysis.get("configs", []):
        for op in cfg.get("pending", []):
            add(op)
    add(analysis.get("op"))
    paths = analysis.get("final-paths", [])
    for path in paths:
        for step in path:
            add(step.get("op"))
    if not want:
        return _svg(title, 200, 60, [])
    fail_i = by_id.get(id(analysis.get("op")))
    # compressed time axis over the drawn ops' calls and returns
    # a crashed op's bar runs to just past the last return drawn
    inf = max((r["ret"] for r in done if r["ret"] != LC_INF), default=0) + 1
    pts = sorted({done[i]["call"] for i in want} |
                 {min(done[i]["ret"], inf) for i in want})
    x_of = {t: _LEFT + 20 + k * _STEP for k, t in enumerate(pts)}
    procs = sorted({done[i]["invoke"].get("process") for i in want},
                   key=lambda p: (str(type(p)), p))
    row = {p: k for k, p in enumerate(procs)}
    out = []
    for p, k in row.items():
        y = _TOP + k * _ROW
        out.append('<text x="4" y="%d" class="proc">process %s</text>' % (y + 16, html.escape(str(p))))
    centre = {}
    for i in want:
        r = done[i]
        x0, x1 = x_of[r["call"]], x_of[min(r["ret"], inf)]
        y = _TOP + row[r["invoke"].get("process")] * _ROW
        crashed = r["ret"] == LC_INF
        cls = "fail" if i == fail_i else ("info" if crashed else "ok")
        op = r["completion"] if r.get("completion") is not None and not crashed else r["invoke"]
        out.append('<rect x="%d" y="%d" width="%d" height="22" rx="3" class="%s"/>'
                   % (x0, y, max(8, x1 - x0), cls))
        out.append('<text x="%d" y="%d" class="op">%s</text>'
                   % (x0 + 3, y + 15, html.escape(_op_label(op))))
        centre[i] = ((x0 + max(x0 + 8, x1)) // 2, y + 11)
    for n, path in enumerate(paths):
        dy = (n - len(paths) / 2.0) * _PATH_DY / max(1, len(paths) / 2.0)
        prev = None
        for s, step in enumerate(path):
            i = by_id.get(id(step.get("op")))
            if i is None or i not in centre:
                continue
            x, y = centre[i]
            y = int(y + dy)
            bad = "inconsistent" in (step.get("model") or {})
            if prev is not None:
                out.append('<line x1="%d" y1="%d" x2="%d" y2="%d" class="%s"/>'
                           % (prev[0], prev[1], x, y, "badpath" if bad else "path"))
            out.append('<circle cx="%d" cy="%d" r="3" class="%s"/>' % (x, y, "bad" if bad else "pt"))
            if s > 0:
                out.append('<text x="%d" y="%d" class="%s">%s</text>'
                           % (x + 5, y - 4, "badmodel" if bad else "model",
                              html.escape(_model_text(step.get("model")))))
            prev = (x, y)
    width = _LEFT + 40 + _STEP * len(pts) + 260
    height = _TOP + _ROW * len(procs) + 30
    return _svg(title, width, height, out)


_STYLE = """
.proc { font: bold 11px sans-serif; }
.op { font: 10px monospace; }
.ok { fill: #B3F3B5; stroke: #6a6; } .info { fill: #FFE0A0; stroke: #ca6; }
.fail { fill: #F3B3B3; stroke: #c33; stroke-width: 2; }
.path { stroke: #3060D0; stroke-width: 1.5; } .badpath { stroke: #D00000; stroke-width: 1.5; stroke-dasharray: 4 2; }
.pt { fill: #3060D0; } .bad { fill: #D00000; }
.model { font: 9px monospace; fill: #3060D0; } .badmodel { font: 9px monospace; fill: #D00000; }
.title { font: bold 13px sans-serif; }
"""


def _svg(title, width, height, body):
    return ('<?xml version="1.0" encoding="UTF-8"?>\n'
            '<svg xmlns="http://www.w3.org/2000/svg" width="%d" height="%d">'
            '<style>%s</style><text x="4" y="18" class="title">%s</text>%s</svg>\n'
            % (width, height, _STYLE, html.escape(title), "".join(body)))


def write(path, done, analysis, title=""):
    """Render into `path` (directories created); returns the path."""
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    with open(path, "w") as f:
        f.write(render(done, analysis, title))
    return path
