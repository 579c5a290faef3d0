"""timeline.html for one key's subhistory: the `:timeline (timeline/html)`
half of the checker the drop-in replaces (register.clj:109-112).

jepsen.checker.timeline/html (jepsen 0.3.x, not in /root/reference) renders
a history as an HTML page with one column per process and one box per
operation, spanning its invocation to its completion, coloured by completion
type, with the op maps in a tooltip; it always returns {:valid? true}.  This
is a host-side restatement of that idea for the Python mirror
(checker.RegisterChecker(timeline_dir=...)); the Clojure shim calls jepsen's
own renderer instead.  Not byte-identical to jepsen's page (parity
unpinned: jepsen is not available here), and never on the verdict path.

Addition over jepsen's page: the counterexample op of an invalid key (the
:ok op whose return empties the linearization frontier) is outlined, and
everything returning after that point is dimmed.
"""
import html
import os

from .history import _kw, is_client

# row height per history index, column width per process (px)
_ROW = 16
_COL = 110
_STYLE = """
body { font-family: sans-serif; font-size: 11px; }
.ops { position: relative; }
.proc { position: absolute; top: 0; font-weight: bold; text-align: center; }
.op { position: absolute; overflow: hidden; border-radius: 3px; padding: 1px 3px;
      box-sizing: border-box; border: 1px solid #888; white-space: nowrap; }
.ok { background: #B3F3B5; } .info { background: #FFE0A0; } .fail { background: #F3B3B3; }
.invoke { background: #EEEEEE; }
.cex { outline: 3px solid #D00000; z-index: 2; }
.after { opacity: 0.35; }
"""


def _fmt(v):
    if v is None:
        return "nil"
    if isinstance(v, (list, tuple)):
        return "[" + " ".join(_fmt(x) for x in v) + "]"
    if isinstance(v, str):
        return ":" + v
    return str(v)


def _op_text(op):
    keys = ("index", "type", "process", "f", "value", "error")
    return "{" + ", ".join(":%s %s" % (k, _fmt(op[k])) for k in keys if k in op) + "}"


def pairs(subhistory):
    """(invoke, completion or None) per client operation, in invoke order;
    indices are the ops' :index (or positions when absent)."""
    open_, out = {}, []
    for pos, op in enumerate(subhistory):
        if not is_client(op):
            continue
        op = dict(op)
        op.setdefault("index", pos)
        op["type"] = _kw(op.get("type"))
        p = op["process"]
        if op["type"] == "invoke":
            open_[p] = len(out)
            out.append([op, None])
        elif p in open_:
            out[open_.pop(p)][1] = op
    return [tuple(x) for x in out]


def render(subhistory, title="", cex_index=None):
    """The HTML page.  cex_index: history index of the counterexample op's
    completion (an invalid key's fail-prefix-end), or None."""
    ps = pairs(subhistory)
    procs = sorted({inv["process"] for inv, _ in ps}, key=lambda p: (str(type(p)), p))
    col = {p: i for i, p in enumerate(procs)}
    lo = min((inv["index"] for inv, _ in ps), default=0)
    hi = max((c["index"] if c else inv["index"] for inv, c in ps), default=0)
    boxes = []
    for inv, comp in ps:
        t = comp["type"] if comp else "invoke"
        end = comp["index"] if comp else hi + 1
        cls = ["op", t]
        if cex_index is not None and comp is not None and comp["index"] == cex_index:
            cls.append("cex")
        elif cex_index is not None and end > cex_index:
            cls.append("after")
        tip = _op_text(inv) + ("\n" + _op_text(comp) if comp else "")
        label = "%s %s" % (_kw(inv.get("f", "")), _fmt((comp or inv).get("value")))
        boxes.append('<div class="%s" style="left:%dpx;top:%dpx;width:%dpx;height:%dpx" '
                     'title="%s">%s</div>'
                     % (" ".join(cls), col[inv["process"]] * _COL,
                        _ROW + (inv["index"] - lo) * _ROW, _COL - 4,
                        max(_ROW, (end - inv["index"]) * _ROW),
                        html.escape(tip), html.escape(label)))
    heads = "".join('<div class="proc" style="left:%dpx;width:%dpx">%s</div>'
                    % (i * _COL, _COL - 4, html.escape(str(p))) for i, p in enumerate(procs))
    height = _ROW * (hi - lo + 3)
    return ("<!DOCTYPE html>\n<html><head><meta charset=\"utf-8\"><title>%s</title>"
            "<style>%s</style></head><body><h1>%s</h1>"
            "<div class=\"ops\" style=\"height:%dpx;width:%dpx\">%s%s</div></body></html>\n"
            % (html.escape(title), _STYLE, html.escape(title), height,
               _COL * max(1, len(procs)), heads, "".join(boxes)))


def write(path, subhistory, title="", cex_index=None):
    """Render into `path` (directories created).  Returns jepsen's result
    for the timeline checker, {"valid?": True}, plus the file written."""
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    with open(path, "w") as f:
        f.write(render(subhistory, title, cex_index))
    return {"valid?": True, "file": path}
