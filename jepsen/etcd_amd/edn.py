"""Jepsen `history.edn` in, independent-checker result out (SURVEY.md §8(f)
rank 2: check stored Jepsen runs without a JVM).

* `read(path_or_bytes)` parses the history with the native reader
  (include/lincheck_edn.h, csrc/edn.cpp): jepsen.independent's per-key split
  (register.clj:108) and knossos history completion, packed into lc_op
  records — the same records `history.pack` builds from op dicts.
* `check(...)` decides every key in one batched GPU call and returns the
  shape `jepsen.independent/checker` gives (register.clj:108-112):
  {"valid?": ..., "results": {key-edn: {...}}, "failures": [...]}, with the
  failing op rendered from the history's own text.
* `to_edn(history)` writes op dicts (history.py's representation) as a
  Jepsen-style history.edn, one op map per line.

CLI:  python -m jepsen.etcd_amd.edn [--single-key] [--gpus MASK] history.edn
prints the result map as EDN.
"""
import argparse
import ctypes
import mmap
import os
import sys

import numpy as np

from . import abi
from .history import Tuple

LC_EDN_INDEPENDENT = 1
MODEL_FLAGS = {"versioned-register": 0 << 8, "cas-register": 1 << 8, "register": 2 << 8,
               "mutex": 3 << 8}
_bound = False


def _lib():
    global _bound
    L = abi.lib()
    if not _bound:
        vp, i64 = ctypes.c_void_p, ctypes.c_int64
        L.lc_edn_parse.argtypes = [ctypes.c_char_p, ctypes.c_size_t, i64, ctypes.c_int,
                                   ctypes.POINTER(vp), ctypes.c_char_p, ctypes.c_size_t]
        L.lc_edn_parse.restype = ctypes.c_int
        for name in ("lc_edn_n_keys", "lc_edn_n_ops", "lc_edn_n_events"):
            getattr(L, name).argtypes = [vp]
            getattr(L, name).restype = i64
        L.lc_edn_ops.argtypes = [vp]
        L.lc_edn_ops.restype = vp
        L.lc_edn_key_off.argtypes = [vp]
        L.lc_edn_key_off.restype = vp
        L.lc_edn_ops32.argtypes = [vp]
        L.lc_edn_ops32.restype = vp
        L.lc_edn_key_base.argtypes = [vp]
        L.lc_edn_key_base.restype = vp
        L.lc_edn_ops16.argtypes = [vp]
        L.lc_edn_ops16.restype = vp
        L.lc_edn_key.argtypes = [vp, i64]
        L.lc_edn_key.restype = ctypes.c_char_p
        L.lc_edn_op_text.argtypes = [vp, i64, ctypes.c_int]
        L.lc_edn_op_text.restype = ctypes.c_char_p
        L.lc_edn_value.argtypes = [vp, i64, i64]
        L.lc_edn_value.restype = ctypes.c_char_p
        L.lc_edn_free.argtypes = [vp]
        L.lc_edn_free.restype = None
        _bound = True
    return L


class EdnHistory:
    """A parsed history.  `ops` (n, 6) int64 and `key_off` are copies; the
    source text is kept alive for op_text()."""

    def __init__(self, text, independent=True, n_threads=0, model="versioned-register"):
        L = _lib()
        self._text = text  # bytes / mmap: the C side keeps pointers into it
        if isinstance(text, bytes):
            ptr = ctypes.c_char_p(text)  # no copy
        else:
            self._buf = np.frombuffer(text, dtype=np.uint8)  # read-only views too
            ptr = ctypes.cast(self._buf.ctypes.data, ctypes.c_char_p)
        h = ctypes.c_void_p()
        err = ctypes.create_string_buffer(256)
        rc = L.lc_edn_parse(ptr, len(text),
                            (LC_EDN_INDEPENDENT if independent else 0) | MODEL_FLAGS[model],
                            n_threads,
                            ctypes.byref(h), err, 256)
        if rc != 0:
            raise abi.LcError(rc, err.value.decode())
        self._h = h
        self.n_keys = L.lc_edn_n_keys(h)
        self.n_events = L.lc_edn_n_events(h)
        n = L.lc_edn_n_ops(h)
        self.ops = np.ctypeslib.as_array(
            ctypes.cast(L.lc_edn_ops(h), ctypes.POINTER(ctypes.c_int64)), shape=(max(n, 1) * 6,)
        )[: n * 6].reshape(n, 6).copy() if n else np.zeros((0, 6), dtype=np.int64)
        self.key_off = np.ctypeslib.as_array(
            ctypes.cast(L.lc_edn_key_off(h), ctypes.POINTER(ctypes.c_int64)),
            shape=(self.n_keys + 1,)).copy()
        self.keys = [L.lc_edn_key(h, i).decode() for i in range(self.n_keys)]

    def ops32(self):
        """The records as lc_op32 ((n, 6) int32) and the keys' bases: what
        lc_check32 takes (include/lincheck_edn.h, lc_edn_ops32)."""
        L = _lib()
        n = len(self.ops)
        p32, pb = L.lc_edn_ops32(self._h), L.lc_edn_key_base(self._h)
        o32 = np.ctypeslib.as_array(ctypes.cast(p32, ctypes.POINTER(ctypes.c_int32)),
                                    shape=(max(n, 1) * 6,))[: n * 6].reshape(n, 6).copy()
        base = np.ctypeslib.as_array(ctypes.cast(pb, ctypes.POINTER(ctypes.c_int64)),
                                     shape=(max(self.n_keys, 1),))[: self.n_keys].copy()
        return o32, base

    def ops16(self):
        """The records as lc_op16 ((n, 4) uint32) and the keys' bases: what
        lc_check16 takes (include/lincheck_edn.h, lc_edn_ops16), or None when
        a value id does not fit 15 bits (use ops32)."""
        L = _lib()
        n = len(self.ops)
        p16 = L.lc_edn_ops16(self._h)
        if not p16:
            return None
        o16 = np.ctypeslib.as_array(ctypes.cast(p16, ctypes.POINTER(ctypes.c_uint32)),
                                    shape=(max(n, 1) * 4,))[: n * 4].reshape(n, 4).copy()
        return o16, self.ops32()[1]

    def op_text(self, rec, which=0):
        """EDN text of record rec's :invoke (0) or completion (1)."""
        t = _lib().lc_edn_op_text(self._h, rec, which)
        return t.decode() if t is not None else None

    def value(self, key, vid):
        t = _lib().lc_edn_value(self._h, key, vid)
        return t.decode() if t is not None else None

    def close(self):
        if getattr(self, "_h", None):
            _lib().lc_edn_free(self._h)
            self._h = None

    __del__ = close


def read(src, independent=True, n_threads=0, model="versioned-register"):
    """Parse a history.edn given as a path, bytes or str."""
    if isinstance(src, str) and os.path.exists(src):
        with open(src, "rb") as fh:
            size = os.fstat(fh.fileno()).st_size
            if size == 0:
                return EdnHistory(b"", independent, n_threads, model)
            # read-only and prefaulted: first-touch faults from the parse
            # threads would cost more than the scan itself
            mm = mmap.mmap(fh.fileno(), 0, flags=mmap.MAP_SHARED | getattr(mmap, "MAP_POPULATE", 0),
                           prot=mmap.PROT_READ)
        return EdnHistory(mm, independent, n_threads, model)
    if isinstance(src, str):
        src = src.encode()
    return EdnHistory(bytes(src), independent, n_threads, model)


def check(src, device_mask=0, independent=True, ctx=None, opts=None, model="versioned-register"):
    """Decide every key of a history.edn on the GPU.  Returns
    (result map, EdnHistory); the map has independent/checker's shape with
    EDN key texts as keys."""
    h = src if isinstance(src, EdnHistory) else read(src, independent, model=model)
    if opts is None:
        # the lock starts free; a key one workgroup's search cannot finish
        # within its budget gets the whole GPU (LC_FLAG_WHOLE_GPU), as knossos
        # would keep searching until it ran out of memory
        opts = abi.default_opts(init_value=0 if model == "mutex" else abi.LC_NIL,
                                flags=abi.LC_FLAG_WHOLE_GPU)
    own = ctx is None
    ctx = ctx or abi.Context(device_mask)
    try:
        # the drop-in's call: 16-byte records across PCIe when every value id
        # fits 15 bits (ABI 5), else 24-byte ones (ABI 4)
        p16 = h.ops16()
        if p16 is not None:
            rc, res = ctx.check16(p16[0], h.key_off, p16[1], opts=opts, raise_on_error=False)
        else:
            o32, base = h.ops32()
            rc, res = ctx.check32(o32, h.key_off, base, opts=opts, raise_on_error=False)
        if rc != 0:
            raise abi.LcError(rc, ctx.last_error())
    finally:
        if own:
            ctx.close()
    results, failures = {}, []
    for k, name in enumerate(h.keys):
        v = int(res["verdict"][k])
        r = {"valid?": True if v == 1 else False if v == 0 else "unknown",
             "analyzer": "mi355x"}
        if v == 0 and res["fail_op"][k] >= 0:
            rec = int(h.key_off[k] + res["fail_op"][k])
            r["op"] = h.op_text(rec, 1) or h.op_text(rec, 0)
            r["fail-prefix-end"] = int(res["fail_prefix_end"][k])
        elif v == -1:
            r["reason"] = int(res["reason"][k])
        if v == 0:
            failures.append(name)
        results[name] = r
    vs = [r["valid?"] for r in results.values()]
    valid = False if any(x is False for x in vs) else "unknown" if "unknown" in vs else True
    return {"valid?": valid, "results": results, "failures": failures}, h


# ------------------------------------------------------------------ writer
_KW_FIELDS = ("type", "f", "error")


def _edn(v):
    if v is None:
        return "nil"
    if v is True:
        return "true"
    if v is False:
        return "false"
    if isinstance(v, int):
        return str(v)
    if isinstance(v, float):
        return repr(v)
    if isinstance(v, str):
        return '"%s"' % v.replace("\\", "\\\\").replace('"', '\\"')
    if isinstance(v, Tuple):
        return "[%s %s]" % (_edn(v.key), _edn(v.value))
    if isinstance(v, (list, tuple)):
        return "[%s]" % " ".join(_edn(x) for x in v)
    if isinstance(v, dict):
        return "{%s}" % ", ".join("%s %s" % (_edn(a), _edn(b)) for a, b in v.items())
    raise TypeError("no EDN form for %r" % (v,))


def op_edn(op):
    """One op dict as a Jepsen op map; type/f/error and string processes are
    keywords."""
    parts = []
    for k, v in op.items():
        if (k in _KW_FIELDS or k == "process") and isinstance(v, str):
            s = ":" + v.lstrip(":")
        else:
            s = _edn(v)
        parts.append(":%s %s" % (k, s))
    return "{%s}" % ", ".join(parts)


def to_edn(history):
    """A Jepsen history.edn: one op map per line."""
    return "".join(op_edn(op) + "\n" for op in history)


def render(result):
    """The result map as EDN text (op texts are already EDN)."""
    def val(x):
        if x is True or x is False or x is None:
            return _edn(x)
        if isinstance(x, str) and x == "unknown":
            return ":unknown"
        return str(x)

    res = []
    for k, r in result["results"].items():
        fields = ["%s %s" % (":valid?", val(r["valid?"])), ":analyzer :mi355x"]
        if "op" in r:
            fields.append(":op %s" % r["op"])
        if "fail-prefix-end" in r:
            fields.append(":fail-prefix-end %d" % r["fail-prefix-end"])
        if "reason" in r:
            fields.append(":reason %d" % r["reason"])
        res.append("%s {%s}" % (k, ", ".join(fields)))
    return "{:valid? %s,\n :results {%s},\n :failures [%s]}" % (
        val(result["valid?"]), ",\n           ".join(res), " ".join(result["failures"]))


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("history")
    ap.add_argument("--single-key", action="store_true",
                    help="values are not independent tuples: one key")
    ap.add_argument("--model", default="versioned-register", choices=sorted(MODEL_FLAGS),
                    help="knossos model (lock workload: mutex with --single-key)")
    ap.add_argument("--gpus", type=lambda s: int(s, 0), default=0,
                    help="device mask (0 = all GPUs)")
    a = ap.parse_args(argv)
    result, h = check(a.history, device_mask=a.gpus, independent=not a.single_key, model=a.model)
    print(render(result))
    return 0 if result["valid?"] is True else 1


if __name__ == "__main__":
    sys.exit(main())
