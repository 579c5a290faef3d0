"""CPU oracle for the register linearizability check — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package; the product path (jepsen/etcd_amd) never does.  PARITY UNPINNED
against outputs of the reference itself (Clojure/Knossos; no JVM here and no
reference fixtures exist for this path): see oracle.h and DESIGN.md.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liboracle.so")

JIT, WGL = 0, 1
# OR into JIT: exact reductions, each checked against plain JIT in tests/
READ_CLOSURE = 0x100
CRASH_SYMMETRY = 0x200
RETIRE = 0x400
DEADLINE_ORDER = 0x800
# the reductions the GPU's search tiers apply (DEADLINE_ORDER since round 2)
JITC = JIT | READ_CLOSURE | CRASH_SYMMETRY | RETIRE | DEADLINE_ORDER

RESULT_DTYPE = np.dtype([
    ("verdict", "<i4"), ("reason", "<i4"), ("fail_op", "<i8"),
    ("fail_prefix_end", "<i8"), ("configs_explored", "<i8"),
    ("max_frontier", "<i8"),
])


class _Opts(ctypes.Structure):
    _fields_ = [("init_version", ctypes.c_int64), ("init_value", ctypes.c_int64),
                ("max_configs_per_key", ctypes.c_int64),
                ("time_budget_ms", ctypes.c_int64), ("flags", ctypes.c_int64)]


_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        vp = ctypes.c_void_p
        L.oracle_check.argtypes = [vp, vp, ctypes.c_int64, ctypes.POINTER(_Opts), vp,
                                   ctypes.c_int, ctypes.c_int]
        L.oracle_check.restype = ctypes.c_int
        L.oracle_check_witness.argtypes = [vp, vp, ctypes.c_int64, ctypes.POINTER(_Opts), vp, vp,
                                           vp, vp, vp, ctypes.c_int]
        L.oracle_check_witness.restype = ctypes.c_int
        L.oracle_check_certificate.argtypes = [vp, vp, ctypes.c_int64, ctypes.POINTER(_Opts),
                                               vp, vp, vp, vp, ctypes.c_int]
        L.oracle_check_certificate.restype = ctypes.c_int
        L.oracle_frontier.argtypes = [vp, ctypes.c_int64, ctypes.POINTER(_Opts), ctypes.c_int,
                                      ctypes.c_int64, vp, ctypes.c_int64, vp]
        L.oracle_frontier.restype = ctypes.c_int
        _lib = L
    return _lib


def check(ops, key_off, algo=JIT, n_threads=1, max_configs=0, init_version=0,
          init_value=-1):
    """Returns (rc, results) with the same layout as the GPU library."""
    ops = np.ascontiguousarray(ops, dtype=np.int64).reshape(-1, 6)
    key_off = np.ascontiguousarray(key_off, dtype=np.int64)
    n = len(key_off) - 1
    out = np.zeros(max(n, 0), dtype=RESULT_DTYPE)
    o = _Opts(init_version, init_value, max_configs, 0, 0)
    rc = lib().oracle_check(ops.ctypes.data_as(ctypes.c_void_p),
                            key_off.ctypes.data_as(ctypes.c_void_p), n,
                            ctypes.byref(o), out.ctypes.data_as(ctypes.c_void_p),
                            algo, n_threads)
    return rc, out


CFG_WORDS = 67


def frontier(ops, stop_op, algo=JITC, max_configs=100000, init_value=-1, init_version=0):
    """The JIT search's frontier just before the :ok return of record
    stop_op: a set of (version, value, pending ops tuple)."""
    ops = np.ascontiguousarray(ops, dtype=np.int64).reshape(-1, 6)
    out = np.zeros((max_configs, CFG_WORDS), dtype=np.int64)
    n = ctypes.c_int64(0)
    o = _Opts(init_version, init_value, 0, 0, 0)
    rc = lib().oracle_frontier(ops.ctypes.data_as(ctypes.c_void_p), len(ops), ctypes.byref(o),
                               algo, int(stop_op), out.ctypes.data_as(ctypes.c_void_p),
                               max_configs, ctypes.byref(n))
    if rc != 0:
        raise ValueError("oracle_frontier: %d" % rc)
    k = min(n.value, max_configs)
    return {(int(r[0]), int(r[1]), tuple(int(v) for v in r[3:3 + r[2]])) for r in out[:k]}, n.value


WIT_OK, WIT_NONE = 1, 0
WIT_CODES = {1: "ok", 0: "none", -1: "bad-position", -2: "not-an-op", -3: "read-unplaceable",
             -4: "inconsistent", -5: "real-time", -6: "missing-ok-op"}


def check_witness(ops, key_off, witness, kind, results=None, init_version=0, init_value=-1,
                  n_threads=8):
    """Certify witnesses (lc_aux) independently: per key WIT_OK, WIT_NONE or
    a negative code (WIT_CODES), plus the length of each rebuilt order.
    `results` (the GPU's lc_key_result array) gives the cut of PREFIX
    witnesses: fail_prefix_end - 1."""
    ops = np.ascontiguousarray(ops, dtype=np.int64).reshape(-1, 6)
    key_off = np.ascontiguousarray(key_off, dtype=np.int64)
    witness = np.ascontiguousarray(witness, dtype=np.int32)
    kind = np.ascontiguousarray(kind, dtype=np.int32)
    n = len(key_off) - 1
    cut = np.full(max(n, 0), -1, dtype=np.int64)
    if results is not None:
        cut = np.ascontiguousarray(results["fail_prefix_end"] - 1, dtype=np.int64)
    st = np.zeros(max(n, 0), dtype=np.int32)
    ln = np.zeros(max(n, 0), dtype=np.int64)
    o = _Opts(init_version, init_value, 0, 0, 0)
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    rc = lib().oracle_check_witness(p(ops), p(key_off), n, ctypes.byref(o), p(witness), p(kind),
                                    p(cut), p(st), p(ln), n_threads)
    if rc != 0:
        raise RuntimeError("oracle_check_witness: %d" % rc)
    return st, ln


CERT_OK, CERT_NONE, CERT_BAD = 1, 0, -1
CERT_KINDS = {0: "none", 1: "dup", 2: "unreach", 3: "claims", 4: "pair", 5: "order", 6: "hall",
              7: "proof"}


def check_certificate(ops, key_off, cert, cert_set, results, init_version=0, init_value=-1,
                      n_threads=8):
    """Check infeasibility certificates (lc_aux, include/lincheck.h) from the
    records alone: per key CERT_OK, CERT_NONE or CERT_BAD.  `results` gives
    each key's cut (fail_prefix_end); cert is int32[4 * n_keys], cert_set
    int32 per record (or None)."""
    ops = np.ascontiguousarray(ops, dtype=np.int64).reshape(-1, 6)
    key_off = np.ascontiguousarray(key_off, dtype=np.int64)
    n = len(key_off) - 1
    cert = np.ascontiguousarray(cert, dtype=np.int32).reshape(-1)
    cset = None if cert_set is None else np.ascontiguousarray(cert_set, dtype=np.int32)
    cut = np.ascontiguousarray(results["fail_prefix_end"], dtype=np.int64)
    st = np.zeros(max(n, 0), dtype=np.int32)
    o = _Opts(init_version, init_value, 0, 0, 0)
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p) if a is not None else None
    rc = lib().oracle_check_certificate(p(ops), p(key_off), n, ctypes.byref(o), p(cert),
                                        p(cset), p(cut), p(st), n_threads)
    if rc != 0:
        raise RuntimeError("oracle_check_certificate: %d" % rc)
    return st
