"""ctypes binding of liblincheck.so (include/lincheck.h, include/lincheck_synth.h).

This is the build's own library, loaded in-process.  It exposes the GPU
checker (lc_*) and the seeded synthetic-history generator (lc_synth_*).
Loading fails loudly when the HIP library is missing, and when it was built
from other sources than the tree it is loaded from (lc_build_id() against
csrc/build_id.py): there is no fallback and no stale binary.
"""
import ctypes
import importlib.util
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# LINCHECK_LIB: dev-only override (A/B builds of the same ABI in tools/)
LIB_PATH = os.environ.get("LINCHECK_LIB") or os.path.join(_HERE, "liblincheck.so")

LC_F_READ, LC_F_WRITE, LC_F_CAS = 0, 1, 2
LC_NIL = -1
LC_INF = (1 << 63) - 1
LC_VALID, LC_INVALID, LC_UNKNOWN = 1, 0, -1

REASONS = {
    0: "none",
    1: "nonlinearizable",
    2: "config-budget",
    3: "window-overflow",
    4: "malformed",
    5: "unknown-f",
    7: "time-budget",
    6: "frontier-lds",
}
LC_REASON_NONLINEARIZABLE = 1
LC_REASON_CONFIG_BUDGET = 2
LC_REASON_WINDOW_OVERFLOW = 3
LC_REASON_MALFORMED = 4
LC_REASON_UNKNOWN_F = 5
LC_FLAG_NO_HBM_RETRY = 1
LC_FLAG_NO_FAST_PATH = 2
LC_FLAG_NO_GAP_TIER = 4
LC_FLAG_WHOLE_GPU = 8
LC_FLAG_NO_TIMING = 16
LC_WITNESS_NONE, LC_WITNESS_FULL, LC_WITNESS_PREFIX = 0, 1, 2
LC_CERT_NONE, LC_CERT_DUP, LC_CERT_UNREACH, LC_CERT_CLAIMS, LC_CERT_PAIR, LC_CERT_ORDER, \
    LC_CERT_HALL, LC_CERT_PROOF = range(8)

# lc_op: 6 x int64 (f, value, expected, version, call, ret); arrays are (n, 6).
# lc_op32 (ABI 4): the same fields as 6 x 32 bits, arrays (n, 6) int32 with
# call / ret holding the uint32 bit patterns (LC_INF32 = 0xFFFFFFFF reads -1).
LC_INF32 = 0xFFFFFFFF
OP_FIELDS = ("f", "value", "expected", "version", "call", "ret")
RESULT_DTYPE = np.dtype([
    ("verdict", "<i4"), ("reason", "<i4"), ("fail_op", "<i8"),
    ("fail_prefix_end", "<i8"), ("configs_explored", "<i8"),
    ("max_frontier", "<i8"),
])
assert RESULT_DTYPE.itemsize == 40


class LcOpts(ctypes.Structure):
    _fields_ = [("init_version", ctypes.c_int64), ("init_value", ctypes.c_int64),
                ("max_configs_per_key", ctypes.c_int64),
                ("time_budget_ms", ctypes.c_int64), ("flags", ctypes.c_int64)]


class LcStats(ctypes.Structure):
    _fields_ = [("kernel_ms", ctypes.c_double), ("hbm_kernel_ms", ctypes.c_double),
                ("total_ms", ctypes.c_double), ("n_keys", ctypes.c_int64),
                ("n_ops", ctypes.c_int64), ("n_hbm_keys", ctypes.c_int64),
                ("n_devices", ctypes.c_int64), ("fast_kernel_ms", ctypes.c_double),
                ("jit_kernel_ms", ctypes.c_double), ("n_jit_keys", ctypes.c_int64),
                ("gap_kernel_ms", ctypes.c_double), ("n_gap_keys", ctypes.c_int64),
                ("n_malformed", ctypes.c_int64)]


class LcDeviceStats(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("pinned", ctypes.c_int32),
                ("key_begin", ctypes.c_int64), ("key_end", ctypes.c_int64),
                ("h2d_bytes", ctypes.c_int64), ("h2d_ms", ctypes.c_double),
                ("kernel_ms", ctypes.c_double), ("total_ms", ctypes.c_double)]


class LcCallProfile(ctypes.Structure):
    _fields_ = [("total_ms", ctypes.c_double), ("checked_ms", ctypes.c_double),
                ("planned_ms", ctypes.c_double), ("first_start_ms", ctypes.c_double),
                ("last_start_ms", ctypes.c_double), ("first_end_ms", ctypes.c_double),
                ("last_end_ms", ctypes.c_double), ("joined_ms", ctypes.c_double),
                ("whole_gpu_ms", ctypes.c_double), ("n_devices", ctypes.c_int64),
                ("n_chunks", ctypes.c_int64)]


class LcTotals(ctypes.Structure):
    _fields_ = [("calls", ctypes.c_int64), ("timed_calls", ctypes.c_int64),
                ("fast_kernel_ms", ctypes.c_double), ("kernel_ms", ctypes.c_double)]


class LcAux(ctypes.Structure):
    _fields_ = [("witness", ctypes.c_void_p), ("witness_kind", ctypes.c_void_p),
                ("certificate", ctypes.c_void_p), ("certificate_set", ctypes.c_void_p)]


class LcSynthParams(ctypes.Structure):
    _fields_ = [("n_keys", ctypes.c_int64), ("ops_per_key", ctypes.c_int64),
                ("concurrency", ctypes.c_int32), ("n_values", ctypes.c_int32),
                ("p_info", ctypes.c_double), ("p_anomaly", ctypes.c_double),
                ("seed", ctypes.c_uint64), ("info_frac", ctypes.c_double)]


_lib = None


def source_build_id():
    """Hash of the csrc/ + include/ sources in this tree (csrc/build_id.py)."""
    spec = importlib.util.spec_from_file_location(
        "lincheck_build_id", os.path.join(_HERE, "csrc", "build_id.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m.build_id()


def lib():
    """Load liblincheck.so once; raise if it has not been built, or was built
    from sources other than this tree's."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                "liblincheck.so not built (%s); run `python -c 'import "
                "__graft_entry__ as g; g.build()'` — there is no CPU fallback" % LIB_PATH)
        # torch ships its own HIP runtime (torch/lib/libamdhip64.so) next to
        # the system one this library links; torch only initialises its GPU
        # if it is loaded first, so load it first whenever it is installed
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        L.lc_build_id.argtypes = []
        L.lc_build_id.restype = ctypes.c_char_p
        built = L.lc_build_id().decode()
        if not os.environ.get("LINCHECK_LIB"):  # dev A/B builds are other sources on purpose
            want = source_build_id()
            if built != want:
                raise RuntimeError(
                    "stale liblincheck.so: built from sources %s, this tree is %s; rebuild "
                    "(make -C jepsen/etcd_amd/csrc)" % (built, want))
        p, i64, i32, u32, vp = (ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
                                ctypes.c_uint32, ctypes.c_void_p)
        L.lc_open.argtypes = [u32, ctypes.POINTER(vp)]
        L.lc_open.restype = ctypes.c_int
        L.lc_check.argtypes = [vp, p, p, i64, ctypes.POINTER(LcOpts), p]
        L.lc_check.restype = ctypes.c_int
        L.lc_check_device.argtypes = [vp, vp, vp, i64, ctypes.POINTER(LcOpts), vp, vp]
        L.lc_check_device.restype = ctypes.c_int
        L.lc_check_ex.argtypes = [vp, p, p, i64, ctypes.POINTER(LcOpts), p, ctypes.POINTER(LcAux)]
        L.lc_check_ex.restype = ctypes.c_int
        L.lc_check_device_ex.argtypes = [vp, vp, vp, i64, ctypes.POINTER(LcOpts), vp, vp,
                                         ctypes.POINTER(LcAux)]
        L.lc_check_device_ex.restype = ctypes.c_int
        L.lc_check32.argtypes = [vp, p, p, p, i64, ctypes.POINTER(LcOpts), p,
                                 ctypes.POINTER(LcAux)]
        L.lc_check32.restype = ctypes.c_int
        L.lc_check_device32.argtypes = [vp, vp, vp, vp, i64, ctypes.POINTER(LcOpts), vp, vp,
                                        ctypes.POINTER(LcAux)]
        L.lc_check_device32.restype = ctypes.c_int
        L.lc_pack32.argtypes = [p, p, i64, p, p]
        L.lc_pack32.restype = ctypes.c_int
        L.lc_pack16.argtypes = [p, p, i64, p, p]
        L.lc_pack16.restype = ctypes.c_int
        L.lc_check16.argtypes = [vp, p, p, p, i64, ctypes.POINTER(LcOpts), p,
                                 ctypes.POINTER(LcAux)]
        L.lc_check16.restype = ctypes.c_int
        L.lc_check_frontiers.argtypes = [vp, p, p, i64, p, ctypes.POINTER(LcOpts), vp, i32, p]
        L.lc_check_frontiers.restype = ctypes.c_int
        L.lc_last_totals.argtypes = [vp, ctypes.POINTER(LcTotals), i32]
        L.lc_last_totals.restype = ctypes.c_int
        L.lc_quiesce.argtypes = [vp]
        L.lc_quiesce.restype = ctypes.c_int
        L.lc_last_call_profile.argtypes = [vp, ctypes.POINTER(LcCallProfile)]
        L.lc_last_call_profile.restype = ctypes.c_int
        L.lc_key_cost.argtypes = [p, p, i64, p]
        L.lc_key_cost.restype = ctypes.c_int
        L.lc_last_stats.argtypes = [vp, ctypes.POINTER(LcStats)]
        L.lc_last_stats.restype = ctypes.c_int
        L.lc_last_device_stats.argtypes = [vp, i32, ctypes.POINTER(LcDeviceStats)]
        L.lc_last_device_stats.restype = ctypes.c_int
        L.lc_host_register.argtypes = [vp, vp, ctypes.c_uint64]
        L.lc_host_register.restype = ctypes.c_int
        L.lc_host_unregister.argtypes = [vp, vp]
        L.lc_host_unregister.restype = ctypes.c_int
        L.lc_last_error.argtypes = [vp]
        L.lc_last_error.restype = ctypes.c_char_p
        L.lc_close.argtypes = [vp]
        L.lc_close.restype = None
        L.lc_default_opts.argtypes = [ctypes.POINTER(LcOpts)]
        L.lc_default_opts.restype = None
        L.lc_plan_partition.argtypes = [p, p, i64, i32, p]
        L.lc_plan_partition.restype = ctypes.c_int
        L.lc_abi_version.argtypes = []
        L.lc_abi_version.restype = ctypes.c_int
        L.lc_synth_register.argtypes = [ctypes.POINTER(LcSynthParams), p, p, p,
                                        ctypes.POINTER(i64), ctypes.c_int]
        L.lc_synth_register.restype = ctypes.c_int
        L.lc_synth_key.argtypes = [ctypes.POINTER(LcSynthParams), i64, p, p, p, i64,
                                   ctypes.POINTER(i64), ctypes.POINTER(i32)]
        L.lc_synth_key.restype = ctypes.c_int
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def default_opts(max_configs_per_key=0, init_version=0, init_value=LC_NIL, flags=0,
                 time_budget_ms=0):
    o = LcOpts()
    lib().lc_default_opts(ctypes.byref(o))
    o.max_configs_per_key = max_configs_per_key
    o.time_budget_ms = time_budget_ms
    o.init_version = init_version
    o.init_value = init_value
    o.flags = flags
    return o


def as_ops(ops):
    a = np.ascontiguousarray(ops, dtype=np.int64)
    if a.ndim != 2 or a.shape[1] != 6:
        a = a.reshape(-1, 6)
    return a


def as_ops32(ops32):
    a = np.ascontiguousarray(ops32, dtype=np.int32)
    if a.ndim != 2 or a.shape[1] != 6:
        a = a.reshape(-1, 6)
    return a


def pack32(ops, key_off):
    """lc_pack32 (ABI 4): (ops32 (n, 6) int32, key_base int64 per key), the
    records narrowed by the device's own rules (include/lincheck.h)."""
    ops = as_ops(ops)
    key_off = np.ascontiguousarray(key_off, dtype=np.int64)
    out = np.zeros((len(ops), 6), dtype=np.int32)
    base = np.zeros(max(len(key_off) - 1, 0), dtype=np.int64)
    rc = lib().lc_pack32(_ptr(ops), _ptr(key_off), len(key_off) - 1, _ptr(out), _ptr(base))
    if rc != 0:
        raise LcError(rc, "lc_pack32")
    return out, base


def as_ops16(ops16):
    a = np.ascontiguousarray(ops16, dtype=np.uint32)
    if a.ndim != 2 or a.shape[1] != 4:
        a = a.reshape(-1, 4)
    return a


LC_ID15_MAX = 0x7FFD
ERANGE = 34


def pack16(ops, key_off):
    """lc_pack16 (include/lincheck.h, round 6): (ops16 (n, 4) uint32 — fve,
    version, call, ret — key_base int64 per key), or None when some record
    that is not malformed holds a value or expected id above LC_ID15_MAX
    (the batch then goes as lc_op32: pack32)."""
    ops = as_ops(ops)
    key_off = np.ascontiguousarray(key_off, dtype=np.int64)
    out = np.zeros((len(ops), 4), dtype=np.uint32)
    base = np.zeros(max(len(key_off) - 1, 0), dtype=np.int64)
    rc = lib().lc_pack16(_ptr(ops), _ptr(key_off), len(key_off) - 1, _ptr(out), _ptr(base))
    if rc == -ERANGE:
        return None
    if rc != 0:
        raise LcError(rc, "lc_pack16")
    return out, base


class LcError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("lincheck error %d: %s" % (code, msg))
        self.code = code


class Context:
    """An lc_ctx on the GPUs of device_mask (0 = all)."""

    def __init__(self, device_mask=0):
        h = ctypes.c_void_p()
        rc = lib().lc_open(device_mask, ctypes.byref(h))
        if rc != 0:
            raise LcError(rc, "lc_open failed (no usable GPU; there is no CPU fallback)")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            lib().lc_close(self._h)
            self._h = None

    __del__ = close

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def last_error(self):
        return lib().lc_last_error(self._h).decode()

    def stats(self):
        s = self.stats_raw()
        return {f: getattr(s, f) for f, _ in LcStats._fields_}

    def stats_raw(self, into=None):
        """lc_last_stats into an LcStats struct (reused when given)."""
        s = into if into is not None else LcStats()
        lib().lc_last_stats(self._h, ctypes.byref(s))
        return s

    def device_stats(self):
        """lc_last_device_stats for every device of the last lc_check: one
        dict per device (its key range, copies, kernels, wall time)."""
        out = []
        for i in range(int(self.stats_raw().n_devices)):
            d = LcDeviceStats()
            if lib().lc_last_device_stats(self._h, i, ctypes.byref(d)) != 0:
                break
            out.append({f: getattr(d, f) for f, _ in LcDeviceStats._fields_})
        return out

    def host_register(self, arr):
        """lc_host_register: page-lock a numpy array's buffer for repeated
        lc_check calls (unregister with host_unregister before freeing it)."""
        rc = lib().lc_host_register(self._h, ctypes.c_void_p(arr.ctypes.data), arr.nbytes)
        if rc != 0:
            raise LcError(rc, self.last_error())

    def host_unregister(self, arr):
        rc = lib().lc_host_unregister(self._h, ctypes.c_void_p(arr.ctypes.data))
        if rc != 0:
            raise LcError(rc, self.last_error())

    def _check_host(self, fn, ops, key_off, extra, opts, raise_on_error, witness, certificate):
        key_off = np.ascontiguousarray(key_off, dtype=np.int64)
        n_keys = len(key_off) - 1
        out = np.zeros(max(n_keys, 0), dtype=RESULT_DTYPE)
        o = opts if opts is not None else default_opts()
        wit = kind = cert = cset = None
        aux = None
        if witness or certificate:
            wit = np.full(len(ops), -3, dtype=np.int32)
            kind = np.full(max(n_keys, 0), -3, dtype=np.int32)
            if certificate:
                cert = np.full((max(n_keys, 0), 4), -3, dtype=np.int32)
                cset = np.zeros(len(ops), dtype=np.int32)
            aux = ctypes.byref(LcAux(wit.ctypes.data, kind.ctypes.data,
                                     cert.ctypes.data if certificate else None,
                                     cset.ctypes.data if certificate else None))
        rc = fn(self._h, _ptr(ops), _ptr(key_off), *extra, n_keys, ctypes.byref(o), _ptr(out), aux)
        if rc != 0 and raise_on_error:
            raise LcError(rc, self.last_error())
        if certificate:
            return rc, out, wit, kind, cert, cset
        return (rc, out, wit, kind) if witness else (rc, out)

    def check(self, ops, key_off, opts=None, raise_on_error=True, witness=False,
              certificate=False):
        """Host-buffer check. Returns (rc, results structured array), or with
        witness=True (rc, results, witness per record, witness kind per key)
        from lc_check_ex (include/lincheck.h, lc_aux); certificate=True adds
        the infeasibility certificates (int32[n_keys, 4]) and their position
        sets (int32 per record): (rc, results, witness, kind, cert, cert_set)."""
        return self._check_host(lib().lc_check_ex, as_ops(ops), key_off, (), opts,
                                raise_on_error, witness, certificate)

    def check32(self, ops32, key_off, key_base=None, opts=None, raise_on_error=True,
                witness=False, certificate=False):
        """lc_check32 (ABI 4): 24-byte records from host memory ((n, 6) int32,
        as pack32 makes them) and their key bases; returns as check()."""
        ops32 = as_ops32(ops32)
        base = None if key_base is None else np.ascontiguousarray(key_base, dtype=np.int64)
        if base is not None and len(base) != len(key_off) - 1:
            # lc_check32 reads n_keys bases: a short array would be read past its end
            raise ValueError(f"key_base has {len(base)} entries for {len(key_off) - 1} keys")
        return self._check_host(lib().lc_check32, ops32, key_off, (_ptr(base),), opts,
                                raise_on_error, witness, certificate)

    def check16(self, ops16, key_off, key_base=None, opts=None, raise_on_error=True,
                witness=False, certificate=False):
        """lc_check16 (round 6): 16-byte records from host memory ((n, 4)
        uint32, as pack16 makes them) and their key bases; returns as check()."""
        ops16 = as_ops16(ops16)
        base = None if key_base is None else np.ascontiguousarray(key_base, dtype=np.int64)
        if base is not None and len(base) != len(key_off) - 1:
            raise ValueError(f"key_base has {len(base)} entries for {len(key_off) - 1} keys")
        return self._check_host(lib().lc_check16, ops16, key_off, (_ptr(base),), opts,
                                raise_on_error, witness, certificate)

    def check_frontiers(self, ops, key_off, stop_ops, max_per_key=10, opts=None):
        """lc_check_frontiers (include/lincheck_fx.h, ABI 4): for every key,
        up to max_per_key configurations of its JIT frontier just before the
        :ok return of record stop_ops[k], as (version, value id, pending
        record indices) tuples — or None where the device search could not
        get there (the caller's fallback: FrontierExchange.frontier)."""
        from .fx import LcFxConfig
        ops = as_ops(ops)
        key_off = np.ascontiguousarray(key_off, dtype=np.int64)
        n_keys = len(key_off) - 1
        stop = np.ascontiguousarray(stop_ops, dtype=np.int64)
        if len(stop) != n_keys:
            raise ValueError(f"stop_ops has {len(stop)} entries for {n_keys} keys")
        buf = (LcFxConfig * max(1, n_keys * max_per_key))()
        n_out = np.zeros(max(n_keys, 1), dtype=np.int32)
        o = opts if opts is not None else default_opts()
        rc = lib().lc_check_frontiers(self._h, _ptr(ops), _ptr(key_off), n_keys, _ptr(stop),
                                      ctypes.byref(o), ctypes.cast(buf, ctypes.c_void_p),
                                      max_per_key, _ptr(n_out))
        if rc != 0:
            raise LcError(rc, self.last_error())
        out = []
        for k in range(n_keys):
            n = int(n_out[k])
            if n < 0:
                out.append(None)
                continue
            out.append([(int(c.version), int(c.value), tuple(int(c.pending[j]) for j in range(c.n_pending)))
                        for c in buf[k * max_per_key:k * max_per_key + n]])
        return out

    def quiesce(self):
        """lc_quiesce (ABI 5): stop the resident version-order grid now (it
        otherwise leaves after LC_RESIDENT_IDLE_US without a call)."""
        rc = lib().lc_quiesce(self._h)
        if rc != 0:
            raise LcError(rc, self.last_error())

    def totals(self, reset=False):
        """lc_last_totals (ABI 4): calls and device time summed since the last
        reset, every pending event read first."""
        t = LcTotals()
        lib().lc_last_totals(self._h, ctypes.byref(t), 1 if reset else 0)
        return {f: getattr(t, f) for f, _ in LcTotals._fields_}

    def call_profile(self):
        """lc_last_call_profile: where the last host call's wall time went."""
        pr = LcCallProfile()
        lib().lc_last_call_profile(self._h, ctypes.byref(pr))
        return {f: getattr(pr, f) for f, _ in LcCallProfile._fields_}

    def check_device(self, d_ops, d_key_off, n_keys, d_out, stream=None, opts=None,
                     d_witness=None, d_witness_kind=None):
        """Device-pointer check (ints), e.g. from torch tensors' data_ptr();
        with d_witness / d_witness_kind (device pointers) lc_check_device_ex."""
        o = opts if opts is not None else default_opts()
        args = (self._h, ctypes.c_void_p(d_ops), ctypes.c_void_p(d_key_off), n_keys,
                ctypes.byref(o), ctypes.c_void_p(d_out),
                ctypes.c_void_p(stream) if stream else None)
        if d_witness is not None:
            aux = LcAux(d_witness, d_witness_kind, None, None)
            rc = lib().lc_check_device_ex(*args, ctypes.byref(aux))
        else:
            rc = lib().lc_check_device(*args)
        if rc != 0:
            raise LcError(rc, self.last_error())
        return rc


    def check_device32(self, d_ops32, d_key_off, d_key_base, n_keys, d_out, stream=None,
                       opts=None):
        """lc_check_device32 (ABI 4): 24-byte records resident on the GPU."""
        o = opts if opts is not None else default_opts()
        rc = lib().lc_check_device32(self._h, ctypes.c_void_p(d_ops32), ctypes.c_void_p(d_key_off),
                                     ctypes.c_void_p(d_key_base) if d_key_base else None, n_keys,
                                     ctypes.byref(o), ctypes.c_void_p(d_out),
                                     ctypes.c_void_p(stream) if stream else None, None)
        if rc != 0:
            raise LcError(rc, self.last_error())
        return rc

    def bind_check_device32(self, d_ops32, d_key_off, d_key_base, n_keys, d_out, stream=None,
                            opts=None):
        """lc_check_device32 (ABI 4) with its arguments converted once, as
        bind_check_device: 24-byte records resident on the device."""
        L = lib()
        o = opts if opts is not None else default_opts()
        args = (self._h, ctypes.c_void_p(d_ops32), ctypes.c_void_p(d_key_off),
                ctypes.c_void_p(d_key_base) if d_key_base else None, ctypes.c_int64(n_keys),
                ctypes.byref(o), ctypes.c_void_p(d_out),
                ctypes.c_void_p(stream) if stream else None, None)
        fn = L.lc_check_device32

        def call():
            rc = fn(*args)
            if rc != 0:
                raise LcError(rc, self.last_error())

        call._keep = (o,)
        return call

    def bind_check_device(self, d_ops, d_key_off, n_keys, d_out, stream=None, opts=None,
                          stats=None):
        """check_device with its arguments converted once: returns a
        zero-argument callable that runs the check (and fills `stats`, an
        LcStats, when given) and raises LcError on failure.  For loops that
        time the same call over and over (bench.py)."""
        L = lib()
        o = opts if opts is not None else default_opts()
        args = (self._h, ctypes.c_void_p(d_ops), ctypes.c_void_p(d_key_off),
                ctypes.c_int64(n_keys), ctypes.byref(o), ctypes.c_void_p(d_out),
                ctypes.c_void_p(stream) if stream else None)
        fn, st_fn = L.lc_check_device, L.lc_last_stats
        st_args = (self._h, ctypes.byref(stats)) if stats is not None else None

        def call():
            rc = fn(*args)
            if rc != 0:
                raise LcError(rc, self.last_error())
            if st_args is not None:
                st_fn(*st_args)
            return stats

        call._keep = (o, stats)  # the byref targets must outlive the closure
        return call


def plan_partition(key_off, n_parts, ops=None):
    """lc_plan_partition: n_parts+1 key bounds at equal estimated cost (by
    lc_key_cost with ops; by record count without)."""
    key_off = np.ascontiguousarray(key_off, dtype=np.int64)
    if ops is not None:
        ops = as_ops(ops)
    bounds = np.zeros(n_parts + 1, dtype=np.int64)
    rc = lib().lc_plan_partition(_ptr(ops), _ptr(key_off), len(key_off) - 1, n_parts,
                                 _ptr(bounds))
    if rc != 0:
        raise LcError(rc, "lc_plan_partition")
    return bounds


def key_cost(ops, key_off):
    """lc_key_cost: estimated device cost per key (record-scan units)."""
    ops = as_ops(ops)
    key_off = np.ascontiguousarray(key_off, dtype=np.int64)
    out = np.zeros(len(key_off) - 1, dtype=np.float64)
    rc = lib().lc_key_cost(_ptr(ops), _ptr(key_off), len(out), _ptr(out))
    if rc != 0:
        raise LcError(rc, "lc_key_cost")
    return out


def synth_params(n_keys, ops_per_key, concurrency=10, n_values=5, p_info=0.0,
                 p_anomaly=0.0, seed=0x5EED0000, info_frac=0.0):
    return LcSynthParams(n_keys, ops_per_key, concurrency, n_values, p_info,
                         p_anomaly, seed, info_frac)


def synth(n_keys, ops_per_key, concurrency=10, n_values=5, p_info=0.0,
          p_anomaly=0.0, seed=0x5EED0000, n_threads=None, info_frac=0.0):
    """Packed synthetic histories: (ops (n,6) int64, key_off, labels, n_invocations).
    info_frac > 0 makes exactly round(info_frac * ops_per_key) records of
    every key crashed writes/CAS (include/lincheck_synth.h)."""
    prm = synth_params(n_keys, ops_per_key, concurrency, n_values, p_info,
                       p_anomaly, seed, info_frac)
    ops = np.zeros((n_keys * ops_per_key, 6), dtype=np.int64)
    key_off = np.zeros(n_keys + 1, dtype=np.int64)
    labels = np.zeros(n_keys, dtype=np.int32)
    ninv = ctypes.c_int64(0)
    if n_threads is None:
        n_threads = min(16, os.cpu_count() or 1)
    rc = lib().lc_synth_register(ctypes.byref(prm), _ptr(ops), _ptr(key_off),
                                 _ptr(labels), ctypes.byref(ninv), n_threads)
    if rc != 0:
        raise LcError(rc, "lc_synth_register")
    return ops, key_off, labels, ninv.value


def synth_key(key, ops_per_key, concurrency=10, n_values=5, p_info=0.0,
              p_anomaly=0.0, seed=0x5EED0000, info_frac=0.0):
    """One key's full op stream incl. :fail: (ops, proc, status, label)."""
    prm = synth_params(1, ops_per_key, concurrency, n_values, p_info, p_anomaly, seed,
                       info_frac)
    n = ctypes.c_int64(0)
    lab = ctypes.c_int32(0)
    cap = 4 * ops_per_key + 64
    while True:
        ops = np.zeros((cap, 6), dtype=np.int64)
        proc = np.zeros(cap, dtype=np.int32)
        st = np.zeros(cap, dtype=np.int32)
        rc = lib().lc_synth_key(ctypes.byref(prm), key, _ptr(ops), _ptr(proc), _ptr(st),
                                cap, ctypes.byref(n), ctypes.byref(lab))
        if rc == 0:
            k = n.value
            return ops[:k], proc[:k], st[:k], lab.value
        cap = n.value
