"""Frontier exchange (include/lincheck_fx.h): ONE oversized key's JIT frontier
search over a whole GPU, and over several ranks by hash ownership — SURVEY.md
§8(e)'s one exception to "keys are independent, no collective"
(register.clj:108 splits keys; a single key's search, knossos.linear behind
checker/linearizable at register.clj:110-111, has no such split).

    with FrontierExchange(device=0) as fx:            # the whole GPU, one rank
        r = fx.check(ops)                              # one key's records (n, 6)

    # one rank per GPU under torchrun; collectives over torch.distributed
    # (RCCL over xGMI under "nccl", host-staged under "gloo")
    fx = FrontierExchange(device=local_rank, group=dist.group.WORLD)

The library calls three collectives back (lc_fx_transport): a count
exchange, an all-to-all-v of 16-byte configurations in device memory, and a
small all-reduce.  `TorchTransport` implements them; the GPU tests drive the
same engine with in-process ranks (`virtual_ranks`) and with two processes
over gloo on one card.
"""
import ctypes

import numpy as np

from . import abi

LC_FX_SUM, LC_FX_MAX = 0, 1

_COUNTS = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64),
                           ctypes.POINTER(ctypes.c_int64))
_A2AV = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                         ctypes.POINTER(ctypes.c_int64), ctypes.c_void_p,
                         ctypes.POINTER(ctypes.c_int64), ctypes.c_int64)
_ALLRED = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64),
                           ctypes.c_int32, ctypes.c_int32)


class LcFxTransport(ctypes.Structure):
    _fields_ = [("user", ctypes.c_void_p), ("rank", ctypes.c_int32),
                ("n_ranks", ctypes.c_int32), ("exchange_counts", _COUNTS),
                ("alltoallv", _A2AV), ("allreduce", _ALLRED)]


class LcFxParams(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("virtual_ranks", ctypes.c_int32),
                ("part_above", ctypes.c_int64), ("repl_below", ctypes.c_int64),
                ("table_log2", ctypes.c_int64), ("flags", ctypes.c_int64)]


LC_FX_FLAG_WIDE_TABLES = 1
LC_FX_FLAG_EXCHANGE_SELF = 2
LC_FX_RCCL_ID_BYTES = 128


class LcFxConfig(ctypes.Structure):
    _fields_ = [("version", ctypes.c_int64), ("value", ctypes.c_int64),
                ("n_pending", ctypes.c_int64), ("pending", ctypes.c_int64 * 64)]


class LcFxStats(ctypes.Structure):
    _fields_ = [("total_ms", ctypes.c_double), ("returns", ctypes.c_int64),
                ("levels", ctypes.c_int64), ("part_returns", ctypes.c_int64),
                ("part_levels", ctypes.c_int64), ("sent_configs", ctypes.c_int64),
                ("gathers", ctypes.c_int64), ("max_local_frontier", ctypes.c_int64),
                ("redos", ctypes.c_int64), ("wide_returns", ctypes.c_int64)]


_bound = False


def _lib():
    global _bound
    L = abi.lib()
    if not _bound:
        vp, p = ctypes.c_void_p, ctypes.c_void_p
        L.lc_fx_open.argtypes = [ctypes.POINTER(LcFxParams), ctypes.POINTER(LcFxTransport),
                                 ctypes.POINTER(vp)]
        L.lc_fx_open.restype = ctypes.c_int
        L.lc_fx_open_devices.argtypes = [ctypes.POINTER(LcFxParams), ctypes.POINTER(ctypes.c_int32),
                                         ctypes.c_int32, ctypes.POINTER(vp)]
        L.lc_fx_open_devices.restype = ctypes.c_int
        L.lc_fx_rccl_unique_id.argtypes = [ctypes.c_char_p]
        L.lc_fx_rccl_unique_id.restype = ctypes.c_int
        L.lc_fx_open_rccl.argtypes = [ctypes.POINTER(LcFxParams), ctypes.c_char_p, ctypes.c_int32,
                                      ctypes.c_int32, ctypes.POINTER(vp)]
        L.lc_fx_open_rccl.restype = ctypes.c_int
        L.lc_fx_check.argtypes = [vp, p, ctypes.c_int64, ctypes.POINTER(abi.LcOpts), p]
        L.lc_fx_check.restype = ctypes.c_int
        L.lc_fx_last_stats.argtypes = [vp, ctypes.POINTER(LcFxStats)]
        L.lc_fx_last_stats.restype = ctypes.c_int
        L.lc_fx_last_error.argtypes = [vp]
        L.lc_fx_last_error.restype = ctypes.c_char_p
        L.lc_fx_close.argtypes = [vp]
        L.lc_fx_close.restype = None
        L.lc_fx_abort.argtypes = [vp]
        L.lc_fx_abort.restype = None
        L.lc_fx_frontier.argtypes = [vp, p, ctypes.c_int64, ctypes.POINTER(abi.LcOpts),
                                     ctypes.c_int64, p, ctypes.c_int32,
                                     ctypes.POINTER(ctypes.c_int32)]
        L.lc_fx_frontier.restype = ctypes.c_int
        _bound = True
    return L


class _DeviceBytes:
    """A device allocation seen by torch through __cuda_array_interface__
    (no copy): lets torch.distributed read and write the engine's buffers."""

    def __init__(self, ptr, nbytes):
        self.__cuda_array_interface__ = {"shape": (int(nbytes),), "typestr": "|u1",
                                         "data": (int(ptr), False), "version": 3}


class TorchTransport:
    """lc_fx_transport over a torch.distributed process group.  Under "nccl"
    (RCCL) the payload moves device to device; under "gloo" it is staged
    through host memory.  Every callback is collective: all ranks call them
    in the same order (the engine guarantees it)."""

    def __init__(self, group=None, device=0):
        import torch
        import torch.distributed as dist
        self.torch, self.dist, self.group = torch, dist, group
        self.rank = dist.get_rank(group)
        self.n_ranks = dist.get_world_size(group)
        self.device = torch.device("cuda", device)
        self.on_device = dist.get_backend(group) == "nccl"
        self.error = None
        self._c = LcFxTransport(None, self.rank, self.n_ranks, _COUNTS(self._counts),
                                _A2AV(self._a2av), _ALLRED(self._allred))

    def _fail(self, e):
        self.error = e
        return -5

    def _dev(self, ptr, nbytes):
        return self.torch.as_tensor(_DeviceBytes(ptr, nbytes), device=self.device)

    def _counts(self, _u, send, recv):
        try:
            t = self.torch
            s = t.tensor([send[j] for j in range(self.n_ranks)], dtype=t.int64)
            if self.on_device:
                s = s.to(self.device)
            r = t.empty_like(s)
            self.dist.all_to_all_single(r, s, group=self.group)
            for j, v in enumerate(r.tolist()):
                recv[j] = v
            return 0
        except Exception as e:  # surfaced by FrontierExchange.check
            return self._fail(e)

    def _a2av(self, _u, d_send, send_counts, d_recv, recv_counts, entry):
        try:
            t = self.torch
            sc = [send_counts[j] * entry for j in range(self.n_ranks)]
            rc = [recv_counts[j] * entry for j in range(self.n_ranks)]
            ns, nr = sum(sc), sum(rc)
            if self.on_device:
                s = self._dev(d_send, max(ns, 1))[:ns]
                r = self._dev(d_recv, max(nr, 1))[:nr]
                self.dist.all_to_all_single(r, s, rc, sc, group=self.group)
                t.cuda.synchronize(self.device)
            else:
                s = self._dev(d_send, max(ns, 1))[:ns].cpu() if ns else t.empty(0, dtype=t.uint8)
                r = t.empty(nr, dtype=t.uint8)
                self.dist.all_to_all_single(r, s, rc, sc, group=self.group)
                if nr:
                    self._dev(d_recv, nr).copy_(r)
                    t.cuda.synchronize(self.device)
            return 0
        except Exception as e:
            return self._fail(e)

    def _allred(self, _u, vals, n, op):
        try:
            t = self.torch
            v = t.tensor([vals[i] for i in range(n)], dtype=t.int64)
            if self.on_device:
                v = v.to(self.device)
            rop = self.dist.ReduceOp.MAX if op == LC_FX_MAX else self.dist.ReduceOp.SUM
            self.dist.all_reduce(v, op=rop, group=self.group)
            for i, x in enumerate(v.tolist()):
                vals[i] = x
            return 0
        except Exception as e:
            return self._fail(e)


class FrontierExchange:
    """One engine.  Collectives, by argument:

    * rccl_devices=[d0, d1, ...]: one rank per listed GPU of this process,
      native RCCL inside the library (lc_fx_open_devices);
    * rccl_group=<torch.distributed group>: this process is one rank, native
      RCCL inside the library (lc_fx_open_rccl; the unique id travels over
      the group, then torch is out of the data path);
    * group=<torch.distributed group>: this process is one rank, collectives
      called back into torch.distributed (TorchTransport);
    * none of them: `virtual_ranks` ranks as threads on `device`.

    part_above / repl_below: the frontier size above which it is partitioned
    by owner, and below which it is replicated again (-1: the library's
    defaults).  table_log2: dedup table size (0: from the budget).  flags:
    LC_FX_FLAG_* (LC_FX_FLAG_WIDE_TABLES: 16-byte-key tables only;
    LC_FX_FLAG_EXCHANGE_SELF: own configurations through the exchange too)."""

    def __init__(self, device=0, virtual_ranks=1, group=None, part_above=-1, repl_below=-1,
                 table_log2=0, flags=0, rccl_devices=None, rccl_group=None):
        L = _lib()
        self._h = ctypes.c_void_p()
        prm = LcFxParams(device, virtual_ranks, part_above, repl_below, table_log2, flags)
        self.transport = None
        if rccl_devices is not None:
            devs = (ctypes.c_int32 * len(rccl_devices))(*rccl_devices)
            rc = L.lc_fx_open_devices(ctypes.byref(prm), devs, len(rccl_devices),
                                      ctypes.byref(self._h))
            what = "lc_fx_open_devices"
        elif rccl_group is not None:
            import torch.distributed as dist
            buf = ctypes.create_string_buffer(LC_FX_RCCL_ID_BYTES)
            rank = dist.get_rank(rccl_group)
            if rank == 0:
                rc = L.lc_fx_rccl_unique_id(buf)
                if rc != 0:
                    raise abi.LcError(rc, "lc_fx_rccl_unique_id")
            obj = [buf.raw if rank == 0 else None]
            dist.broadcast_object_list(obj, src=dist.get_global_rank(rccl_group, 0),
                                       group=rccl_group)
            rc = L.lc_fx_open_rccl(ctypes.byref(prm), obj[0], rank,
                                   dist.get_world_size(rccl_group), ctypes.byref(self._h))
            what = "lc_fx_open_rccl"
        else:
            tr = None
            if group is not None:
                self.transport = TorchTransport(group, device)
                tr = ctypes.byref(self.transport._c)
            rc = L.lc_fx_open(ctypes.byref(prm), tr, ctypes.byref(self._h))
            what = "lc_fx_open"
        if rc != 0:
            raise abi.LcError(rc, what)

    def check(self, ops, opts=None):
        """Decide one key (records (n, 6) int64): a RESULT_DTYPE record."""
        L = _lib()
        ops = abi.as_ops(ops)
        out = np.zeros(1, dtype=abi.RESULT_DTYPE)
        o = opts if opts is not None else abi.default_opts()
        rc = L.lc_fx_check(self._h, abi._ptr(ops), len(ops), ctypes.byref(o), abi._ptr(out))
        if rc != 0:
            err = L.lc_fx_last_error(self._h).decode()
            if self.transport is not None and self.transport.error is not None:
                err += " (transport: %r)" % (self.transport.error,)
            raise abi.LcError(rc, "lc_fx_check: " + err)
        return out[0]

    def frontier(self, ops, stop_op, max_configs=10, opts=None):
        """knossos's :configs: up to max_configs configurations of the
        frontier just before the :ok return of record stop_op (for an invalid
        key, its fail_op), as (version, value id, pending record indices)."""
        L = _lib()
        ops = abi.as_ops(ops)
        buf = (LcFxConfig * max(1, max_configs))()
        n = ctypes.c_int32(0)
        o = opts if opts is not None else abi.default_opts()
        rc = L.lc_fx_frontier(self._h, abi._ptr(ops), len(ops), ctypes.byref(o), int(stop_op),
                              ctypes.cast(buf, ctypes.c_void_p), max_configs, ctypes.byref(n))
        if rc != 0:
            raise abi.LcError(rc, "lc_fx_frontier: " + L.lc_fx_last_error(self._h).decode())
        return [(int(c.version), int(c.value), tuple(int(c.pending[j]) for j in range(c.n_pending)))
                for c in buf[:n.value]]

    def stats(self):
        s = LcFxStats()
        _lib().lc_fx_last_stats(self._h, ctypes.byref(s))
        return {k: getattr(s, k) for k, _ in LcFxStats._fields_}

    def abort(self):
        """From another thread (a watchdog): stop the search in progress —
        RCCL communicators are aborted, so a rank stuck in a collective
        returns and check() raises; an RCCL engine is unusable afterwards."""
        if self._h:
            _lib().lc_fx_abort(self._h)

    def close(self):
        if self._h:
            _lib().lc_fx_close(self._h)
            self._h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()
