"""World-size-2 multi-rank paths on CPU with the gloo backend.

The GPU path shards keys across ranks with no data-path collective; here the
same sharding/gather code runs with the oracle standing in for the GPU
checker (tests may use the oracle), and bench.py's whole-job reduction
(max time, summed counts) runs over gloo."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import torch
    import torch.distributed as dist
    import oracle
    from jepsen.etcd_amd import abi
    from jepsen.etcd_amd import dist as D
    import bench

    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port,
                            rank=rank, world_size=world)
    ops, off, lab, _ = abi.synth(120, 150, concurrency=10, p_anomaly=0.25, seed=31)
    a, b = D.shard(off, rank, world, ops=ops)   # bench.py's C3 split
    sub, soff = D.slice_keys(ops, off, a, b)
    _, r = oracle.check(sub, soff, algo=oracle.JITC)   # stand-in for the GPU
    verd, fail = D.gather_results(r, (a, b), len(off) - 1)
    el, counts = bench.reduce_run(0.5 + rank, len(sub), r, world, torch.device("cpu"))
    rows = D.gather_rows([rank, a, b, len(sub)])
    if rank == 0:
        _, full = oracle.check(ops, off, algo=oracle.JITC)
        out.put(((verd == full["verdict"]).all(), (fail == full["fail_op"]).all(),
                 D.merge_verdicts(verd), el, counts, int(off[-1]),
                 int((full["verdict"] == 1).sum()), rows))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_shard_gather_and_reduce():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ok_v, ok_f, merged, el, counts, n_ops, n_valid, rows = res
    # the ranks' key ranges tile the batch, contiguously
    assert rows[0][1] == 0 and rows[0][2] == rows[1][1] and rows[1][2] == 120
    assert rows[0][3] + rows[1][3] == n_ops
    assert ok_v and ok_f
    assert merged is False            # the batch holds injected anomalies
    assert el == 1.5                  # max over ranks
    assert counts[0] == n_ops and counts[1] == n_valid
    assert counts[1] + counts[2] + counts[3] == 120


def test_merge_rule():
    from jepsen.etcd_amd.dist import merge_verdicts
    assert merge_verdicts([1, 1]) is True
    assert merge_verdicts([1, -1]) == "unknown"
    assert merge_verdicts([-1, 0, 1]) is False
    assert merge_verdicts(np.array([], dtype=np.int32)) is True


def _fx_transport_worker(rank, world, port, out):
    import ctypes
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import torch.distributed as dist
    from jepsen.etcd_amd import fx as F
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port,
                            rank=rank, world_size=world)
    try:
        tr = F.TorchTransport(dist.group.WORLD, device=0)
        send = (ctypes.c_int64 * world)(*[100 * rank + j for j in range(world)])
        recv = (ctypes.c_int64 * world)()
        rc1 = tr._counts(None, send, recv)
        vals = (ctypes.c_int64 * 3)(rank + 1, 7, -rank)
        rc2 = tr._allred(None, vals, 3, F.LC_FX_SUM)
        mx = (ctypes.c_int64 * 1)(rank * 5)
        rc3 = tr._allred(None, mx, 1, F.LC_FX_MAX)
        out.put((rank, tr.on_device, rc1, list(recv), rc2, list(vals), rc3, mx[0],
                 repr(tr.error)))
    finally:
        dist.destroy_process_group()


def test_fx_transport_collectives_two_ranks_gloo():
    """The frontier exchange's collectives (jepsen/etcd_amd/fx.py
    TorchTransport, the lc_fx_transport callbacks): the count exchange is an
    all-to-all (recv[j] = what rank j sends here), the all-reduce sums or
    maxes, host-staged under gloo.  The payload all-to-all-v needs device
    buffers and runs in the GPU tests (tests/test_fx.py)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    world = 3
    procs = [ctx.Process(target=_fx_transport_worker, args=(r, world, port, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, on_dev, rc1, recv, rc2, vals, rc3, mx, err in res:
        assert not on_dev and rc1 == rc2 == rc3 == 0, err
        assert recv == [100 * j + rank for j in range(world)]
        assert vals == [1 + 2 + 3, 7 * world, -(0 + 1 + 2)]
        assert mx == 5 * (world - 1)
