"""Time the frontier exchange with ranks as processes (torch.distributed,
TorchTransport) on the oversized key of bench.py, e.g. two processes sharing
one GPU over gloo:

    python tools/fx_ranks.py --world 2 --backend gloo --part-above 16384
"""
import argparse
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def rank_main(rank, a, port, q):
    import numpy as np  # noqa: F401
    import torch.distributed as dist
    from jepsen.etcd_amd import abi
    from jepsen.etcd_amd.fx import FrontierExchange
    dist.init_process_group(a.backend, init_method="tcp://127.0.0.1:%d" % port, rank=rank,
                            world_size=a.world)
    try:
        ops, _, _, _ = abi.synth(1, a.ops, concurrency=a.conc, seed=0x5EED0004)
        ops = ops.copy()
        ops[:, 3] = abi.LC_NIL
        fx = FrontierExchange(device=a.device if a.device >= 0 else rank, group=dist.group.WORLD,
                              part_above=a.part_above)
        fx.check(ops)
        dist.barrier()
        t0 = time.perf_counter()
        r = fx.check(ops)
        dt = (time.perf_counter() - t0) * 1e3
        q.put((rank, dt, [int(r[f]) for f in ("verdict", "configs_explored", "max_frontier")],
               fx.stats()))
        fx.close()
    except Exception as e:
        q.put((rank, repr(e), None, None))
    finally:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--backend", default="gloo")
    ap.add_argument("--device", type=int, default=0, help="-1: rank i on GPU i")
    ap.add_argument("--ops", type=int, default=2000)
    ap.add_argument("--conc", type=int, default=50)
    ap.add_argument("--part-above", type=int, default=16384)
    a = ap.parse_args()
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=rank_main, args=(r, a, port, q)) for r in range(a.world)]
    for p in ps:
        p.start()
    out = [q.get(timeout=600) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    out.sort(key=lambda x: x[0])
    print(json.dumps({"world": a.world, "backend": a.backend, "part_above": a.part_above,
                      "ms": [o[1] for o in out], "result": out[0][2],
                      "stats": [o[3] for o in out]}))


if __name__ == "__main__":
    main()
