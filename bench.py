#!/usr/bin/env python3
"""Benchmark: history ops linearizability-checked per second (BASELINE.json).

One step = one lc_check_device() call over one batch of resident synthetic
register histories: by default the C2 workload of BASELINE.json configs[1],
10k keys x 1k ops (packed records), concurrency 20, valid CAS-register+version
histories, on one MI355X.  For N GPUs (torchrun, one rank per GPU) it is
BASELINE configs[2] (C3): every rank builds the SAME seeded 10k-key batch,
lc_plan_partition splits it into N contiguous key ranges of equal estimated
cost (lc_key_cost), and each rank checks its own range: total work is fixed
("scaling": "strong").  Keys are independent (register.clj:108), so the
data path has no collective; the only cross-rank traffic is the timing
barrier/max and the gather of per-rank ranges and times (RCCL).

Prints ONE JSON line on rank 0 (contract in the task statement), with the
roofline of the dominant kernel (fast_tier_kernel on C2; HIP events on its
stream) and a CPU baseline: the oracle's C restatement of knossos (faster of
its JIT and WGL analyzers) on a bounded sample of the same workload, on host
threads.  Outside the timed region, rank 0 also decides BASELINE configs[3]
(one hot key, 5k ops, concurrency 50, 20 % :info) and reports its time.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = ("history ops linearizability-checked/sec (1/2/4/8 GPU) + per-key "
          "verdict parity")
# Algorithmic HBM bytes: every record is read once (48 B/op)
# and every key's result written once (40 B/key).  SURVEY.md §8(d)'s 176 B/op
# adds one 128-B configuration-table probe per op; this design never probes
# HBM for configurations (the frontier lives in SGPRs/LDS and version-pinned
# keys need no frontier at all), so those bytes do not exist here and would
# only inflate `achieved` (above the physical peak).
ALGO_BYTES_PER_OP = 48
ALGO_BYTES_PER_KEY = 40
HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--keys", type=int, default=10000)
    ap.add_argument("--ops-per-key", type=int, default=1000)
    ap.add_argument("--concurrency", type=int, default=20)
    ap.add_argument("--p-info", type=float, default=0.0)
    ap.add_argument("--cpu-sample-keys", type=int, default=10000)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--bare", action="store_true",
                    help="timed region only (no CPU baseline, no hot-key leg): "
                         "for rocprofv3 runs whose per-kernel averages must "
                         "match the bench line")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "r06", "traffic_fast_tier.json"))
    return ap.parse_args()


def main():
    args = parse()
    # stdout carries only the JSON line: everything else written to fd 1 —
    # RCCL's version banner, gloo's "Rank r is connected to n peer ranks"
    # whenever a gloo group forms, the library's RCCL communicators — goes to
    # stderr; the line is written to a duplicate of the original stdout
    sys.stdout.flush()
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    import torch
    import torch.distributed as dist
    from jepsen.etcd_amd import abi

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal knobs for a 1-GPU box (never set by the driver): every rank on
    # device LC_BENCH_DEVICE, process group LC_BENCH_BACKEND (gloo) instead of
    # RCCL, which refuses two ranks on one GPU
    if os.environ.get("LC_BENCH_DEVICE"):
        local = int(os.environ["LC_BENCH_DEVICE"])
    backend = os.environ.get("LC_BENCH_BACKEND", "nccl")
    torch.cuda.set_device(local)
    # under torchrun (even with one rank) the RCCL group carries the timing
    # barrier and the max/sum reductions
    distributed = "TORCHELASTIC_RUN_ID" in os.environ or world > 1
    if distributed:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
        dist.barrier()
    dev = torch.device("cuda", local)

    # ---- workload: configs[1] = C2, seed 0x5EED0002, the same on every
    # rank; configs[2] = C3: rank r checks its cost-balanced key range
    from jepsen.etcd_amd import dist as D
    seed = 0x5EED0002
    ops, key_off, _, n_inv = abi.synth(args.keys, args.ops_per_key,
                                       concurrency=args.concurrency,
                                       p_info=args.p_info, seed=seed)
    bounds = abi.plan_partition(key_off, world, ops=ops)
    ka, kb = int(bounds[rank]), int(bounds[rank + 1])
    my_keys = kb - ka
    n_ops = int(key_off[kb] - key_off[ka])  # this rank's records
    d_ops = torch.from_numpy(np.ascontiguousarray(ops[key_off[ka]:key_off[kb]])).to(dev)
    d_off = torch.from_numpy(np.ascontiguousarray(key_off[ka:kb + 1])).to(dev)
    d_out = torch.zeros(max(my_keys, 1) * abi.RESULT_DTYPE.itemsize, dtype=torch.uint8,
                        device=dev)
    stream = torch.cuda.current_stream(dev)
    ctx = abi.Context(device_mask=1 << local)

    # one step = one lc_check_device call, arguments converted once.  The
    # call returns on the version-order pass's follower signal (no event
    # wait).  The pass is timed by HIP events on the launch stream on every
    # TIME_EVERY-th step (each event record costs ~2 us of host time per
    # call, so the other steps run with LC_FLAG_NO_TIMING); the event times
    # are read after the loop (lc_last_totals), so no step waits for them
    steps = bind_steps(ctx, abi, d_ops.data_ptr(), d_off.data_ptr(), my_keys, d_out.data_ptr(),
                       stream.cuda_stream)

    for i in range(args.warmup):
        steps[i % TIME_EVERY != 0]()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    ctx.totals(reset=True)
    t0 = time.perf_counter()
    for i in range(args.steps):
        steps[i % TIME_EVERY != 0]()
    # a batch of at most one key per resident workgroup (a C3 shard) is
    # served by the resident version-order grid (lc_quiesce, lincheck.h):
    # stopping it is part of the job, inside the timed region
    ctx.quiesce()
    torch.cuda.synchronize()
    # this rank's own K steps; the job time is the MAX of these over ranks
    # (reduce_run).  The trailing barrier closes the timed region on every
    # rank but is not counted: at N = 8 a step is ~27 us and one RCCL barrier
    # would be a visible share of it.
    own = time.perf_counter() - t0
    if distributed:
        dist.barrier()
    after_barrier = time.perf_counter() - t0
    elapsed = own
    tot = ctx.totals(reset=True)
    assert tot["calls"] == args.steps and tot["timed_calls"] >= 1, tot
    last = ctx.stats()  # the last call's tiers (nothing has run since)
    kms = [tot["kernel_ms"] / tot["timed_calls"]]
    fms = [tot["fast_kernel_ms"] / tot["timed_calls"]]
    hms, jms, gms = [last["hbm_kernel_ms"]], [last["jit_kernel_ms"]], [last["gap_kernel_ms"]]
    njit = [last["n_jit_keys"]]
    res = np.frombuffer(d_out.cpu().numpy().tobytes(), dtype=abi.RESULT_DTYPE)[:my_keys]
    ranks = (D.gather_rows([rank, ka, kb, n_ops, own * 1e3 / args.steps,
                            float(np.mean(kms))])
             if distributed else
             [[0, ka, kb, n_ops, own * 1e3 / args.steps, float(np.mean(kms))]])
    elapsed, (total_ops, n_valid, n_invalid, n_unknown) = reduce_run(
        elapsed, n_ops, res, distributed, dev)
    after_barrier = reduce_run(after_barrier, 0, res, distributed, dev)[0]
    # every rank together, outside the timed region: the one collective path
    fx_ranks = (oversized_key_ranks(abi, world, local)
                if distributed and world > 1 and not args.bare else None)
    # rank 0 alone, the other ranks parked on a CPU (gloo) barrier so no
    # spinning collective kernel shares their GPUs: the drop-in's own
    # multi-GPU path — one lc_ctx over all N GPUs, lc_check from host memory
    fanout = None
    if not args.bare:
        park = None
        if distributed:
            import datetime
            park = dist.new_group(backend="gloo", timeout=datetime.timedelta(seconds=600))
        if rank == 0:
            fanout = fanout_leg(abi, ops, key_off, world, local)
        if park is not None:
            dist.barrier(group=park)

    ms_per_step = elapsed * 1e3 / args.steps
    value = total_ops * args.steps / elapsed
    kernel_ms = float(np.mean(kms))
    fast_ms, jit_ms, gap_ms = float(np.mean(fms)), float(np.mean(jms)), float(np.mean(gms))
    # the dominant kernel: the version-order tier unless a later tier
    # dominates (invalid / crash-heavy workloads)
    dom, dom_ms = max((("fast_tier_kernel", fast_ms), ("gap_tier_kernel", gap_ms),
                       ("lds_tier_kernel", jit_ms)), key=lambda t: t[1])
    algo_bytes = ALGO_BYTES_PER_OP * n_ops + ALGO_BYTES_PER_KEY * my_keys
    achieved = algo_bytes / (dom_ms * 1e-3) / 1e9
    traffic = l2_hit = None
    if os.path.exists(args.traffic_json):
        try:
            tj = json.load(open(args.traffic_json))
            if tj.get("n_ops") == n_ops and tj.get("kernel") == dom:
                traffic = tj.get("hbm_bytes_per_launch")
                l2_hit = tj.get("l2_hit_rate")
        except (ValueError, OSError):
            traffic = None

    line = {
        "metric": METRIC,
        "value": value,
        "unit": "ops/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic (seeded register+version histories, lc_synth_register)",
        "config": {
            "workload": ("C2: %d keys x %d ops/key (packed records), concurrency %d, "
                         "valid CAS-register+version histories" if world == 1 else
                         "C3: the C2 batch (%d keys x %d ops/key, concurrency %d) sharded "
                         "by estimated cost over the GPUs")
                        % (args.keys, args.ops_per_key, args.concurrency),
            "keys": args.keys,
            "ops_per_key": args.ops_per_key,
            "invocations_incl_fail": int(n_inv),
            "concurrency": args.concurrency,
            "p_info": args.p_info,
            "parallelism": "keys sharded by lc_plan_partition, 1 rank per GPU, "
                           "no data-path collective",
        },
        "timing": "job time = max over ranks of each rank's own timed loop (barrier + "
                  "synchronize before it, synchronize after it); ms_after_trailing_barrier "
                  "also counts the closing barrier",
        "ms_after_trailing_barrier": after_barrier * 1e3 / args.steps,
        "ranks": [{"rank": int(r[0]), "keys": [int(r[1]), int(r[2])], "records": int(r[3]),
                   "ms_per_step": r[4], "kernel_ms": r[5]} for r in ranks],
        "rank_ms_per_step_min_max": [min(r[4] for r in ranks), max(r[4] for r in ranks)],
        "roofline": {
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic,
            "kernel": dom,
            "kernel_ms": dom_ms,
            "algorithmic_bytes_per_launch": algo_bytes,
            "algorithmic_bytes": "48 B/op record read + 40 B/key result (DESIGN.md §6)",
            "traffic_source": "rocprofv3 FETCH_SIZE x2 + WRITE_SIZE per launch, "
                              + os.path.relpath(args.traffic_json, ROOT),
            "l2_hit_rate": l2_hit,
        },
        "tiers": {"fast_kernel_ms": fast_ms, "gap_kernel_ms": gap_ms, "jit_kernel_ms": jit_ms,
                  "jit_keys": float(np.mean(njit)), "all_kernels_ms": kernel_ms,
                  "kernel_ms_source": "lc_last_totals: HIP events around the version-order "
                                      "launch on the launch stream, every %d-th of the K timed "
                                      "steps (%d of them; the others LC_FLAG_NO_TIMING), "
                                      "mean" % (TIME_EVERY, tot["timed_calls"])},
        "verdicts": {"valid": n_valid, "invalid": n_invalid, "unknown": n_unknown},
        "hbm_tier_ms": float(np.mean(hms)),
        "cpu_baseline": None,
        "hot_key": None,
    }
    if fx_ranks is not None:
        line["oversized_key_ranks"] = fx_ranks
    if fanout is not None:
        line["fanout_leg"] = fanout
    if rank == 0 and not args.bare:
        if world == 1:  # first, in the timed loop's own state (no leg has run on the context yet)
            line["c3_shards"] = c3_shards(ctx, abi, ops, key_off, d_ops, d_off, dev, stream)
            line["resident32_leg"] = resident32_leg(ctx, abi, ops, key_off, d_ops, d_off, dev, stream)
        line["c1_leg"] = c1_leg(ctx, abi)
        line["host_leg"] = host_leg(ctx, abi, ops, key_off, n_inv)
        line["host_leg32"] = host_leg32(ctx, abi, ops, key_off)
        line["host_leg16"] = host_leg16(ctx, abi, ops, key_off)
        line["hot_key"] = hot_key(ctx, abi)
        line["search_leg"] = search_leg(ctx, abi, d_ops, d_off, d_out, my_keys, stream, n_ops)
        line["mixed_leg"] = mixed_leg(ctx, abi, dev, stream)
        line["dropin_leg"] = dropin_leg(ctx, abi)
        line["model_leg"] = model_leg(ctx, abi)
        line["crash_leg"] = crash_leg(ctx, abi, dev, stream)
        line["oversized_key"] = oversized_key(ctx, abi)

    if rank == 0 and world == 1 and not (args.no_cpu_baseline or args.bare):
        line["cpu_baseline"] = cpu_baseline(args, ops, key_off, res)

    if rank == 0:
        json_out.write(json.dumps(line) + "\n")
        json_out.flush()
    ctx.close()
    if distributed:
        dist.destroy_process_group()


# every TIME_EVERY-th timed step records HIP events around the version-order
# pass (their host cost kept out of the other steps: LC_FLAG_NO_TIMING)
TIME_EVERY = 4


def bind_steps(ctx, abi, d_ops, d_off, n_keys, d_out, stream):
    """[timed step, untimed step]: lc_check_device with the arguments
    converted once, with and without LC_FLAG_NO_TIMING."""
    return [ctx.bind_check_device(d_ops, d_off, n_keys, d_out, stream=stream,
                                  opts=abi.default_opts(flags=f))
            for f in (0, abi.LC_FLAG_NO_TIMING)]


def c3_shards(ctx, abi, ops, key_off, d_ops, d_off, dev, stream, steps=200, warmup=20):
    """A one-GPU predictor of BASELINE configs[2] (C3): the same C2 batch cut
    by lc_plan_partition into 1, 2, 4 and 8 shards, and each shard timed as
    one lc_check_device step on this GPU (a shard of at most one key per
    resident workgroup — 8 shards of C2 — is served by the resident grid:
    kernel_ms is then its device-clock time per request).  A step at N GPUs takes as long as
    its slowest shard (the ranks share nothing but the timing barrier), so
    max over shards is the implied N-GPU step and records / that the implied
    throughput.  A per-shard cost, not a scaling curve: the driver's 8-GPU
    run measures the curve.  Not part of `value`."""
    import torch
    out = []
    n_rec = int(key_off[-1] - key_off[0])
    for n in (1, 2, 4, 8):
        bounds = abi.plan_partition(key_off, n, ops=ops)
        shard_ms = []
        for p in range(n):
            a, b = int(bounds[p]), int(bounds[p + 1])
            outb = torch.zeros(max(b - a, 1) * abi.RESULT_DTYPE.itemsize, dtype=torch.uint8,
                               device=dev)
            st2 = bind_steps(ctx, abi, d_ops.data_ptr() + int(key_off[a] - key_off[0]) * 48,
                             d_off.data_ptr() + a * 8, b - a, outb.data_ptr(), stream.cuda_stream)
            for i in range(warmup):
                st2[i % TIME_EVERY != 0]()
            torch.cuda.synchronize()
            ctx.totals(reset=True)
            t0 = time.perf_counter()
            for i in range(steps):
                st2[i % TIME_EVERY != 0]()
            ctx.quiesce()  # (the resident grid, as in the main loop)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3 / steps
            tot = ctx.totals(reset=True)
            kms = [tot["kernel_ms"] / max(1, tot["timed_calls"])]
            res = np.frombuffer(outb.cpu().numpy().tobytes(), dtype=abi.RESULT_DTYPE)[:b - a]
            shard_ms.append({"keys": [a, b], "ms_per_step": ms, "kernel_ms": float(np.mean(kms)),
                             "valid": int((res["verdict"] == 1).sum())})
        worst = max(x["ms_per_step"] for x in shard_ms)
        out.append({"n_gpus": n, "implied_ms_per_step": worst,
                    "implied_ops_per_s": n_rec / (worst * 1e-3),
                    "shard_ms_min_max": [min(x["ms_per_step"] for x in shard_ms), worst],
                    "shards": shard_ms})
    base = out[0]["implied_ms_per_step"]
    for o in out:
        o["implied_speedup"] = base / o["implied_ms_per_step"]
    return out


def resident32_leg(ctx, abi, ops, key_off, d_ops, d_off, dev, stream, steps=200, warmup=20):
    """The same C2 batch as 24-byte lc_op32 records resident in HBM — the
    format the JVM drop-in and the EDN reader hand over (ABI 4, lc_pack32's
    output) — decided by lc_check_device32, which reads them as they are
    (fast_tier32_kernel; a key handed to the later tiers would be widened
    then), timed as the main loop times lc_check_device (every TIME_EVERY-th
    step with HIP events).  Every result field is compared with the 48-byte
    path's.  Not part of `value`, which stays on the 48-byte records of
    SURVEY §8(b)'s boundary."""
    import torch
    n_keys = len(key_off) - 1
    n_rec = int(key_off[-1] - key_off[0])
    t0 = time.perf_counter()
    o32, base = abi.pack32(ops, key_off)
    pack_ms = (time.perf_counter() - t0) * 1e3
    d32 = torch.from_numpy(np.ascontiguousarray(o32)).to(dev)
    d_base = torch.from_numpy(np.ascontiguousarray(base)).to(dev)
    nb = max(n_keys, 1) * abi.RESULT_DTYPE.itemsize
    out32 = torch.zeros(nb, dtype=torch.uint8, device=dev)
    out48 = torch.zeros(nb, dtype=torch.uint8, device=dev)
    st = [ctx.bind_check_device32(d32.data_ptr(), d_off.data_ptr(), d_base.data_ptr(), n_keys,
                                  out32.data_ptr(), stream=stream.cuda_stream,
                                  opts=abi.default_opts(flags=f))
          for f in (0, abi.LC_FLAG_NO_TIMING)]
    for i in range(warmup):
        st[i % TIME_EVERY != 0]()
    torch.cuda.synchronize()
    ctx.totals(reset=True)
    t0 = time.perf_counter()
    for i in range(steps):
        st[i % TIME_EVERY != 0]()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / steps
    tot = ctx.totals(reset=True)
    kms = tot["fast_kernel_ms"] / max(1, tot["timed_calls"])
    ctx.check_device(d_ops.data_ptr(), d_off.data_ptr(), n_keys, out48.data_ptr(),
                     stream=stream.cuda_stream)
    torch.cuda.synchronize()
    r32 = np.frombuffer(out32.cpu().numpy().tobytes(), dtype=abi.RESULT_DTYPE)[:n_keys]
    r48 = np.frombuffer(out48.cpu().numpy().tobytes(), dtype=abi.RESULT_DTYPE)[:n_keys]
    algo = 24 * n_rec + ALGO_BYTES_PER_KEY * n_keys
    return {"workload": "the C2 batch as 24-byte lc_op32 records resident in HBM (lc_check_device32)",
            "ms_per_step": ms, "ops_per_s": n_rec / (ms * 1e-3), "kernel": "fast_tier32_kernel",
            "kernel_ms": kms, "algorithmic_bytes_per_launch": algo,
            "achieved_gb_per_s": algo / (kms * 1e-3) / 1e9 if kms > 0 else None,
            "frac_of_hbm_peak": algo / (kms * 1e-3) / 1e9 / HBM_PEAK_GBS if kms > 0 else None,
            "pack32_ms": pack_ms, "valid": int((r32["verdict"] == 1).sum()),
            "result_mismatches_vs_48_byte": int((r32 != r48).sum())}


def c1_leg(ctx, abi):
    """BASELINE configs[0] (C1): 100 keys x 200 ops, concurrency 10, the
    configuration the reference's CPU checker is quoted on.  GPU call (host
    buffers) against the oracle's C restatement of knossos on one host thread,
    verdicts compared key by key.  Not part of `value`."""
    import oracle
    ops, off, _, _ = abi.synth(100, 200, concurrency=10, seed=0x5EED0001)
    times = []
    for _ in range(6):
        t0 = time.perf_counter()
        _, r = ctx.check(ops, off)
        times.append((time.perf_counter() - t0) * 1e3)
    # the drop-in's call: the same records as 24-byte lc_op32 (packed before)
    o32, base = abi.pack32(ops, off)
    times32 = []
    for _ in range(6):
        t0 = time.perf_counter()
        _, r32 = ctx.check32(o32, off, base)
        times32.append((time.perf_counter() - t0) * 1e3)
    best = None
    for name, algo in (("jit", oracle.JIT), ("wgl", oracle.WGL)):
        t0 = time.perf_counter()
        _, o = oracle.check(ops, off, algo=algo, n_threads=1)
        dt = (time.perf_counter() - t0) * 1e3
        if best is None or dt < best[1]:
            best = (name, dt, o)
    return {"workload": "C1: 100 keys x 200 ops, concurrency 10 (host buffers)",
            "gpu_call_ms": float(np.median(times[1:])),
            "gpu_call32_ms": float(np.median(times32[1:])),
            "check32_result_mismatches": int((r32 != r).sum()),
            "cpu_oracle_ms": best[1], "cpu_oracle": best[0] + ", 1 thread",
            "valid": int((r["verdict"] == 1).sum()),
            "verdict_mismatches_vs_oracle": int((r["verdict"] != best[2]["verdict"]).sum())}


def host_leg(ctx, abi, ops, key_off, n_inv):
    """The same C2 batch handed over as host buffers (lc_check: H2D copy of
    the 480 MB of records in chunks overlapped with the version-order tier,
    D2H of the results), as a JVM caller would: the PCIe-inclusive rate.
    Never `value`; median of 3 calls."""
    times, profs = [], []
    for _ in range(4):
        t0 = time.perf_counter()
        _, r = ctx.check(ops, key_off)
        times.append(time.perf_counter() - t0)
        profs.append(ctx.call_profile())
    i = 1 + int(np.argsort(times[1:])[1])
    t = times[i]
    return {"workload": "C2 batch from host memory (lc_check, 48-byte records)", "call_ms": t * 1e3,
            "ops_per_s": int(key_off[-1]) / t, "h2d_gb_per_s": ops.nbytes / t / 1e9,
            "profile": profs[i], "valid": int((r["verdict"] == 1).sum())}


def host_leg32(ctx, abi, ops, key_off):
    """The drop-in's rate (ABI 4): the C2 batch as 24-byte lc_op32 records
    (what the JVM packer emits), lc_check32 from host memory — half the PCIe
    bytes of lc_check, chunked copies overlapped with the widening and the
    version-order tier.  Pageable, then page-locked (lc_host_register).
    Results compared with lc_check's field for field.  lc_pack32 (narrowing
    the 48-byte records on the host) is timed apart: a packer that emits
    lc_op32 directly never runs it.  Never `value`; median of 3 calls."""
    t0 = time.perf_counter()
    o32, base = abi.pack32(ops, key_off)
    pack_ms = (time.perf_counter() - t0) * 1e3
    _, want = ctx.check(ops, key_off)
    out = {"workload": "C2 batch from host memory as 24-byte records (lc_check32)",
           "pack32_ms": pack_ms, "bytes": int(o32.nbytes)}
    for mode in ("pageable", "registered"):
        if mode == "registered":
            t0 = time.perf_counter()
            ctx.host_register(o32)
            out["register_ms"] = (time.perf_counter() - t0) * 1e3
        try:
            times, profs, devs = [], [], []
            for _ in range(4):
                t0 = time.perf_counter()
                _, r = ctx.check32(o32, key_off, base)
                times.append(time.perf_counter() - t0)
                profs.append(ctx.call_profile())
                devs.append(ctx.device_stats())
        finally:
            if mode == "registered":
                ctx.host_unregister(o32)
        i = 1 + int(np.argsort(times[1:])[1])
        t = times[i]
        d = devs[i][0]
        out[mode] = {"call_ms": t * 1e3, "ops_per_s": int(key_off[-1]) / t,
                     "h2d_ms": d["h2d_ms"],
                     "h2d_gb_per_s": d["h2d_bytes"] / (d["h2d_ms"] * 1e-3) / 1e9
                     if d["h2d_ms"] > 0 else None,
                     "profile": profs[i], "valid": int((r["verdict"] == 1).sum()),
                     "result_mismatches_vs_lc_check": int((r != want).sum())}
    return out


def host_leg16(ctx, abi, ops, key_off):
    """The drop-in's rate on 16-byte lc_op16 records (round 6: 15-bit value
    ids, which every key of C2 fits — the JVM shim and the EDN reader emit
    them directly when a batch fits): lc_check16 from host memory, a third of
    lc_check's PCIe bytes (two thirds of lc_check32's); chunked copies, each chunk
    widened on the device and decided while the next crosses.  Pageable, then
    page-locked.  Results compared with lc_check's field for field; lc_pack16
    timed apart.  Never `value`; the median of calls 2-4."""
    t0 = time.perf_counter()
    got = abi.pack16(ops, key_off)
    pack_ms = (time.perf_counter() - t0) * 1e3
    if got is None:
        return {"skipped": "an id above LC_ID15_MAX (the batch goes as lc_op32)"}
    o16, base = got
    _, want = ctx.check(ops, key_off)
    out = {"workload": "C2 batch from host memory as 16-byte records (lc_check16)",
           "pack16_ms": pack_ms, "bytes": int(o16.nbytes)}
    for mode in ("pageable", "registered"):
        if mode == "registered":
            t0 = time.perf_counter()
            ctx.host_register(o16)
            out["register_ms"] = (time.perf_counter() - t0) * 1e3
        try:
            times, profs, devs = [], [], []
            for _ in range(4):
                t0 = time.perf_counter()
                _, r = ctx.check16(o16, key_off, base)
                times.append(time.perf_counter() - t0)
                profs.append(ctx.call_profile())
                devs.append(ctx.device_stats())
        finally:
            if mode == "registered":
                ctx.host_unregister(o16)
        i = 1 + int(np.argsort(times[1:])[1])
        t = times[i]
        d = devs[i][0]
        out[mode] = {"call_ms": t * 1e3, "ops_per_s": int(key_off[-1]) / t,
                     "h2d_ms": d["h2d_ms"],
                     "h2d_gb_per_s": d["h2d_bytes"] / (d["h2d_ms"] * 1e-3) / 1e9
                     if d["h2d_ms"] > 0 else None,
                     "profile": profs[i], "valid": int((r["verdict"] == 1).sum()),
                     "result_mismatches_vs_lc_check": int((r != want).sum())}
    return out


def fanout_leg(abi, ops, key_off, world, local, calls=3):
    """BASELINE configs[2] (C3) as the drop-in runs it: ONE lc_ctx over all
    N GPUs of this node (device_mask (1 << N) - 1) and lc_check on the whole
    C2 batch from host memory — the JVM shim's call (lincheck.cpp: one host
    thread and one HIP stream per GPU over its cost-balanced key range, no
    collective; register.clj:108's independent keys).  Per device: key
    range, H2D time (HIP events), kernel time, wall time; aggregate H2D rate.
    A/B: the records as pageable memory, then page-locked by
    lc_host_register (DMA straight from the caller's buffer; registration
    time reported); then the same as 24-byte records (lc_check32, ABI 4).
    Each mode's lc_call_profile attributes the call's wall time (the split,
    the threads' start and end, the join).  Median of `calls` after one warm-up; not `value` (the
    PCIe-inclusive rate).  Rehearsal on one GPU (LC_BENCH_DEVICE): N device
    contexts on that GPU (LC_VIRTUAL_DEVICES)."""
    rehearsal = bool(os.environ.get("LC_BENCH_DEVICE"))
    mask = (1 << local) if rehearsal else (1 << world) - 1
    saved = os.environ.get("LC_VIRTUAL_DEVICES")
    if rehearsal and world > 1:
        os.environ["LC_VIRTUAL_DEVICES"] = str(world)
    out = {"workload": "C2 batch (10000 keys x 1000 ops) from host buffers, one lc_ctx over "
                       "all N GPUs (lc_check's in-process fan-out: the JVM drop-in's path)",
           "rehearsal_virtual_devices": rehearsal and world > 1}
    try:
        ctx = abi.Context(device_mask=mask)
    except Exception as e:  # reported, never fatal to the bench line
        out["error"] = repr(e)
        return out
    finally:
        if saved is None:
            os.environ.pop("LC_VIRTUAL_DEVICES", None)
        else:
            os.environ["LC_VIRTUAL_DEVICES"] = saved
    try:
        o32, base = abi.pack32(ops, key_off)
        for mode in ("pageable", "registered", "pageable32", "registered32"):
            buf = o32 if mode.endswith("32") else ops
            if mode.startswith("registered"):
                t0 = time.perf_counter()
                ctx.host_register(buf)
                out["register_ms" + ("32" if buf is o32 else "")] = (time.perf_counter() - t0) * 1e3
            try:
                rows = []
                for i in range(calls + 1):
                    t0 = time.perf_counter()
                    if buf is o32:
                        _, r = ctx.check32(o32, key_off, base)
                    else:
                        _, r = ctx.check(ops, key_off)
                    ms = (time.perf_counter() - t0) * 1e3
                    if i:
                        rows.append((ms, ctx.device_stats(), ctx.call_profile()))
                rows.sort(key=lambda x: x[0])
                ms, devs, prof = rows[len(rows) // 2]
            finally:
                if mode.startswith("registered"):
                    ctx.host_unregister(buf)
            h2d = sum(d["h2d_bytes"] for d in devs)
            slow = max(d["h2d_ms"] for d in devs)
            out[mode] = {
                "call_ms": ms, "n_devices": len(devs), "profile": prof,
                "ops_per_s": int(key_off[-1] - key_off[0]) / (ms * 1e-3),
                "h2d_gb_per_s_aggregate": h2d / (slow * 1e-3) / 1e9 if slow > 0 else None,
                "valid": int((r["verdict"] == 1).sum()),
                "devices": [{"device": d["device"], "keys": [d["key_begin"], d["key_end"]],
                             "pinned": d["pinned"], "h2d_ms": d["h2d_ms"],
                             "h2d_gb_per_s": d["h2d_bytes"] / (d["h2d_ms"] * 1e-3) / 1e9
                             if d["h2d_ms"] > 0 else None,
                             "kernel_ms": d["kernel_ms"], "total_ms": d["total_ms"]}
                            for d in devs]}
    except Exception as e:  # reported, never fatal to the bench line
        out["error"] = repr(e)
    finally:
        ctx.close()
    return out


def hot_key(ctx, abi):
    """BASELINE configs[3]: one key, 5k ops, concurrency 50, 20 % :info
    (exactly 1,000 crashed writes/CAS of 5,000 records: info_frac 0.2),
    decided by the gap tier (every frontier search, knossos's included, runs
    out of budget on it); also the same shape with injected anomalies, whose
    counterexample search (multisection rounds over the whole GPU) is timed
    too.  Not part of `value`; median of 5 calls after one warm-up."""
    out = {}
    for tag, anom, seed in (("valid", 0.0, 0x5EED0004), ("invalid", 1.0, 1007)):
        ops, off, _, n_inv = abi.synth(1, 5000, concurrency=50, p_info=0.2, info_frac=0.2,
                                       p_anomaly=anom, seed=seed)
        times, gap = [], []
        for _ in range(6):
            t0 = time.perf_counter()
            _, r = ctx.check(ops, off)
            times.append((time.perf_counter() - t0) * 1e3)
            gap.append(ctx.stats()["gap_kernel_ms"])
        out[tag] = {"verdict": int(r["verdict"][0]),
                    "crashed_ops": int((ops[:, 5] == abi.LC_INF).sum()),
                    "matchings": int(r["configs_explored"][0]), "gaps": int(r["max_frontier"][0]),
                    "gap_kernel_ms": float(np.median(gap[1:])),
                    "call_ms": float(np.median(times[1:]))}
        if tag == "invalid":
            out[tag]["fail_op"] = int(r["fail_op"][0])
    v = out["valid"]
    return dict(v, workload="C4: 1 key x 5000 ops, concurrency 50, 20 % (1000) crashed "
                            "writes/CAS (host buffers)",
                invalid=out["invalid"])


def search_leg(ctx, abi, d_ops, d_off, d_out, n_keys, stream, n_ops):
    """The same resident C2 batch (this rank's key range) with the
    version-order and gap tiers off (LC_FLAG_NO_FAST_PATH): every key goes
    through the JIT frontier search (lds_tier_kernel).  Not part of `value`;
    shows the search kernel's rate."""
    import torch
    opts = abi.default_opts(flags=abi.LC_FLAG_NO_FAST_PATH)
    ms, wall = [], []
    for i in range(4):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ctx.check_device(d_ops.data_ptr(), d_off.data_ptr(), n_keys, d_out.data_ptr(),
                         stream=stream.cuda_stream, opts=opts)
        wall.append(time.perf_counter() - t0)
        ms.append(ctx.stats()["jit_kernel_ms"])
    res = np.frombuffer(d_out.cpu().numpy().tobytes(), dtype=abi.RESULT_DTYPE)
    k = float(np.median(ms[1:]))
    return {"workload": "C2 batch, JIT search for every key (LC_FLAG_NO_FAST_PATH)",
            "kernel": "lds_tier_kernel", "kernel_ms": k,
            "ops_per_s": n_ops / (float(np.median(wall[1:]))),
            "kernel_ops_per_s": n_ops / (k * 1e-3),
            "valid": int((res["verdict"] == 1).sum()),
            "max_frontier": int(res["max_frontier"].max())}


def mixed_leg(ctx, abi, dev, stream):
    """BASELINE configs[4] (C5): 1,000 keys x 200 ops, concurrency 10, 10 %
    of keys with an injected stale read or lost CAS.  Invalid keys pass from
    the version-order tier to the gap tier, which names the counterexample.
    Device-resident; verdicts and fail ops checked against the oracle's JIT
    restatement (not part of `value`)."""
    import torch
    import oracle
    ops, off, labels, _ = abi.synth(1000, 200, concurrency=10, p_anomaly=0.1,
                                    seed=0x5EED0005)
    d_ops = torch.from_numpy(ops).to(dev)
    d_off = torch.from_numpy(off).to(dev)
    d_out = torch.zeros(1000 * abi.RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    opts = abi.default_opts()
    wall, st = [], []
    for i in range(6):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ctx.check_device(d_ops.data_ptr(), d_off.data_ptr(), 1000, d_out.data_ptr(),
                         stream=stream.cuda_stream, opts=opts)
        wall.append((time.perf_counter() - t0) * 1e3)
        st.append(ctx.stats())
    res = np.frombuffer(d_out.cpu().numpy().tobytes(), dtype=abi.RESULT_DTYPE)
    _, ref = oracle.check(ops, off, algo=oracle.JIT, n_threads=16)
    mism = int(((res["verdict"] != ref["verdict"]) | (res["fail_op"] != ref["fail_op"])).sum())
    med = lambda f: float(np.median([x[f] for x in st[1:]]))
    return {"workload": "C5: 1000 keys x 200 ops, concurrency 10, 10 % injected anomalies",
            "call_ms": float(np.median(wall[1:])), "fast_kernel_ms": med("fast_kernel_ms"),
            "gap_kernel_ms": med("gap_kernel_ms"), "jit_kernel_ms": med("jit_kernel_ms"),
            "invalid": int((res["verdict"] == 0).sum()),
            "unknown": int((res["verdict"] == -1).sum()),
            "ops_per_s": int(off[-1]) / (float(np.median(wall[1:])) * 1e-3),
            "verdict_or_fail_op_mismatches_vs_oracle": mism}


def dropin_leg(ctx, abi):
    """What a Jepsen user waits for on C5 (BASELINE configs[4]): the drop-in's
    calls from host memory — lc_check32 with witnesses and infeasibility
    certificates (lc_aux), then knossos's :configs for every invalid key in
    one batched device search (lc_check_frontiers) — timed apart and
    together; the configurations compared with the oracle's JITC frontier
    on every invalid key.  Not part of `value`; median of 5 after a warm-up."""
    import oracle
    ops, off, _, _ = abi.synth(1000, 200, concurrency=10, p_anomaly=0.1, seed=0x5EED0005)
    o32, base = abi.pack32(ops, off)
    check_ms, cfg_ms, tot = [], [], []
    for _ in range(6):
        t0 = time.perf_counter()
        _, r, wit, kind, cert, cset = ctx.check32(o32, off, base, witness=True, certificate=True)
        t1 = time.perf_counter()
        inv = np.nonzero(r["verdict"] == 0)[0]
        parts = [ops[off[i]:off[i + 1]] for i in inv]
        sub = np.zeros(len(inv) + 1, dtype=np.int64)
        sub[1:] = np.cumsum([len(p) for p in parts])
        cfgs = ctx.check_frontiers(np.concatenate(parts), sub, r["fail_op"][inv], 10)
        t2 = time.perf_counter()
        check_ms.append((t1 - t0) * 1e3)
        cfg_ms.append((t2 - t1) * 1e3)
        tot.append((t2 - t0) * 1e3)
    bad = n_fallback = 0
    for j, i in enumerate(inv):
        if cfgs[j] is None:
            n_fallback += 1
            continue
        want, n_want = oracle.frontier(parts[j], int(r["fail_op"][i]))
        bad += int(len(cfgs[j]) != min(10, n_want) or any(c not in want for c in cfgs[j]))
    med = lambda x: float(np.median(x[1:]))
    return {"workload": "C5: 1000 keys x 200 ops, 10 % injected anomalies, host buffers",
            "check32_with_witness_and_certificates_ms": med(check_ms),
            "configs_ms": med(cfg_ms), "total_ms": med(tot), "invalid_keys": int(len(inv)),
            "certified_kinds": int((cert[inv, 0] != 0).sum()),
            "configs_keys_left_to_lc_fx_frontier": n_fallback,
            "configs_mismatches_vs_oracle_frontier": bad}


def crash_leg(ctx, abi, dev, stream):
    """C2 with crashes: 10,000 keys x 1,000 ops, concurrency 20, 5 % of the
    writes/CAS crashed (:info), as a run under a partition nemesis leaves
    them.  Every key has crashed ops, so the version-order tier hands each
    over (flag + compaction) and the gap tier decides it.  Device-resident,
    median of 5 calls after one warm-up; not part of `value`."""
    import torch
    ops, off, _, _ = abi.synth(10000, 1000, concurrency=20, p_info=0.05, seed=0x5EED0012)
    d_ops = torch.from_numpy(ops).to(dev)
    d_off = torch.from_numpy(off).to(dev)
    d_out = torch.zeros(10000 * abi.RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    # the timed region is the check call alone; its statistics are read after
    call = ctx.bind_check_device(d_ops.data_ptr(), d_off.data_ptr(), 10000, d_out.data_ptr(),
                                 stream=stream.cuda_stream)
    wall, fast, gap = [], [], []
    for _ in range(6):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        call()
        wall.append((time.perf_counter() - t0) * 1e3)
        st = ctx.stats()
        fast.append(st["fast_kernel_ms"])
        gap.append(st["gap_kernel_ms"])
    res = np.frombuffer(d_out.cpu().numpy().tobytes(), dtype=abi.RESULT_DTYPE)
    t = float(np.median(wall[1:]))
    return {"workload": "C2 with 5 % crashed writes/CAS: 10000 keys x 1000 ops, concurrency 20",
            "call_ms": t, "ops_per_s": int(off[-1]) / (t * 1e-3),
            "fast_kernel_ms": float(np.median(fast[1:])), "gap_kernel_ms": float(np.median(gap[1:])),
            "crashed_ops": int((ops[:, 5] == abi.LC_INF).sum()),
            "valid": int((res["verdict"] == 1).sum()), "unknown": int((res["verdict"] == -1).sum())}


def model_leg(ctx, abi):
    """knossos's cas-register model (no versions) on C2-shaped histories,
    1,000 keys x 1,000 ops, concurrency 20: without version pinning every key
    needs the frontier search and its HBM tier (§9 of DESIGN.md).  Not part
    of `value`; median of 5 calls after one warm-up."""
    ops, off, _, _ = abi.synth(1000, 1000, concurrency=20, seed=7)
    ops = ops.copy()
    ops[:, 3] = abi.LC_NIL  # cas-register: the same histories without versions
    times, st = [], []
    for _ in range(6):
        t0 = time.perf_counter()
        _, r = ctx.check(ops, off)
        times.append((time.perf_counter() - t0) * 1e3)
        st.append(ctx.stats())
    t = float(np.median(times[1:]))
    hbm_ms = float(np.median([x["hbm_kernel_ms"] for x in st[1:]]))
    explored = int(r["configs_explored"].sum())
    # the same batch as the drop-ins send it (checker.py, mi355x.clj: 16-byte
    # records when every id fits): a third of the PCIe bytes; beside call_ms
    # (48-byte records), which stays the leg's figure
    call16 = None
    p16 = abi.pack16(ops, off)
    if p16 is not None:
        t16 = []
        for _ in range(4):
            t0 = time.perf_counter()
            _, r16 = ctx.check16(p16[0], off, p16[1])
            t16.append((time.perf_counter() - t0) * 1e3)
        call16 = {"call_ms": float(np.median(t16[1:])),
                  "result_mismatches_vs_48_byte": int((r16 != r).sum())}
    # the roofline SURVEY §8(d) states for the search: one 128-B table probe
    # per configuration explored, against the HBM peak; beside it the
    # counters' own traffic of hbm_coop_kernel<4> (a PMC pass of this leg,
    # tools/pmc_kernel.sh + pmc_summary.py: the probes mostly hit LDS tables
    # and L2, so the search is bound by its probes' latency, not by HBM)
    roof = {"bound": "probe latency (LDS/L2 tables)", "unit": "GB/s", "peak": HBM_PEAK_GBS,
            "bytes_per_probe": 128, "kernel": "hbm_coop_kernel<4>", "kernel_ms": hbm_ms}
    if hbm_ms > 0:
        roof["achieved"] = 128.0 * explored / (hbm_ms * 1e-3) / 1e9
        roof["frac"] = roof["achieved"] / HBM_PEAK_GBS
    pmc = os.path.join(ROOT, "profiles", "r06", "pmc_model_hbm_coop4.json")
    if os.path.exists(pmc):
        try:
            dj = json.load(open(pmc))["derived"]
            roof["traffic_source"] = os.path.relpath(pmc, ROOT)
            for k in ("hbm_bytes", "hbm_gb_per_s", "l2_hit_rate", "wait_any_frac_of_wave_cycles",
                      "active_inst_frac_of_wave_cycles", "lds_bank_conflict_cycles_per_lds_inst"):
                if k in dj:
                    roof[k] = dj[k]
        except (ValueError, OSError, KeyError):
            pass
    return {"workload": "cas-register model: 1000 keys x 1000 ops, concurrency 20 (host buffers)",
            "roofline": roof,
            "call_ms": t, "ops_per_s": int(off[-1]) / (t * 1e-3),
            "jit_kernel_ms": float(np.median([x["jit_kernel_ms"] for x in st[1:]])),
            "hbm_kernel_ms": hbm_ms,
            "hbm_keys": int(st[-1]["n_hbm_keys"]),
            "configs_explored": explored,
            # probe throughput: every configuration explored is one dedup probe
            # (most in LDS tables since round 2; HBM bytes per probe from the
            # PMC pass, profiles/r06/pmc_model_hbm_coop4.json)
            "probes_per_s": explored / (hbm_ms * 1e-3) if hbm_ms > 0 else None,
            "max_frontier": int(r["max_frontier"].max()),
            "records16": call16,
            "valid": int((r["verdict"] == 1).sum()), "unknown": int((r["verdict"] == -1).sum())}


def oversized_key_ops(abi):
    """One version-less key (cas-register model) of 2,000 ops at concurrency
    50: frontiers of up to 115,648 configurations, 72 M explored."""
    ops, off, _, _ = abi.synth(1, 2000, concurrency=50, seed=0x5EED0004)
    ops = ops.copy()
    ops[:, 3] = abi.LC_NIL
    return ops, off


def oversized_key_ranks(abi, world, local):
    """SURVEY §8(e)'s exchange on real ranks: the oversized key searched by
    every rank together (include/lincheck_fx.h), its frontier partitioned by
    hash owner while above 16,384 configurations, successors exchanged by an
    all-to-all-v per level.  Collectives by the library's own RCCL transport
    (lc_fx_open_rccl: ncclCommInitRank, counts by ncclAllToAll on the device,
    payload by grouped ncclSend / ncclRecv on the engine's stream; the unique
    id travels over the bench's process group), with a watchdog that aborts
    the communicators (lc_fx_abort) rather than let a stuck collective hang
    the bench.  LC_BENCH_FX_BACKEND=gloo|nccl drives the same engine through
    torch.distributed callbacks instead.  Not part of `value`; every rank
    returns the same result."""
    import datetime
    import threading
    import torch.distributed as dist
    from jepsen.etcd_amd.fx import FrontierExchange
    backend = os.environ.get("LC_BENCH_FX_BACKEND", "rccl")
    fx = None
    timer = None
    try:
        ops, _ = oversized_key_ops(abi)
        if backend == "rccl":
            group = dist.new_group(backend="gloo", timeout=datetime.timedelta(seconds=120))
            fx = FrontierExchange(device=local, rccl_group=group, part_above=16384)
        else:
            group = (dist.new_group(backend="gloo", timeout=datetime.timedelta(seconds=120))
                     if backend == "gloo" else dist.group.WORLD)
            fx = FrontierExchange(device=local, group=group, part_above=16384)
        timer = threading.Timer(120.0, fx.abort)
        timer.daemon = True
        timer.start()
        fx.check(ops)  # warm-up (allocations)
        dist.barrier(group=group)
        t0 = time.perf_counter()
        r = fx.check(ops)
        ms = (time.perf_counter() - t0) * 1e3
        st = fx.stats()
        return {"ranks": world, "backend": backend, "ms": ms, "verdict": int(r["verdict"]),
                "configs_explored": int(r["configs_explored"]),
                "max_frontier": int(r["max_frontier"]),
                "part_returns": st["part_returns"], "part_levels": st["part_levels"],
                "gathers": st["gathers"], "sent_configs_rank0": st["sent_configs"],
                "max_local_frontier_rank0": st["max_local_frontier"]}
    except Exception as e:  # reported, never fatal to the bench line
        return {"ranks": world, "backend": backend, "error": repr(e)}
    finally:
        if timer is not None:
            timer.cancel()
            timer.join()  # a callback already running (fx.abort) ends before fx.close()
        if fx is not None:
            fx.close()


def oversized_key(ctx, abi):
    """SURVEY §8(e)'s one exception: a single key too large for one
    workgroup.  The frontier exchange (include/lincheck_fx.h) runs its JIT
    search over the whole GPU; lc_check's tiers give the same key one
    cooperative workgroup and its configuration budget.  Not part of `value`."""
    from jepsen.etcd_amd.fx import FrontierExchange
    ops, off = oversized_key_ops(abi)
    with FrontierExchange(device=0) as fx:
        fx.check(ops)  # warm-up (table allocation)
        times = []
        for _ in range(3):
            t0 = time.perf_counter()
            r = fx.check(ops)
            times.append((time.perf_counter() - t0) * 1e3)
        st = fx.stats()
    t = min(times)
    t0 = time.perf_counter()
    _, rt = ctx.check(ops, off)
    tiers_ms = (time.perf_counter() - t0) * 1e3
    return {"workload": "1 key x 2000 ops, concurrency 50, cas-register model (no versions; host buffers)",
            "fx_ms": t, "verdict": int(r["verdict"]), "configs_explored": int(r["configs_explored"]),
            "max_frontier": int(r["max_frontier"]),
            "configs_per_s": int(r["configs_explored"]) / (t * 1e-3),
            "returns": st["returns"], "levels": st["levels"], "redos": st["redos"],
            "tiers": {"call_ms": tiers_ms, "verdict": int(rt["verdict"][0]),
                      "reason": abi.REASONS.get(int(rt["reason"][0])),
                      "configs_explored": int(rt["configs_explored"][0])}}


def reduce_run(elapsed, n_ops, res, distributed, dev):
    """Whole-job numbers: the MAX of the ranks' timed-region wall times and
    the SUM of their checked ops and verdict counts (every rank checks its
    own key range of the one batch, so the sums are the whole batch's)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    counts = torch.tensor([n_ops, int((res["verdict"] == 1).sum()),
                           int((res["verdict"] == 0).sum()),
                           int((res["verdict"] == -1).sum())],
                          dtype=torch.int64, device=dev)
    if distributed:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(counts)
    return float(t.item()), [int(v) for v in counts.tolist()]


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(args, ops, key_off, gpu_res):
    """The oracle (C restatement of knossos.linear / knossos.wgl; no JVM on
    the box, so not Knossos itself) on the first --cpu-sample-keys keys of the
    same workload, on --cpu-threads host threads.  Knossos races both
    analyzers per key; the faster analyzer's whole-sample rate is reported.
    Also checks the sample's verdicts against the GPU's."""
    import oracle
    k = min(args.cpu_sample_keys, len(key_off) - 1)
    sub_ops = ops[: key_off[k]]
    sub_off = key_off[: k + 1]
    best = None
    mism = 0
    for name, algo in (("jit", oracle.JIT), ("wgl", oracle.WGL)):
        t0 = time.perf_counter()
        _, r = oracle.check(sub_ops, sub_off, algo=algo, n_threads=args.cpu_threads)
        dt = time.perf_counter() - t0
        mism += int((r["verdict"] != gpu_res["verdict"][:k]).sum())
        rate = len(sub_ops) / dt
        if best is None or rate > best[0]:
            best = (rate, name, dt)
    return {
        "value": best[0],
        "unit": "ops/s",
        "cores": args.cpu_threads,
        "host_nproc": os.cpu_count(),
        "cpu_model": cpu_model(),
        "cores_note": "threads used = this box's CPU share; host_nproc counts the whole machine",
        "kind": "port",
        "sample": "%d keys x %d ops of the same C2 workload (%d records), "
                  "oracle/%s restatement of knossos (faster of jit/wgl), %.1f s"
                  % (k, args.ops_per_key, len(sub_ops), best[1], best[2]),
        "verdict_mismatches_vs_gpu": mism,
        "model_leg": cpu_model_leg(args),
        "oversized_key": cpu_oversized_key(),
    }


def cpu_oversized_key():
    """The oversized key on one host thread: the oracle's JIT with the GPU's
    exact reductions (oracle.JITC) — one key's search is sequential, in the
    oracle as in knossos.  Compare with oversized_key.fx_ms."""
    import oracle
    from jepsen.etcd_amd import abi
    ops, off = oversized_key_ops(abi)
    t0 = time.perf_counter()
    _, r = oracle.check(ops, off, algo=oracle.JITC, n_threads=1, max_configs=1 << 24)
    dt = time.perf_counter() - t0
    return {"value": int(r["configs_explored"][0]) / dt, "unit": "configs/s", "cores": 1,
            "kind": "port", "ms": dt * 1e3, "verdict": int(r["verdict"][0]),
            "sample": "the whole oversized key (2000 ops), oracle JITC, %.1f s" % dt,
            "configs_explored": int(r["configs_explored"][0])}


def cpu_model_leg(args, n_keys=200):
    """The model leg's workload (version-less, 1,000 ops, concurrency 20) on
    the CPU: the oracle's JIT with the same exact reductions as the GPU's
    search (oracle.JITC), on the first n_keys keys, same threads.  Compare
    with model_leg.ops_per_s (whole 1,000-key batch, host buffers)."""
    import oracle
    from jepsen.etcd_amd import abi
    ops, off, _, _ = abi.synth(1000, 1000, concurrency=20, seed=7)
    ops = ops.copy()
    ops[:, 3] = abi.LC_NIL
    sub_ops, sub_off = ops[: off[n_keys]], off[: n_keys + 1]
    t0 = time.perf_counter()
    _, r = oracle.check(sub_ops, sub_off, algo=oracle.JITC, n_threads=args.cpu_threads,
                        max_configs=1 << 24)
    dt = time.perf_counter() - t0
    return {"value": len(sub_ops) / dt, "unit": "ops/s", "cores": args.cpu_threads,
            "kind": "port",
            "sample": "%d keys x 1000 ops of the model leg's workload, oracle JITC (knossos.linear "
                      "restated with the GPU's exact reductions), %.2f s" % (n_keys, dt),
            "configs_explored": int(r["configs_explored"].sum())}


if __name__ == "__main__":
    main()
