"""Dev: the stored-history path end to end, as `python -m jepsen.etcd_amd.edn`
runs it: a Jepsen-style history.edn (edn.to_edn of a synthetic history: one op
map per line, nemesis ops mixed in, 2 % crashed ops) is parsed by the native
reader on N threads (scan, parse, per-key split, knossos completion, packing)
and every key is decided in one GPU call.  Prints one JSON line; the parse
phases come from LC_EDN_TIMING on stderr.
    python tools/edn_e2e.py [keys] [ops_per_key] [threads] [reps]"""
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from jepsen.etcd_amd import abi, edn, synth  # noqa: E402

nk = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
threads = int(sys.argv[3]) if len(sys.argv) > 3 else 16
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 3
t0 = time.perf_counter()
hist, _ = synth.jepsen_history(nk, n, concurrency=20, p_info=0.02, seed=5)
path = os.path.join(tempfile.gettempdir(), "lc_e2e_history.edn")
with open(path, "w") as f:
    f.write(edn.to_edn(hist))
del hist
size = os.path.getsize(path)
print("history written: %.1f MB in %.1f s" % (size / 1e6, time.perf_counter() - t0), flush=True)
out = {"keys": nk, "ops_per_key": n, "history_mb": round(size / 1e6, 1), "threads": threads}
parse, check = [], []
with abi.Context(device_mask=1) as ctx:
    for rep in range(reps):
        a = time.perf_counter()
        h = edn.read(path, n_threads=threads)
        b = time.perf_counter()
        result, _ = edn.check(h, ctx=ctx)
        c = time.perf_counter()
        parse.append(b - a)
        check.append(c - b)
        print("rep %d: parse %.3f s, check %.1f ms" % (rep, b - a, (c - b) * 1e3), flush=True)
        out["events"] = int(h.n_events)
        out["records"] = int(h.key_off[-1])
        out["failures"] = len(result["failures"])
        del h
os.remove(path)
out["parse_s"] = round(min(parse), 3)
out["parse_mb_per_s"] = round(size / 1e6 / min(parse), 1)
out["check_ms"] = round(min(check) * 1e3, 2)
out["end_to_end_s"] = round(min(p + q for p, q in zip(parse, check)), 3)
print(json.dumps(out))
