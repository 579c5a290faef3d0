"""Summarise an interleaved leg A/B file (tools/gpu_r6l.sh): per variant, the
median HBM-tier and call times over the warm calls, and the configurations."""
import json
import statistics
import sys

cur, d = None, {}
for line in open(sys.argv[1]):
    if line.startswith("=="):
        cur = line.split()[1]
        continue
    if line.startswith("{"):
        j = json.loads(line)
        if j["rep"] == 0:
            continue  # (the first call of a process: warm-up)
        d.setdefault(cur, []).append((j["hbm_ms"], j["wall_ms"], j["configs"]))
for k, v in d.items():
    print(k, "hbm_ms %.2f" % statistics.median(x[0] for x in v), "call_ms %.2f" % statistics.median(x[1] for x in v),
          "configs", sorted(set(x[2] for x in v)), "n", len(v))
