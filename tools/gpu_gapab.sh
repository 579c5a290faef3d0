# Dev: gap-tier A/B — in-tree against each tools/variants/<v> named, C4 / C4x / C4x1004 / C5
# timings (gap_probe.py), interleaved twice
set -o pipefail
for rep in 1 2; do
  for v in in-tree "$@"; do
    if [ "$v" = in-tree ]; then
      out=$(timeout -k 10 100 python tools/gap_probe.py 3 C4,C4x,C4x1004,C5 2>/dev/null) || exit 1
    else
      out=$(LINCHECK_LIB=tools/variants/$v/liblincheck.so timeout -k 10 100 python tools/gap_probe.py 3 C4,C4x,C4x1004,C5 2>/dev/null) || exit 1
    fi
    echo "$v $(echo "$out" | python -c "
import sys, json, collections
d = collections.defaultdict(list)
for l in sys.stdin:
    if l.startswith('{'):
        j = json.loads(l); d[j['cfg']].append((j['wall_ms'], j['gap_ms'], j['invalid'], j['valid']))
print(' '.join('%s %.3f/%.3f v%d/i%d' % (k, min(x[0] for x in v[1:]), min(x[1] for x in v[1:]), v[-1][3], v[-1][2]) for k, v in d.items()))")"
  done
done
