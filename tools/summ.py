"""Print the headline fields of bench.py JSON lines (dev helper)."""
import json
import sys

for f in sys.argv[1:]:
    line = [l for l in open(f).read().strip().splitlines() if l.startswith("{")][-1]
    d = json.loads(line)
    r = d.get("roofline") or {}
    print(f, "ms/step", round(d["ms_per_step"], 4), "frac", round(r.get("frac", 0), 4),
          {k: (round(v["ms"], 4), round(v["GB/s"])) for k, v in r.get("per_kernel", {}).items()})
