"""Print the headline numbers of bench.py JSON lines (C2 roofline, C3, C4, unstructured, c2_arrays, C5)."""
import json
import sys

for f in sys.argv[1:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    r = d.get("roofline", {})
    out = [f, "C2 %.4f ms/step kern %.4f frac %.4f" % (d["ms_per_step"], r.get("kernel_ms", 0), r.get("frac", 0)),
           "cg %.1f it/s" % d.get("cg_iter_per_s", 0)]
    for leg in ("c4", "c3", "unstructured", "c2_arrays"):
        if leg in d and isinstance(d[leg], dict):
            L = d[leg]
            km = L.get("kernel_ms_median", L.get("kernel_ms"))
            out.append("%s %s ms frac %s" % (leg, km, (L.get("roofline") or {}).get("frac")))
    if "c5" in d and isinstance(d["c5"], dict):
        out.append("c5 %s ms/step" % d["c5"].get("ms_per_step"))
    print(" | ".join(out))
