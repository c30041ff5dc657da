"""Exit 0 only if every solo (precision 3) row of tools/solo_probe.py's output is within the bf16
gate (>= 99.9 % of elements within 5 % of |f32| + 0.1 max|f32|): run before timing variants."""
import json
import sys

ok = True
n = 0
for line in open(sys.argv[1]):
    if line.startswith("{") and '"p3_ok"' in line:
        d = json.loads(line)
        n += 1
        if d["p3_ok"] < 0.999 or not d["p3_finite"]:
            ok = False
            print("solo kernel out of gate:", d)
print("solo gate", "ok" if ok and n else "FAILED", n, "rows")
sys.exit(0 if ok and n else 1)
