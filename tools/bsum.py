"""Print the headline numbers of bench.py JSON lines in the given logs (value, ms/step, stage times, per-path stats)."""
import json
import sys

for f in sys.argv[1:]:
    lines = [x for x in open(f) if x.startswith("{")]
    if not lines:
        print(f, "no JSON line")
        continue
    d = json.loads(lines[-1])
    r = d.get("roofline", {})
    os_ = r.get("onestep_regime", {})
    print(f, "value", d["value"], "ms/step", d["ms_per_step"], "stages", d.get("stages_ms_last_frame"),
          "onestep_ms", os_.get("ms"), "field_w", r.get("field_sample_weighted", {}).get("frac"), "net_frac", r.get("frac"),
          "per_launch", [(p["samples"], p["ms"], p["frac"]) for p in r.get("per_launch") or []])
