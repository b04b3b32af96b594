"""One-line digest of a bench.py JSON line: headline, median step, roofline,
batch sweep, the latency legs and the host / TS legs when present.
    python tools/bench_brief.py BENCH.json"""
import json
import sys

d = json.load(open(sys.argv[1]))
rf = d.get("roofline") or {}
out = [f"value {d['value']:.1f}", f"median {d.get('value_at_median_step')}",
       f"ms/step {d.get('ms_per_step')}",
       f"dominant {rf.get('kernel', '')[:60]} frac {rf.get('frac')} achieved {rf.get('achieved')}"]
if d.get("batch_sweep"):
    out.append("sweep " + " ".join(f"b{s['batch']}/{s['inflight']}:{s['value']:.0f}" for s in d["batch_sweep"]))
if d.get("latency"):
    out.append("latency " + json.dumps(d["latency"])[:400])
hp = d.get("host_path")
if hp:
    out.append("host " + json.dumps(hp)[:300])
ts = d.get("ts_path")
if ts:
    out.append("ts " + json.dumps(ts)[:300])
print(" | ".join(out))
