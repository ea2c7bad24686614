"""One-line summary of a bench.py JSON (used by scripts/gpu.sh)."""
import json
import sys

d = json.load(open(sys.argv[1]))
parts = [f"{d['metric'][:24]}={d['value']:.4g}", f"ms/step={d.get('ms_per_step')}"]
rf = d.get("roofline") or {}
if rf:
    parts.append(f"frac={rf.get('frac')}")
par = d.get("parity") or {}
if par:
    parts.append(f"parity={par.get('ok')}")
cb = d.get("cpu_baseline") or {}
if cb:
    parts.append(f"cpu={cb.get('value')}")
lcd = d.get("lcd") or {}
if lcd:
    parts.append(f"lcd={lcd.get('value')}")
    for k in ("hamming", "stream", "bow"):
        if isinstance(lcd.get(k), dict):
            parts.append(f"lcd.{k}={lcd[k].get('value')}")
print(" ".join(parts))
