"""One-line summary of a bench.py JSON (used by scripts/gpu.sh)."""
import json
import sys

# the last JSON line (gloo rehearsals print their own connection lines first)
d = json.loads([ln for ln in open(sys.argv[1]).read().splitlines() if ln.startswith("{")][-1])
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
    for k in ("hamming", "bow"):
        if isinstance(lcd.get(k), dict):
            parts.append(f"lcd.{k}={lcd[k].get('value')}")
    st = lcd.get("stream")
    if isinstance(st, dict):
        parts.append(f"lcd.stream_us_per_frame={st.get('us_per_frame')}")
        if isinstance(st.get("verify_matches"), dict):
            parts.append(f"lcd.verify_matches={st['verify_matches'].get('value')}")
print(" ".join(parts))
