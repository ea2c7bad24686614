set -o pipefail
timeout -k 10 300 python -m pytest tests -x -q -m gpu 2>&1 | tail -3
timeout -k 10 300 python scripts/gather_bench.py synth100k ${GB_VARIANTS:-0,10,20,30,31,32,33}
