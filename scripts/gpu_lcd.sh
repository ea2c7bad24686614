set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests/test_lcd_gpu.py -x -q -m gpu 2>&1 | tail -25
timeout -k 10 300 python scripts/lcd_timing.py ${LCD_N:-2000}
