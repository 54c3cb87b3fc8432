# development: one GPU step
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_xxh3.py -m gpu -x -v --timeout 120 --timeout-method thread 2>&1 | grep -E "PASS|FAIL|Error|passed|failed|assert" | tail -15
