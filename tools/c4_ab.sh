# C4 fused enc/dec timing (bench.py --extra), two runs
set -e
for r in 1 2; do timeout -k 10 300 python bench.py --extra --no-cpu --steps 10 2>/dev/null | grep '^{' | python3 -c 'import json,sys; d=json.loads(sys.stdin.read())["extra"]; print({k: v for k, v in d.items() if "C4" in k})'; done
