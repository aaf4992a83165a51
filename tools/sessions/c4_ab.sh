# C4 fused enc/dec timing (bench.py's cfg_C4 entry of the default run), two runs
set -e
for r in 1 2; do timeout -k 10 400 python bench.py --no-cpu --steps 10 2>/dev/null | grep '^{' | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["cfg_C4"])'; done
