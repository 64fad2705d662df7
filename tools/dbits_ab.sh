# bench with sign-bit D activations from 512^2 (default), from 1024^2 only, and off
cd "$(dirname "$0")/.."
for r in 1 2; do for v in 512 1024 4096; do
  echo "== $v"; PG_DBITS_MIN_RES=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-baseline off --no-kernel-events 2>&1 | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])" || exit 1
done; done
