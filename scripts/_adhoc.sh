set -o pipefail
for i in 1 2; do
timeout -k 10 300 python scripts/_bench_prev.py --steps 30 --warmup 6 2>&1 | tail -1 | cut -c1-150
timeout -k 10 300 python bench.py --steps 30 --warmup 6 2>&1 | tail -1 | cut -c1-150
done
