# Round-end validation: every GPU test, smoke, the headline at the driver's 20 and 40
# steps, KL / K-grid benches, five e2e pipeline runs, a kernel trace of the headline.
# usage: bash tools/gpu/round_end.sh <tag>   (logs under gpurun_out/<tag>)
exec bash "$(dirname "$0")/run.sh" "$1" pytest smoke \
  'bench|150|python bench.py --steps 20 --warmup 5' \
  'bench40|150|python bench.py --steps 40 --warmup 5 --no-stream-value' \
  'bench_kl|300|python bench.py --beta-loss kullback-leibler --steps 3 --warmup 1' \
  'grid|150|python bench.py --kmin 5 --kmax 13 --steps 5 --warmup 2' \
  'e2e1|200|python tools/bench_e2e.py' 'e2e2|200|python tools/bench_e2e.py' \
  'e2e3|200|python tools/bench_e2e.py' 'e2e4|200|python tools/bench_e2e.py' \
  'e2e5|200|python tools/bench_e2e.py' \
  "prof|240|rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$1 -o run -- python3 bench.py --steps 10 --warmup 3 --no-stream-value" \
  "prof_cp|30|cp /tmp/prof_$1/run_kernel_stats.csv gpurun_out/$1/headline_kernel_stats.csv"
