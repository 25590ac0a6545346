# device-swap streaming v2 (in-ring staging, host mailbox, vector swap copies)
export TMPDIR=/tmp
out=gpurun_out/r5f
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_solve_pipe_gpu.py -x -v --timeout 170 --timeout-method thread -k "stream" > $out/pytest_stream.log 2>&1 || { echo PYTEST_FAILED; grep -E "Error|assert|FAILED|passed|failed" $out/pytest_stream.log | head -30; exit 1; }
run() {
  local name=$1; shift
  timeout -k 10 200 env "$@" > $out/$name.log 2>&1 || { echo "FAIL $name"; tail -20 $out/$name.log; return 1; }
  python - "$out/$name.log" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d["value"], d["ms_per_step"], d["config"].get("schedule", "")[:220])
PY
}
run k10 python bench.py &&
run k10b python bench.py &&
run k10_L128 python bench.py --live 128 &&
run grid python bench.py --kmin 5 --kmax 13 --steps 6 --warmup 2 &&
run k20 python bench.py --k 20 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_stream -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 > $out/prof_stream.log 2>&1
echo rc=$?
