# device-side streaming swap (stream.hip): tests, K=10 / K=20 / grid, kernel trace
export TMPDIR=/tmp
out=gpurun_out/r5e
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_solve_pipe_gpu.py -x -v --timeout 170 --timeout-method thread -k "stream" > $out/pytest_stream.log 2>&1 || { echo PYTEST_FAILED; grep -E "Error|assert|FAILED|passed|failed" $out/pytest_stream.log | head -30; exit 1; }
run() {  # name, env..., -- bench args
  local name=$1; shift
  timeout -k 10 200 env "$@" > $out/$name.log 2>&1 || { echo "FAIL $name"; tail -20 $out/$name.log; return 1; }
  python - "$out/$name.log" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d["value"], d["ms_per_step"], d["config"].get("schedule", "")[:200])
PY
}
run k10 CNMF_GEMM_WAVE_PLAN=1 python bench.py &&
run k10_L128 CNMF_GEMM_WAVE_PLAN=1 python bench.py --live 128 &&
run k10_L100 CNMF_GEMM_WAVE_PLAN=1 python bench.py --live 100 &&
run k20_L80 CNMF_GEMM_WAVE_PLAN=1 python bench.py --k 20 &&
run k20_L100 CNMF_GEMM_WAVE_PLAN=1 python bench.py --k 20 --live 100 &&
run grid_L137 CNMF_GEMM_WAVE_PLAN=1 python bench.py --kmin 5 --kmax 13 --steps 6 --warmup 2 &&
run grid_L100 CNMF_GEMM_WAVE_PLAN=1 python bench.py --kmin 5 --kmax 13 --steps 6 --warmup 2 --live 100 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_stream -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 > $out/prof_stream.log 2>&1
echo rc=$?
