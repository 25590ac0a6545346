# live-slot / GEMM-plan sweep of the streaming schedule (K=10, K=20), device-moment tests
export TMPDIR=/tmp
out=gpurun_out/r5d
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_prepare_gpu.py -x -v --timeout 170 --timeout-method thread > $out/pytest_prep.log 2>&1
echo pytest_rc=$?
run() {  # name, env..., -- bench args
  local name=$1; shift
  timeout -k 10 200 env "$@" > $out/$name.log 2>&1 || { echo "FAIL $name"; return 1; }
  python - "$out/$name.log" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d["value"], d["ms_per_step"], d["config"].get("schedule", "")[:160])
PY
}
run k10_L100 CNMF_GEMM_WAVE_PLAN=1 python bench.py --live 100 &&
run k10_L112 CNMF_GEMM_WAVE_PLAN=1 python bench.py --live 112 &&
run k10_L128 CNMF_GEMM_WAVE_PLAN=1 python bench.py --live 128 &&
run k10_L137 CNMF_GEMM_WAVE_PLAN=1 python bench.py --live 137 &&
run k10_L128_nw CNMF_GEMM_WAVE_PLAN=0 python bench.py --live 128 &&
run k10_L137_nw CNMF_GEMM_WAVE_PLAN=0 python bench.py --live 137 &&
run k10_L137_mf4 CNMF_STREAM_MIN_FILL=4 python bench.py --live 137 &&
run k20_L64 CNMF_GEMM_WAVE_PLAN=1 python bench.py --k 20 --live 64 &&
run k20_L80 CNMF_GEMM_WAVE_PLAN=1 python bench.py --k 20 --live 80 &&
run k20_L100 CNMF_GEMM_WAVE_PLAN=1 python bench.py --k 20 --live 100 &&
run k20_batch CNMF_GEMM_WAVE_PLAN=1 python bench.py --k 20 --schedule batch &&
run grid_batch CNMF_GEMM_WAVE_PLAN=1 python bench.py --kmin 5 --kmax 13 --steps 6 --warmup 2 --schedule batch &&
run grid_L64 CNMF_GEMM_WAVE_PLAN=1 python bench.py --kmin 5 --kmax 13 --steps 6 --warmup 2 --live 64
echo rc=$?
