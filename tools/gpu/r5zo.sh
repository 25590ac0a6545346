# k-selection threads 4 vs 8 (e2e x2 each)
export TMPDIR=/tmp
out=gpurun_out/r5zo
mkdir -p $out
for t in 4 8 4 8; do
  sed -i "s/^_KSEL_THREADS = .*/_KSEL_THREADS = $t/" cnmf_torch_amd/api.py
  timeout -k 10 300 python tools/bench_e2e.py > $out/e2e_t$t.log 2>&1 || { echo E2E_FAILED; tail -20 $out/e2e_t$t.log; exit 1; }
  echo "threads=$t $(tail -n 1 $out/e2e_t$t.log | cut -c1-200)"
done
