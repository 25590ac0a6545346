# env A/B at HEAD for K=20 / K=30: device slots off, slice width 320 / 448
export TMPDIR=/tmp
out=gpurun_out/r4zi
mkdir -p $out
run() { tag=$1; k=$2; shift 2; env "$@" timeout -k 10 150 python bench.py --k $k > $out/$tag.log 2>&1 && tail -1 $out/$tag.log | python -c "import json,sys; print('$tag', json.loads(sys.stdin.read())['value'])"; }
for r in 1 2; do
run k20_base$r 20 A=1 && run k20_noslots$r 20 CNMF_DEV_SLOTS=0 && run k20_c320_$r 20 CNMF_PIPE_SLICE_COLS=320 && run k20_c448_$r 20 CNMF_PIPE_SLICE_COLS=448 &&
run k30_base$r 30 A=1 && run k30_noslots$r 30 CNMF_DEV_SLOTS=0 && run k30_c320_$r 30 CNMF_PIPE_SLICE_COLS=320 && run k30_c448_$r 30 CNMF_PIPE_SLICE_COLS=448 || exit 1
done
echo rc=$?
