# env A/B at HEAD on the headline: flag side stream, device slots at K=10, late compaction fraction
export TMPDIR=/tmp
out=gpurun_out/r4zh
mkdir -p $out
run() { tag=$1; shift; env "$@" timeout -k 10 120 python bench.py > $out/$tag.log 2>&1 && tail -1 $out/$tag.log | python -c "import json,sys; print('$tag', json.loads(sys.stdin.read())['value'])"; }
run base1 A=1 && run flag CNMF_FLAG_STREAM=1 && run slots CNMF_DEV_SLOTS=1 && run frac50 CNMF_COMPACT_FRAC_SMALL=0.5 && run frac90 CNMF_COMPACT_FRAC_SMALL=0.9 && run base2 A=1 && run flag2 CNMF_FLAG_STREAM=1 && run slots2 CNMF_DEV_SLOTS=1 && run frac50b CNMF_COMPACT_FRAC_SMALL=0.5 && run frac90b CNMF_COMPACT_FRAC_SMALL=0.9
echo rc=$?
