# PMC of the KL fp16-numerator beta kernels (bench chunk shape) + sparse kernel
set -e
export TMPDIR=/tmp
bash tools/pmc_bp.sh r3k
echo done
