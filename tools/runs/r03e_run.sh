# restructured spread anchor step: A/B against the previous build; cfg5 fused zero+spread
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03e
bash tools/var_ab.sh r03e cfg4 10 2 prev default || exit 1
BENCH_ARGS=--unfused-zero bash tools/var_ab.sh r03e_unf cfg5 10 1 prev default || exit 1
bash tools/var_ab.sh r03e cfg5 10 1 default
