# HBM traffic of the sweeps on this build (FETCH_SIZE / WRITE_SIZE passes) and cfg5 kernel stats
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03k; mkdir -p $out
bash tools/pmc_traffic.sh $out/pmc cfg4 IB_4 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_cfg5 -o run -- python3 bench.py --config cfg5 --steps 5 --warmup 1 --no-cpu-baseline > $out/prof_cfg5.log 2>&1 || exit 1
echo done
