# rocPRIM onesweep block / items-per-thread variants of the bin's sort (cfg4 bin time)
set -o pipefail
export TMPDIR=/tmp
bash tools/var_ab.sh r03u cfg4 5 2 default s512x16 s1024x12 s256x16
