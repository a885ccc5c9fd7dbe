# spread occupancy: probes with 4 / 5 ring slots (wrong sums), column heights 12 and 8 (valid)
set -o pipefail
export TMPDIR=/tmp
bash tools/var_ab.sh r03g cfg4 5 2 default nsl5 nsl4 coly12 coly8
