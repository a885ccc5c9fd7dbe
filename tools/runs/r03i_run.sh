# spread: 5/6-slot split (default) vs split launches with full rings vs one launch; the 5-slot probe
set -o pipefail
export TMPDIR=/tmp
bash tools/var_ab.sh r03i cfg4 5 2 default split6 one6 nsl5
