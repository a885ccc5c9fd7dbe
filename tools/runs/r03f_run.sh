# interp diagnostics: LDS reads replaced by constants (idiag1), the sum chain split (idiag2)
set -o pipefail
export TMPDIR=/tmp
bash tools/var_ab.sh r03f cfg4 5 2 default idiag1 idiag2 nsl3
