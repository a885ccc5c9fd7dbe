#!/bin/bash
# FETCH/WRITE passes (tools/pmc_traffic.sh) for a library variant: tools/pmc_variant.sh <tag> <variant> [cfg]
set -o pipefail
tag=$1; v=$2; cfg=${3:-cfg4}
if [ "$v" = default ]; then export IBTK_LE_LIB=$PWD/ibamr_amd/lib/libibtk_le.so; else export IBTK_LE_LIB=$PWD/ibamr_amd/lib/var/$v/libibtk_le.so; fi
bash tools/pmc_traffic.sh gpurun_out/$tag/pmc_$v $cfg IB_4 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', {k: round(v/1e9,2) for k,v in d['read_bytes'].items()}, {k: round(v/1e9,2) for k,v in d['write_bytes'].items()})"
