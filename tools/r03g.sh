#!/bin/bash
# spread plane prefetch depth 2 (variant spf2): parity subset + cfg4, then cfg5 A/B and cfg5 spread phase clocks
set -o pipefail
tools/lib_variants.sh r03g cfg4 spf2 default || exit 1
STEPS=5 tools/diag_variants.sh r03g5 cfg5 spf2 default || exit 1
tools/stamps_run.sh r03g cfg5 || exit 1
