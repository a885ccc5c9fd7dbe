#!/bin/bash
# stream-only diagnostics and spread phase clocks on cfg4
set -o pipefail
tools/diag_variants.sh r03b cfg4 default d_noproc || exit 1
tools/stamps_run.sh r03b cfg4 || exit 1
