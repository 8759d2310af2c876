#!/bin/bash
# r04ag: the VALU-side counter passes (tools/pmc_valu.sh) on the final round-4 library
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04ag
mkdir -p $O
echo "== pmc valu" && timeout -k 10 1000 bash tools/pmc_valu.sh $O/pmcv > $O/pmc_valu.log 2>&1 && tail -2 $O/pmc_valu.log && echo "== all ok"
