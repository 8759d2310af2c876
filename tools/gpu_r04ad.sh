#!/bin/bash
# r04ad: config-5 ego / uniform on 12-wave blocks (MG_QWS_WIDE=1: 32-env forwards beside 8 env
# waves, 3 waves per SIMD). Parity first: the Q-net GPU tests with the variant as the product
# library (on the box's scratch copy only), then the in-process A/B against the product.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04ad
mkdir -p $O
L=merging-gym_amd/merging_gym/libmerging_hip.so
cp $L $O/prod_backup.so
echo "== qnet tests (wide)" && cp tools/variants/lib_wide.so $L && timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_qnet.py tests/test_gpu_policy_statistics.py > $O/pytest_wide.log 2>&1 ; rc=$?; cp $O/prod_backup.so $L; rm -f $O/prod_backup.so; tail -2 $O/pytest_wide.log; [ $rc -eq 0 ] \
&& echo "== ab qnet" && MG_AB_FLAGS=1 timeout -k 10 400 python tools/ab_kernels.py tools/variants/lib_prod.so tools/variants/lib_wide.so --qnet --rounds 6 --warm 1200 > $O/ab_qnet.log 2>&1 && tail -3 $O/ab_qnet.log \
&& echo "== ab qnet rev" && MG_AB_FLAGS=1 timeout -k 10 400 python tools/ab_kernels.py tools/variants/lib_wide.so tools/variants/lib_prod.so --qnet --rounds 6 --warm 1200 > $O/ab_qnet_rev.log 2>&1 && tail -3 $O/ab_qnet_rev.log \
&& echo "== all ok"
