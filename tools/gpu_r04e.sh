# r04e: GPU tests + bench (tools/gpu_r04.sh), the 2^22 probe, the rollout store twin, then the
# in-process A/B of the round's variants. Each GPU step has its own limit; chained with &&.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=r04e SKIP_PROF=1 bash tools/gpu_r04.sh \
&& echo "== size2 probe" && timeout -k 10 300 python tools/size2_probe.py > gpurun_out/r04e/size2_probe.json \
&& echo "== rollout twin" && timeout -k 10 120 ./tools/micro/rollout_twin > gpurun_out/r04e/rollout_twin.txt && cat gpurun_out/r04e/rollout_twin.txt \
&& TAG=r04e_ab LIBS="tools/variants/lib_base.so tools/variants/lib_r0.so tools/variants/lib_r0lat.so tools/variants/lib_r0latph.so tools/variants/lib_r0latphhb.so tools/variants/lib_rwpe5.so" bash tools/gpu_r04ab.sh
