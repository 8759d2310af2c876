# Per-kernel VGPR / SGPR / spill / LDS / occupancy of libmerging_hip's device code (hipcc's
# kernel-resource-usage remarks), for a source file (default: the product source).
# Usage: bash tools/resource_usage.sh [file.hip] > out.txt
SRC=${1:-merging-gym_amd/csrc/merging_hip.hip}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math --cuda-device-only -c \
  -I ${INC:-include} -Rpass-analysis=kernel-resource-usage -o /dev/null "$SRC" 2>&1 \
  | grep -E "Function Name|VGPRs:|AGPRs|ScratchSize|Occupancy|LDS Size|SGPRs Spill|VGPRs Spill" \
  | sed -E 's/^.*remark: //'
