# Build libmerging_hip.so variants with compile-time knobs for in-process / per-run A/B:
#   bash tools/build_variants.sh name "-DKNOB=0 -DOTHER=1" [name2 "flags2" ...]
# -> tools/variants/lib_<name>.so (same flags as merging_gym/build.py plus the knobs)
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/variants
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -fno-fast-math \
    -Wall $flags -I include -o tools/variants/lib_$name.so merging-gym_amd/csrc/merging_hip.hip &
done
wait
ls -la tools/variants
