# Ablation binaries of the 16x16 forward (tools/micro/qfwd_l1x16.hip, MG_SRC): the shipped source, and
# copies with the permlane16_swap pass removed, the ReLU / bf16 packing reduced to a move, and both.
# Timing only (the Q values are not a forward's). Build here, run on the GPU box:
#   bash tools/micro/qfwd_ablate.sh build && bash tools/micro/qfwd_ablate.sh run OUTDIR
set -e
cd "$(dirname "$0")/../.."
SRC=merging-gym_amd/csrc/merging_hip.hip
if [ "$1" = build ]; then
  mkdir -p tools/micro/ablate
  python3 - "$SRC" <<'PY'
import sys
s = open(sys.argv[1]).read()
swap_old = """  const uint32_t a = x, b = y;
  const uint64_t sw = __builtin_bit_cast(uint64_t, __builtin_amdgcn_permlane16_swap(a, b, false, false));
  x = static_cast<uint32_t>(sw);
  y = static_cast<uint32_t>(sw >> 32);"""
relu_old = """  i16x2 v = __builtin_bit_cast(i16x2, __builtin_convertvector(f32x2{x, y}, bf16x2));
  const i16x2 zero = {0, 0};
  v = __builtin_elementwise_max(v, zero);
  return __builtin_bit_cast(uint32_t, v);"""
assert s.count(swap_old) == 1 and s.count(relu_old) == 1
noswap = s.replace(swap_old, "  (void)x; (void)y;")
norelu = s.replace(relu_old, "  return __builtin_bit_cast(uint32_t, x) ^ (__builtin_bit_cast(uint32_t, y) >> 16);")
both = noswap.replace(relu_old, "  return __builtin_bit_cast(uint32_t, x) ^ (__builtin_bit_cast(uint32_t, y) >> 16);")
for name, t in (("noswap", noswap), ("norelu", norelu), ("noswap_norelu", both)):
    open(f"tools/micro/ablate/{name}.hip", "w").write(t)
PY
  for v in shipped noswap norelu noswap_norelu; do
    if [ $v = shipped ]; then def=""; else def="-DMG_SRC=\"ablate/$v.hip\""; fi
    hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I include -I tools/micro $def \
      -o tools/micro/ablate/qfwd_$v tools/micro/qfwd_l1x16.hip
  done
elif [ "$1" = run ]; then
  O=${2:-gpurun_out/ablate}
  mkdir -p $O
  for v in shipped noswap norelu noswap_norelu; do
    timeout -k 10 120 tools/micro/ablate/qfwd_$v $v >> $O/qfwd_ablate.log 2>&1
  done
fi
