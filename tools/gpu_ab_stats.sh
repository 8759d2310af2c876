# Step kernel with statistics at 2^22 and 2^20 envs (tools/stats_cost_probe.py) for each library
# given, interleaved over ROUNDS rounds. Usage: ROUNDS=2 bash tools/gpu_ab_stats.sh tools/variants/lib_a.so ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
ROUNDS=${ROUNDS:-2}
for r in $(seq 1 "$ROUNDS"); do
  for lib in "$@"; do
    export MERGING_HIP_LIB=$PWD/$lib
    for n in 4194304 1048576; do
      out=$(timeout -k 10 200 python tools/stats_cost_probe.py $n) || { echo "$lib failed"; exit 1; }
      echo "$(basename $lib .so) r$r n=$n $(echo "$out" | python -c 'import json,sys; d=json.load(sys.stdin); print(d["median"])')"
    done
  done
done
