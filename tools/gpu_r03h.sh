# Round-3 GPU session: the 2^22 leg first / last / last with its env allocated before the legs,
# each with the rehearsal window and the collector off. Usage: TAG=r03h bash tools/gpu_r03h.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r03h}
O=gpurun_out/$TAG
mkdir -p $O
for w in first last last_prealloc; do
  extra="--size2-when ${w%%_*}"
  [ "$w" = last_prealloc ] && extra="$extra --size2-prealloc"
  echo "== bench $w" && timeout -k 10 400 python bench.py --no-cpu-baseline $extra > $O/bench_$w.log 2>&1 || { tail -3 $O/bench_$w.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/bench_$w.log').read().strip().splitlines()[-1]); s=d['size_2p22']; print('$w', round(s['kernel_ms']*1e3,1), s['window_us'], s['window_host_enqueue_ms'], s['rehearsal_window_us'])"
done
echo "== all ok"
