# r05zb: round-5 final pass, part 2: HBM traffic (FETCH_SIZE / WRITE_SIZE passes), the 8-rank gloo
# rehearsal of the multi-GPU bench line on the one GPU (2^17 envs per rank), the VALU / MFMA counters
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05zb
mkdir -p $O
echo "== 8-rank rehearsal (gloo, shared GPU)" && timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 8 --steps 100 --warmup 10 --envs 131072 --dist-backend gloo --rollout-launches 20 --qnet-launches 8 --replay-stores 4 --cpu-seconds 3 > $O/bench_8rank.log 2>&1 && tail -1 $O/bench_8rank.log | cut -c1-300 \
&& echo "== pmc fetch" && timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o pmc -- python tools/profile_pmc.py > $O/pmc_fetch.log 2>&1 \
&& echo "== pmc write" && timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o pmc -- python tools/profile_pmc.py > $O/pmc_write.log 2>&1 \
&& echo "== valu" && timeout -k 10 600 bash tools/pmc_valu.sh $O/valu > $O/valu.log 2>&1 && tail -2 $O/valu.log \
&& echo "== all ok"
