# One GPU session on the box: the named steps in order, each under its own time limit, stopping at
# the first failure. Replaces the per-pass gpu_r0*.sh scripts of rounds 2-5.
#
#   gpurun --timeout 1200 -- 'bash tools/gpu_run.sh TAG step [step ...]'
#
# Output under gpurun_out/TAG/. Steps:
#   smoke          __graft_entry__.smoke()
#   pytest         the whole -m gpu suite (one process)
#   pytest:EXPR    the -m gpu tests matching -k EXPR
#   bench_k20      bench.py as the driver runs it at N = 1 (--gpus 1 --steps 20 --warmup 5)
#   bench          bench.py with its defaults
#   prof           rocprofv3 --kernel-trace --stats of a bench run (no CPU legs)
#   pmc            HBM traffic: FETCH_SIZE and WRITE_SIZE, one pass each (tools/profile_pmc.py)
#   valu           the SQ / MFMA / LDS counter passes of tools/pmc_valu.sh
#   rank8_gloo     bench.py --gpus 8 --dist-backend gloo, self-launched (no torchrun), 2^17 envs per rank
#   rank2_nccl     bench.py --gpus 2 on a one-GPU box: must exit non-zero (RCCL needs a GPU per rank)
#   mfma_numerics  tools/mfma_numerics.py collect (the bf16 MFMA rule probe)
#   mfma_struct    tools/mfma_numerics.py struct (structured probes: grouping, alignment, rounding)
#   ab_qnet:A:B    tools/ab_kernels.py --qnet A B  (two library builds, in process)
#   ab_hdqn:A:B    tools/ab_hdqn.py A B
#   clk:LIB        tools/clk_segments.py LIB
#   py:SCRIPT      python SCRIPT (any tools/ probe), 600 s
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1
shift
O=gpurun_out/$TAG
mkdir -p $O
for step in "$@"; do
  echo "== $step"
  case $step in
    smoke) timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 && tail -1 $O/smoke.log ;;
    pytest) timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 && tail -2 $O/pytest_gpu.log ;;
    pytest:*) timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests -k "${step#pytest:}" > $O/pytest_k.log 2>&1 && tail -2 $O/pytest_k.log ;;
    bench_k20) timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_k20.log 2>&1 && tail -1 $O/bench_k20.log | cut -c1-300 ;;
    bench) timeout -k 10 400 python bench.py > $O/bench_default.log 2>&1 && tail -1 $O/bench_default.log | cut -c1-300 ;;
    prof) timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o $TAG -- python bench.py --steps 300 --warmup 20 --no-cpu-baseline > $O/prof.log 2>&1 && tail -1 $O/prof.log | cut -c1-200 ;;
    pmc) timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o pmc -- python tools/profile_pmc.py > $O/pmc_fetch.log 2>&1 \
         && timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o pmc -- python tools/profile_pmc.py > $O/pmc_write.log 2>&1 ;;
    valu) timeout -k 10 900 bash tools/pmc_valu.sh $O/valu > $O/valu.log 2>&1 && tail -2 $O/valu.log ;;
    rank8_gloo) timeout -k 10 600 python bench.py --gpus 8 --steps 100 --warmup 10 --envs 131072 --dist-backend gloo --rollout-launches 20 --qnet-launches 8 --replay-stores 4 --cpu-seconds 3 > $O/bench_8rank.log 2>&1 && tail -1 $O/bench_8rank.log | cut -c1-300 ;;
    rank2_nccl) timeout -k 10 300 python bench.py --gpus 2 --steps 5 --warmup 1 > $O/bench_2rank_nccl.log 2>&1; rc=$?; tail -2 $O/bench_2rank_nccl.log; echo "rc=$rc"; [ $rc -ne 0 ] && [ $rc -ne 124 ] && [ $rc -ne 137 ] ;;
    mfma_numerics) timeout -k 10 300 python tools/mfma_numerics.py collect --cases 2048 --out $O/mfma_numerics.npz > $O/mfma_numerics.log 2>&1 && tail -2 $O/mfma_numerics.log ;;
    mfma_struct) timeout -k 10 300 python tools/mfma_numerics.py struct --out $O/mfma_struct.npz > $O/mfma_struct.log 2>&1 && tail -2 $O/mfma_struct.log ;;
    mfma_single) timeout -k 10 300 python tools/mfma_numerics.py single --cases 1024 --out $O/mfma_single.npz > $O/mfma_single.log 2>&1 && tail -2 $O/mfma_single.log ;;
    ab_qnet:*) IFS=: read -r _ a b <<< "$step"; timeout -k 10 900 python tools/ab_kernels.py --qnet $a $b --rounds 8 > $O/ab_qnet.log 2>&1 && tail -3 $O/ab_qnet.log ;;
    ab_hdqn:*) IFS=: read -r _ a b <<< "$step"; timeout -k 10 900 python tools/ab_hdqn.py $a $b --rounds 6 > $O/ab_hdqn.log 2>&1 && tail -3 $O/ab_hdqn.log ;;
    clk:*) timeout -k 10 300 python tools/clk_segments.py "${step#clk:}" > $O/clk_$(basename ${step#clk:} .so).log 2>&1 && grep -v amdgpu.ids $O/clk_$(basename ${step#clk:} .so).log | tail -3 ;;
    py:*) s=${step#py:}; timeout -k 10 600 python $s > $O/$(basename $s .py).log 2>&1 && tail -3 $O/$(basename $s .py).log ;;
    *) echo "unknown step $step"; false ;;
  esac || { echo "step $step failed"; exit 1; }
done
echo "== all ok"
