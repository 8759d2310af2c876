# r04s: HBM traffic (FETCH_SIZE / WRITE_SIZE passes) of the step kernel and, new, the random rollout.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04s
mkdir -p $O
echo "== pmc fetch" && timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o pmc -- python tools/profile_pmc.py > $O/pmc_fetch.log 2>&1 \
&& echo "== pmc write" && timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o pmc -- python tools/profile_pmc.py > $O/pmc_write.log 2>&1 \
&& echo "== all ok"
