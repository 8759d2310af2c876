# r05zn: smoke and the whole GPU suite on the final tree (kernel as r05zg; tests and checkpoint loader since)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05zn
mkdir -p $O
echo "== smoke" && timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 && tail -1 $O/smoke.log \
&& echo "== pytest gpu" && timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 && tail -2 $O/pytest_gpu.log \
&& echo "== all ok"
