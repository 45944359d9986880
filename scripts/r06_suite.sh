# the whole GPU suite + smoke, as the driver runs them at round end
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r06}
timeout -k 10 1500 python -u -m pytest tests -x -v -m gpu --timeout 600 --timeout-method thread \
    > gpurun_out/${tag}_gpu_tests.log 2>&1 || { echo SUITE FAILED; tail -40 gpurun_out/${tag}_gpu_tests.log; exit 1; }
tail -3 gpurun_out/${tag}_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" \
    > gpurun_out/${tag}_smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 gpurun_out/${tag}_smoke.log; exit 1; }
