# the GPU suite under the device-checked library with per-launch sync checks
set -o pipefail
mkdir -p gpurun_out
VCLASSIFY_LIB=vproxy_amd/libvclassify_chk.so VC_SYNC_CHECK=1 timeout -k 10 1100 \
    python -u -m pytest tests -x -v -m gpu --timeout 600 --timeout-method thread \
    --deselect tests/test_gpu_pin_loop.py::test_batches_never_wait_for_a_recompile \
    > gpurun_out/r06_gpu_tests_chk.log 2>&1 || { echo CHK FAILED; tail -30 gpurun_out/r06_gpu_tests_chk.log; exit 1; }
tail -2 gpurun_out/r06_gpu_tests_chk.log
