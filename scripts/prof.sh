#!/bin/bash
# Profile passes of bench.py workloads on the GPU box (one gpu_steps.sh step
# per pass, so a failing pass stops the call):
#
#   bash scripts/prof.sh TAG "name|bench args" ...     e.g.
#   bash scripts/prof.sh r05 "c5|" "mix15|--workload mix --compact6"
#   PASSES="trace l2" bash scripts/prof.sh r05 "c4|--workload c4"
#   bash scripts/prof.sh r05 cal                       (tools/gather_probe cal)
#
# Passes (PASSES, default "trace fetch write l2"), each its own rocprofv3 run
# as MI355X_MICROARCH.md asks (no tracing beside counters, one block's
# counter budget per run):
#   trace  --kernel-trace --stats                  -> gpurun_out/TAG/<name>_trace
#   fetch  --pmc FETCH_SIZE                        -> .../<name>_fetch
#   write  --pmc WRITE_SIZE                        -> .../<name>_write
#   l2     --pmc TCC_HIT_sum TCC_MISS_sum          -> .../<name>_l2
#   sq     --pmc $SQ (issue counters + GRBM_GUI_ACTIVE) -> .../<name>_sq
# Summaries on this side: scripts/pmc_traffic.py, scripts/fetch_calibration.py,
# scripts/sq_summary.py, scripts/timed_window.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
export VC_BENCH_NO_E2E=1
tag=$1; shift
O=gpurun_out/$tag
SQ=${SQ:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"}
steps=()
for spec in "$@"; do
  if [ "$spec" = cal ]; then
    w=cal; C="tools/gather_probe cal"
  else
    w=${spec%%|*}; args=${spec#*|}
    C="python3 bench.py $args --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline"
  fi
  for p in ${PASSES:-trace fetch write l2}; do
    case $p in
      trace) steps+=("${tag}_${w}_trace:300:rocprofv3 --kernel-trace --stats --output-format csv -d $O/${w}_trace -o run -- $C") ;;
      fetch) steps+=("${tag}_${w}_fetch:300:timeout -s KILL 280 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${w}_fetch -o run -- $C") ;;
      write) steps+=("${tag}_${w}_write:300:timeout -s KILL 280 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${w}_write -o run -- $C") ;;
      l2)    steps+=("${tag}_${w}_l2:300:timeout -s KILL 280 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/${w}_l2 -o run -- $C") ;;
      sq)    steps+=("${tag}_${w}_sq:300:timeout -s KILL 280 rocprofv3 --pmc $SQ --output-format csv -d $O/${w}_sq -o run -- $C") ;;
      *) echo "unknown pass $p"; exit 2 ;;
    esac
  done
done
bash scripts/gpu_steps.sh "${steps[@]}"
