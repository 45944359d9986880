#!/bin/bash
# A/B of library builds on one GPU box: scripts/ab_libs.sh "<workloads>" <lib dir>...
# Each build runs every workload twice, interleaved; prints value and ms/step.
# Builds: make -C vproxy_amd/csrc OUT=../../build/<x>/libvclassify.so BUILD=../../build/obj<x> EXTRA=...
set -o pipefail
wls=$1; shift
mkdir -p gpurun_out/ab
for rep in 1 2; do
  for wl in $wls; do
    for d in "$@"; do
      tag=$(basename $d)
      VCLASSIFY_LIB=$d/libvclassify.so timeout -k 10 240 python -u bench.py --workload $wl --steps 20 --warmup 5 \
        --no-cpu-baseline > gpurun_out/ab/$tag.$wl.$rep.json 2> gpurun_out/ab/$tag.$wl.$rep.err || { echo "FAIL $tag $wl"; exit 1; }
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%-8s %-5s rep%s %10.1f %s  %.4f ms' % (sys.argv[2], sys.argv[3], sys.argv[4], d.get('value', d.get('M_items_per_s')), d.get('unit', 'M items/s'), d['ms_per_step']))" gpurun_out/ab/$tag.$wl.$rep.json $tag $wl $rep
    done
  done
done
