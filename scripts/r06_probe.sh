set -o pipefail
mkdir -p gpurun_out
{
echo "== env"; env | grep -E 'VISIBLE|ROCR|HIP_|GPU_' ;
echo "== kfd nodes"; for d in /sys/class/kfd/kfd/topology/nodes/*; do echo "$d gfx=$(grep gfx_target_version $d/properties) minor=$(grep drm_render_minor $d/properties)"; done;
echo "== dri"; ls -la /dev/dri /dev/kfd;
echo "== render open test"; python3 - <<'PY'
import os, glob
for p in sorted(glob.glob('/dev/dri/renderD*')):
    try:
        fd = os.open(p, os.O_RDWR); os.close(fd); print(p, "open ok")
    except OSError as e:
        print(p, "open fail", e)
PY
echo "== amdsmi"; timeout 60 python3 -c "
import amdsmi
amdsmi.amdsmi_init()
print('amdsmi handles', len(amdsmi.amdsmi_get_processor_handles()))
" ;
echo "== torch count"; timeout 120 python3 -c "import torch; print('torch count', torch.cuda.device_count())";
} > gpurun_out/r06_probe.txt 2>&1
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 > gpurun_out/r06_head_bench.json 2> gpurun_out/r06_head_bench.err
