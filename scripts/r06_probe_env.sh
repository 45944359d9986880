# facts about the box for the GPU-count code in bench.py (no HIP call here)
echo "== env"; env | grep -E 'VISIBLE|ROCR|HIP_|GPU_' || true
echo "== kfd nodes"
for d in /sys/class/kfd/kfd/topology/nodes/*; do
    echo "$d gfx=$(grep gfx_target_version $d/properties) minor=$(grep drm_render_minor $d/properties)"
done
echo "== dri"; ls -la /dev/dri /dev/kfd
python3 - <<'PY'
import os, glob
for p in sorted(glob.glob('/dev/dri/renderD*')):
    try:
        fd = os.open(p, os.O_RDWR | os.O_CLOEXEC); os.close(fd); print(p, "open ok")
    except OSError as e:
        print(p, "open fail", e)
PY
echo "== amdsmi"
timeout 60 python3 -c "
import amdsmi
amdsmi.amdsmi_init()
print('amdsmi handles', len(amdsmi.amdsmi_get_processor_handles()))
" || true
echo "== torch count"; timeout 120 python3 -c "import torch; print('torch count', torch.cuda.device_count())" || true
