"""GPU tier: bench.py's multi-rank path end to end, as the driver's scaling
run takes it (`python bench.py --gpus N`, no launcher): the parent spawns
the ranks (bench.launch_ranks), every rank compiles the C5 tables, the
digests are all-gathered and compared, each rank classifies its shard of
the seeded global batch with the counter bucket all-reduced per batch, and
rank 0 prints the one JSON line with the slowest rank's time.  On this
one-GPU box the two ranks share cuda:0 (VC_BENCH_SHARED_GPU=1, gloo
collectives: RCCL refuses two ranks on one device), with a small batch so
the run takes seconds; the times are a shared GPU's, not a scaling result.
Runs late in the suite (file name) since it starts child processes."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_without_launcher():
    env = dict(os.environ, VC_BENCH_SHARED_GPU="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--steps", "2", "--warmup", "1", "--packets", "4000000",
                        "--pool", str(1 << 20), "--no-cpu-baseline"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]             # rank 0's line only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2"
    assert d["config"]["global_batch"] == 8_000_000
    assert d["value"] > 0 and d["steps"] == 2
    assert "tables replicated: 2 ranks" in r.stderr


CHILD = r"""
import os, sys
sys.path.insert(0, sys.argv[1])
import bench
n = bench.visible_gpus()
try:
    bench.resolve_world(8, None, device_count=None)
    verdict = "launch"
except SystemExit as e:
    verdict = "exit%s" % e.code
fds = []
for f in os.listdir("/proc/self/fd"):
    try:
        fds.append(os.readlink("/proc/self/fd/" + f))
    except OSError:
        pass
print("VISIBLE", n, verdict, "KFD" if any(x == "/dev/kfd" or x.startswith("/dev/dri") for x in fds)
      else "NOKFD")
"""


def test_gpu_count_takes_no_hip_call():
    """The parent of the driver's N-GPU run (`python bench.py --gpus N`, no
    launcher) counts GPUs from the KFD topology (bench.visible_gpus), never
    through hipGetDeviceCount: after resolve_world(8) on this one-GPU box
    the process has not opened /dev/kfd or a render node, and it refuses
    the run (exit 2) before any work."""
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("VISIBLE")][0]
    assert line == "VISIBLE 1 exit2 NOKFD", (line, r.stderr[-500:])
    assert "--gpus 8 but 1 GPU(s) visible" in r.stderr


def test_bench_refuses_more_gpus_than_visible():
    """bench.py --gpus 2 as the driver runs it (no launcher, no shared-GPU
    rehearsal) on this one-GPU box: exit 2, '1 GPU(s) visible', no JSON
    line and no rank started."""
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT",
              "VC_BENCH_SHARED_GPU"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--steps", "1", "--warmup", "0"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "--gpus 2 but 1 GPU(s) visible" in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]
