"""CPU tier: bench.py's rank launcher (`python bench.py --gpus N` run without
torch.distributed.run spawns the N ranks itself) and its argument checks.

The launcher is exercised with a stand-in rank script (tests/native/ is not
needed: the script is written to tmp_path), so no GPU is touched.
"""
import json
import os
import subprocess
import sys
import time

import pytest

import bench as B

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

RANK_SCRIPT = r"""
import json, os, sys, time
out = sys.argv[1]
mode = sys.argv[2]
r = int(os.environ["RANK"])
with open(os.path.join(out, "rank%d.json" % r), "w") as f:
    json.dump({k: os.environ.get(k) for k in
               ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}, f)
if mode == "ok":
    if r == 0:
        print(json.dumps({"n_gpus": int(os.environ["WORLD_SIZE"])}), flush=True)
    sys.exit(0)
if mode == "fail1":
    if r == 1:
        sys.exit(3)
    time.sleep(120)          # a rank stuck in a collective for its dead peer
if mode == "kill1":
    if r == 1:
        os.kill(os.getpid(), 9)
    time.sleep(120)
"""


@pytest.fixture
def rank_script(tmp_path):
    p = tmp_path / "rank.py"
    p.write_text(RANK_SCRIPT)
    return str(p)


def test_launch_sets_rank_env(tmp_path, rank_script, capfd):
    rc = B.launch_ranks(4, [str(tmp_path), "ok"], script=rank_script,
                        env=dict(os.environ, MASTER_PORT="29999"))
    assert rc == 0
    envs = [json.loads((tmp_path / ("rank%d.json" % r)).read_text()) for r in range(4)]
    assert [e["RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert {e["WORLD_SIZE"] for e in envs} == {"4"}
    assert {e["MASTER_ADDR"] for e in envs} == {"127.0.0.1"}
    assert {e["MASTER_PORT"] for e in envs} == {"29999"}
    # exactly one JSON line (rank 0's) on the job's stdout
    lines = [l for l in capfd.readouterr().out.splitlines() if l.startswith("{")]
    assert lines == ['{"n_gpus": 4}']


def test_launch_picks_a_port(tmp_path, rank_script):
    env = {k: v for k, v in os.environ.items() if k not in ("MASTER_PORT", "MASTER_ADDR")}
    assert B.launch_ranks(2, [str(tmp_path), "ok"], script=rank_script, env=env) == 0
    ports = {json.loads((tmp_path / ("rank%d.json" % r)).read_text())["MASTER_PORT"]
             for r in range(2)}
    assert len(ports) == 1 and int(ports.pop()) > 0


def test_launch_failure_stops_the_job(tmp_path, rank_script):
    t0 = time.time()
    rc = B.launch_ranks(3, [str(tmp_path), "fail1"], script=rank_script, grace_s=5)
    assert rc == 3
    assert time.time() - t0 < 60          # the sleeping ranks were terminated


def test_launch_signal_status(tmp_path, rank_script):
    rc = B.launch_ranks(2, [str(tmp_path), "kill1"], script=rank_script, grace_s=5)
    assert rc == 128 + 9


def test_resolve_world():
    R = B.resolve_world
    assert R(1, {}) == ("run", 1)
    assert R(8, {"WORLD_SIZE": "8"}) == ("run", 8)
    assert R(8, {}, device_count=8) == ("launch", 8)
    assert R(2, {}, shared=True, device_count=1) == ("launch", 2)
    with pytest.raises(SystemExit) as e:
        R(8, {"WORLD_SIZE": "1"})
    assert e.value.code == 2
    with pytest.raises(SystemExit) as e:
        R(1, {"WORLD_SIZE": "2"})
    assert e.value.code == 2
    with pytest.raises(SystemExit) as e:
        R(4, {}, device_count=1)
    assert e.value.code == 2
    with pytest.raises(SystemExit):
        R(0, {})


@pytest.mark.parametrize("env_ws,gpus", [("2", 4), (None, 2)])
def test_bench_refuses_mismatch(env_ws, gpus):
    """bench.py itself: WORLD_SIZE disagreeing with --gpus, or --gpus above
    the visible GPUs (none in this container), exits 2 before any work."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    if env_ws:
        env["WORLD_SIZE"] = env_ws
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus),
                        "--steps", "1", "--warmup", "0"], env=env, capture_output=True,
                       text=True, timeout=300)
    assert p.returncode == 2, p.stderr[-2000:]
    assert "--gpus %d" % gpus in p.stderr
    assert not [l for l in p.stdout.splitlines() if l.startswith("{")]


def _node(root, i, gfx, minor=None, readable=True):
    d = root / "nodes" / str(i)
    d.mkdir(parents=True)
    if readable:
        (d / "properties").write_text("cpu_cores_count 0\ngfx_target_version %d\n%s" % (
            gfx, "" if minor is None else "drm_render_minor %d\n" % minor))


def test_visible_gpus_from_kfd_topology(tmp_path):
    """bench.visible_gpus counts GPUs with no HIP call: KFD nodes with a
    gfx target whose render node exists (the GPU box hides the other nodes'
    properties and render nodes), then the *_VISIBLE_DEVICES lists."""
    _node(tmp_path, 0, 0)                       # CPU
    _node(tmp_path, 1, 90500, 128)
    _node(tmp_path, 2, 90500, 136)
    _node(tmp_path, 3, 90500, 144)              # render node not in this container
    _node(tmp_path, 4, 90500, readable=False)   # properties not readable
    dri = tmp_path / "dri"
    dri.mkdir()
    for m in (128, 136):
        (dri / ("renderD%d" % m)).write_text("")
    V = lambda env: B.visible_gpus(env, str(tmp_path / "nodes"), str(dri))
    assert V({}) == 2
    assert V({"HIP_VISIBLE_DEVICES": "0"}) == 1
    assert V({"ROCR_VISIBLE_DEVICES": "1", "HIP_VISIBLE_DEVICES": "0"}) == 1
    assert V({"CUDA_VISIBLE_DEVICES": "0,1,2"}) == 2          # 2 names no device: cut there
    assert V({"HIP_VISIBLE_DEVICES": "-1,0"}) == 0
    assert V({"HIP_VISIBLE_DEVICES": ""}) == 0
    assert V({"ROCR_VISIBLE_DEVICES": "GPU-abc,GPU-def"}) == 2
    assert B.visible_gpus({}, str(tmp_path / "absent"), str(dri)) == 0
    with pytest.raises(SystemExit) as e:
        B.resolve_world(2, {"HIP_VISIBLE_DEVICES": "0"}, device_count=V({"HIP_VISIBLE_DEVICES": "0"}))
    assert e.value.code == 2
