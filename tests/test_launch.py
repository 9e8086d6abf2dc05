"""The bench scripts' rank launcher (orb_slam3_vio_fixes_amd/launch.py): the
driver's `python bench.py --gpus N` (no torch.distributed.run around it)
must run N ranks, with the parent touching neither torch nor the GPU; under
a launcher WORLD_SIZE must equal --gpus.  SURVEY.md §8(e)."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from orb_slam3_vio_fixes_amd import launch  # noqa: E402


class _Rc:
    def __init__(self, rc):
        self.returncode = rc


def test_launcher_command_shape():
    cmd = launch.launcher_command("bench.py", ["--gpus", "4", "--steps", "3"], 4, 29511)
    assert cmd[0] == sys.executable
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"]
    assert "--nproc-per-node=4" in cmd
    i = cmd.index("--master-addr")
    assert cmd[i + 1] == "127.0.0.1" and cmd[cmd.index("--master-port") + 1] == "29511"
    assert cmd[-5:] == ["bench.py", "--gpus", "4", "--steps", "3"]


def test_ensure_ranks_spawns_without_world_size():
    seen = {}

    def fake_run(cmd, env):
        seen["cmd"], seen["env"] = cmd, env
        return _Rc(5)
    env = {"PATH": os.environ.get("PATH", "")}
    rc = launch.ensure_ranks(2, "bench.py", ["--gpus", "2", "--batch", "8"], env=env, run=fake_run)
    assert rc == 5
    assert "--nproc-per-node=2" in seen["cmd"] and seen["cmd"][-4:] == ["--gpus", "2", "--batch", "8"]
    assert seen["env"]["MASTER_ADDR"] == "127.0.0.1" and "WORLD_SIZE" not in seen["env"]


def test_ensure_ranks_single_and_under_launcher():
    def boom(*a, **k):
        raise AssertionError("must not spawn")
    assert launch.ensure_ranks(1, "bench.py", [], env={}, run=boom) is None
    assert launch.ensure_ranks(2, "bench.py", [], env={"WORLD_SIZE": "2"}, run=boom) is None
    with pytest.raises(ValueError):
        launch.ensure_ranks(2, "bench.py", [], env={"WORLD_SIZE": "4"}, run=boom)
    with pytest.raises(ValueError):
        launch.ensure_ranks(1, "bench.py", [], env={"WORLD_SIZE": "2"}, run=boom)
    with pytest.raises(ValueError):
        launch.ensure_ranks(0, "bench.py", [], env={}, run=boom)


_PARENT_PROBE = r"""
import sys, json
sys.path.insert(0, {root!r})
sys.path.insert(0, {tools!r})
from orb_slam3_vio_fixes_amd import launch
seen = []
class R: returncode = 3
def fake(cmd, env):
    seen.append(cmd)
    return R()
launch.subprocess.run = fake
launch.ensure_ranks.__defaults__ = (None, fake)
import {mod} as m
sys.argv = [{script!r}] + {argv!r}
try:
    m.main()
    code = None
except SystemExit as e:
    code = e.code
print(json.dumps({{"code": code, "cmd": seen[0] if seen else None, "torch": "torch" in sys.modules}}))
"""


@pytest.mark.parametrize("mod,script,argv", [
    ("bench", "bench.py", ["--gpus", "2", "--steps", "2"]),
    ("bench", "bench.py", ["--gpus", "8", "--workload", "c5"]),
    ("bench_c5", "tools/bench_c5.py", ["--gpus", "2", "--nkf", "10"]),
    ("bench_stereo", "tools/bench_stereo.py", ["--gpus", "2", "--workload", "c4"]),
])
def test_bench_parent_launches_ranks_without_torch(mod, script, argv):
    """`--gpus N` with no WORLD_SIZE: the script's main() builds the launcher
    command for ITSELF with the same arguments, exits with the child's code,
    and has not imported torch (so it cannot have touched the GPU)."""
    code = _PARENT_PROBE.format(root=str(ROOT), tools=str(ROOT / "tools"), mod=mod, script=script, argv=argv)
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["code"] == 3 and out["torch"] is False
    n = int(argv[1])
    assert f"--nproc-per-node={n}" in out["cmd"]
    assert Path(out["cmd"][out["cmd"].index("127.0.0.1") + 3]).resolve() == (ROOT / script).resolve()
    assert out["cmd"][-len(argv):] == argv


_RANK_SCRIPT = r"""
import os, sys
sys.path.insert(0, {root!r})
from orb_slam3_vio_fixes_amd import launch
rc = launch.ensure_ranks(int(sys.argv[2]), __file__, sys.argv[1:])
if rc is not None:
    sys.exit(rc)
import torch.distributed as dist
dist.init_process_group("gloo")
open(os.path.join(sys.argv[3], f"rank{{dist.get_rank()}}"), "w").write(os.environ["WORLD_SIZE"])
dist.barrier()
dist.destroy_process_group()
"""


def test_launcher_runs_real_ranks(tmp_path):
    """End to end on the CPU: a script using ensure_ranks, started as one
    plain process with --gpus 2, runs as 2 gloo ranks of torch.distributed.run."""
    s = tmp_path / "launch_probe.py"
    s.write_text(_RANK_SCRIPT.format(root=str(ROOT)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, str(s), "--gpus", "2", str(tmp_path)], env=env, capture_output=True,
                       text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-3000:]
    assert sorted(p.name for p in tmp_path.glob("rank*")) == ["rank0", "rank1"]
    assert (tmp_path / "rank1").read_text() == "2"
