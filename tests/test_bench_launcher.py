"""bench.py --gpus N without an outer torchrun: the parent starts
torch.distributed.run as a child before any GPU call and passes rank 0's line and the exit code
through. CPU only: the ranks here run a gloo stand-in script, not the GPU bench."""
import json
import os
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

RANK_SCRIPT = textwrap.dedent("""
    import json, os, sys
    import torch.distributed as dist
    dist.init_process_group("gloo")
    r, P = dist.get_rank(), dist.get_world_size()
    ids = [None] * P
    dist.all_gather_object(ids, os.getpid())
    if r == 0:
        print(json.dumps({"ranks_seen": P, "pids": ids, "argv": sys.argv[1:],
                          "local": os.environ["LOCAL_RANK"]}), flush=True)
    dist.destroy_process_group()
    sys.exit(int(os.environ.get("FAIL_RC", "0")) if r == 1 else 0)
""")


@pytest.fixture()
def rank_script(tmp_path):
    p = tmp_path / "rank.py"
    p.write_text(RANK_SCRIPT)
    return str(p)


def _run_launcher(n, script, env_extra=None):
    code = ("import sys; sys.path.insert(0, %r); import bench; "
            "sys.exit(bench.launch_ranks(%d, ['--gpus', '%d', '--no-e2e'], script=%r))"
            % (ROOT, n, n, script))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                          timeout=180, env=env)


def test_launcher_starts_n_ranks_and_forwards_rank0_line(rank_script):
    r = _run_launcher(2, rank_script)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["ranks_seen"] == 2 and len(set(d["pids"])) == 2
    assert d["argv"] == ["--gpus", "2", "--no-e2e"]


def test_launcher_propagates_a_failing_rank(rank_script):
    r = _run_launcher(2, rank_script, {"FAIL_RC": "3"})
    assert r.returncode != 0


def test_main_self_launches_before_touching_the_gpu(monkeypatch):
    import bench
    import torch

    seen = {}

    def fake_launch(n, argv, script=None, timeout_s=None):
        seen["n"], seen["argv"] = n, list(argv)
        seen["cuda_initialized"] = torch.cuda.is_initialized()
        return 0

    monkeypatch.setattr(bench, "launch_ranks", fake_launch)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "3"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 0
    assert seen == {"n": 4, "argv": ["--gpus", "4", "--steps", "3"], "cuda_initialized": False}
