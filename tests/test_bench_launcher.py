"""bench.py --gpus N without torchrun: the launcher starts N fresh rank
processes itself (no torch in the parent), each joins a world of N, and rank
0's JSON line reaches the parent's stdout.  Runs on CPU over gloo with a stub
worker in place of the GPU bench (the driver's scale runs use the real one)."""
import json
import os
import subprocess
import sys
import textwrap
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]

STUB = textwrap.dedent("""
    import json, os, sys
    import torch
    import torch.distributed as dist
    args = sys.argv[1:]
    n = int(args[args.index("--gpus") + 1])
    assert int(os.environ["WORLD_SIZE"]) == n
    assert os.environ["MASTER_ADDR"] == "127.0.0.1"
    dist.init_process_group("gloo")
    assert dist.get_world_size() == n
    if "--fail-rank" in args and dist.get_rank() == int(args[args.index("--fail-rank") + 1]):
        sys.exit(3)
    t = torch.tensor([float(dist.get_rank() + 1)])
    dist.all_reduce(t)
    if dist.get_rank() == 0:
        print(json.dumps({"n_gpus": dist.get_world_size(), "sum": float(t.item()),
                          "launcher": os.environ.get("CEP_LAUNCHED_BY")}), flush=True)
    dist.barrier()
    dist.destroy_process_group()
""")


def _run_launcher(tmp_path, argv, timeout=240):
    stub = tmp_path / "stub_rank.py"
    stub.write_text(STUB)
    drv = tmp_path / "drive.py"
    drv.write_text(textwrap.dedent("""
        import sys
        sys.path.insert(0, %r)
        assert "torch" not in sys.modules
        import bench
        rc = bench.launch_ranks(int(sys.argv[1]), argv=sys.argv[2:], script=%r)
        assert "torch" not in sys.modules, "the launcher parent must not import torch"
        sys.exit(rc)
    """ % (str(ROOT), str(stub))))
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env["GLOO_SOCKET_IFNAME"] = "lo"
    return subprocess.run([sys.executable, str(drv)] + argv, capture_output=True, text=True,
                          timeout=timeout, env=env)


def test_launcher_world2_prints_rank0_line(tmp_path):
    r = _run_launcher(tmp_path, ["2", "--gpus", "2"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d == {"n_gpus": 2, "sum": 3.0, "launcher": "bench.py"}


def test_launcher_world3(tmp_path):
    r = _run_launcher(tmp_path, ["3", "--gpus", "3"])
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert d["n_gpus"] == 3 and d["sum"] == 6.0


def test_launcher_failing_rank_fails_the_job(tmp_path):
    # rank 1 exits before the collective: rank 0 would block in all_reduce;
    # the launcher must stop it and return non-zero
    r = _run_launcher(tmp_path, ["2", "--gpus", "2", "--fail-rank", "1"])
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])
    assert "rank 1 exited with 3" in r.stderr


def test_bench_refuses_world_mismatch():
    # a torchrun world that disagrees with --gpus is an error, not a silent 1-GPU run
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2"], capture_output=True,
                       text=True, timeout=240, env=env)
    assert r.returncode != 0
    assert "--gpus 2 but WORLD_SIZE=1" in (r.stderr + r.stdout)
