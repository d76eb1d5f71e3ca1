"""dmlab.launch: the docker-compose replacement (codes/task2/docker-compose.yml,
codes/task4/docker-compose.yml) — env contract, per-rank argument templating,
fail-fast, timeout, compose-like config files."""
import io
import sys
import textwrap
from pathlib import Path

from dmlab import launch

ROOT = Path(__file__).resolve().parent.parent

ALLREDUCE = textwrap.dedent("""
    import os, sys, torch, torch.distributed as dist
    sys.path.insert(0, %r)
    from dmlab.parallel import env
    env.init()
    t = torch.tensor([float(env.get_rank() + 1)])
    dist.all_reduce(t)
    print("rank", env.get_rank(), "of", env.get_world_size(), "local", os.environ["LOCAL_RANK"],
          "sum", int(t.item()), "arg", sys.argv[1])
    env.destroy()
""") % str(ROOT)


def _run(argv, tmp_path, script):
    f = tmp_path / "job.py"
    f.write_text(script)
    out = io.StringIO()
    cmds, envs = launch.build(3, [str(f)] + argv, "127.0.0.1", launch.free_port(), cpu=True)
    job = launch.Job(cmds, envs, out=out)
    job.start()
    return job.wait(120), out.getvalue()


def test_launch_env_contract_and_templating(tmp_path):
    code, out = _run(["r{rank}-of-{world_size}"], tmp_path, ALLREDUCE)
    assert code == 0, out
    for r in range(3):
        assert f"[rank {r}] rank {r} of 3 local {r} sum 6 arg r{r}-of-3" in out


def test_launch_fail_fast(tmp_path):
    script = textwrap.dedent("""
        import os, sys, time
        if os.environ["RANK"] == "1":
            sys.exit(3)
        time.sleep(60)
    """)
    code, out = _run([], tmp_path, script)
    assert code == 3
    assert "rank 1 exited with 3" in out


def test_launch_timeout(tmp_path):
    f = tmp_path / "hang.py"
    f.write_text("import time\ntime.sleep(60)\n")
    cmds, envs = launch.build(2, [str(f)], "127.0.0.1", launch.free_port(), cpu=True)
    out = io.StringIO()
    job = launch.Job(cmds, envs, out=out, grace_s=1)
    job.start()
    assert job.wait(1.0) == 124
    assert all(p.poll() is not None for p in job.procs)


def test_launch_config_order_and_env(tmp_path):
    f = tmp_path / "job.py"
    f.write_text("import os\nprint('svc', os.environ['RANK'], os.environ.get('ROLE'))\n")
    cfg = tmp_path / "c.yaml"
    cfg.write_text(textwrap.dedent(f"""
        services:
          node01: {{command: [{sys.executable}, {f}], env: {{ROLE: driver}}}}
          node02: {{command: [{sys.executable}, {f}], depends_on: [node03]}}
          node03: {{command: [{sys.executable}, {f}]}}
    """))
    cmds, envs, order = launch.from_config(str(cfg), "127.0.0.1", cpu=True)
    assert order == [0, 2, 1]
    assert [e["RANK"] for e in envs] == ["0", "1", "2"]
    out = io.StringIO()
    job = launch.Job(cmds, envs, order, out=out)
    job.start()
    assert job.wait(60) == 0
    assert "svc 0 driver" in out.getvalue() and "svc 2 None" in out.getvalue()


def test_shipped_configs_parse():
    for name in ("task2_dp.yaml", "task4_rpc.yaml"):
        cmds, envs, order = launch.from_config(str(ROOT / "configs" / name), "127.0.0.1", cpu=True)
        assert len(cmds) == len(envs) >= 2
        assert "--rank=1" in cmds[1]
