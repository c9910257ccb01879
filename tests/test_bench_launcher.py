"""bench.py --gpus N without torchrun starts its own N ranks; no GPU needed:
the launch plan, the refusal of a WORLD_SIZE that disagrees with --gpus, and the process supervision
(all children succeed / one fails / the watchdog fires) with stand-in child commands."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _env_without_dist():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "LOCAL_WORLD_SIZE"):
        env.pop(k, None)
    return env


def test_dry_run_lists_n_ranks():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--steps", "7",
                          "--launch-dry-run"], env=_env_without_dist(), capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    plan = json.loads(out.stdout.strip().splitlines()[-1])
    ranks = plan["ranks"]
    assert len(ranks) == 4 and not plan["in_process"]
    ports = {r["env"]["MASTER_PORT"] for r in ranks}
    assert len(ports) == 1
    for i, r in enumerate(ranks):
        e = r["env"]
        assert (e["RANK"], e["LOCAL_RANK"], e["WORLD_SIZE"], e["MASTER_ADDR"]) == (str(i), str(i), "4", "127.0.0.1")
        assert r["cmd"][1:2] == ["-u"] and r["cmd"][2].endswith("bench.py")
        assert r["cmd"][3:] == ["--gpus", "4", "--steps", "7"]


def test_dry_run_rehearsal_sets_host_ids():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3", "--rehearse-one-gpu",
                          "--launch-dry-run"], env=_env_without_dist(), capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    ranks = json.loads(out.stdout.strip().splitlines()[-1])["ranks"]
    assert [r["env"]["NCCL_HOSTID"] for r in ranks] == ["fvhip-rehearsal-%d" % i for i in range(3)]
    assert all(r["env"]["NCCL_SOCKET_IFNAME"] == "lo" for r in ranks)
    plain = bench.rank_launch_plan(3, [], port=29500)
    assert all("NCCL_HOSTID" not in e for _, e in plain)


def test_dry_run_one_gpu_runs_in_process():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--launch-dry-run"],
                         env=_env_without_dist(), capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    plan = json.loads(out.stdout.strip().splitlines()[-1])
    assert plan["ranks"] == [] and plan["in_process"]


def test_world_size_mismatch_refused():
    env = dict(_env_without_dist(), WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--launch-dry-run"],
                         env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode != 0
    assert "differs from --gpus" in out.stderr


def test_under_torchrun_no_second_launch():
    env = dict(_env_without_dist(), WORLD_SIZE="4", RANK="1", LOCAL_RANK="1")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--launch-dry-run"],
                         env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    plan = json.loads(out.stdout.strip().splitlines()[-1])
    assert plan["ranks"] == [] and plan["under_launcher"] and plan["world_size"] == 4


def _plan(code):
    cmd = [sys.executable, "-c", code]
    return [(cmd, e) for _, e in bench.rank_launch_plan(3, [], port=29999)]


def test_run_ranks_all_succeed(tmp_path):
    code = ("import os; open(os.path.join(%r, 'r' + os.environ['RANK']), 'w').write("
            "os.environ['WORLD_SIZE'] + ' ' + os.environ['MASTER_ADDR'])" % str(tmp_path))
    assert bench.run_ranks(_plan(code), timeout_s=60) == 0
    assert sorted(os.listdir(tmp_path)) == ["r0", "r1", "r2"]
    assert open(tmp_path / "r2").read() == "3 127.0.0.1"


def test_run_ranks_one_fails_others_killed():
    code = "import os, sys, time; r = int(os.environ['RANK']); sys.exit(3) if r == 1 else time.sleep(60)"
    t0 = time.time()
    assert bench.run_ranks(_plan(code), timeout_s=120) == 3
    assert time.time() - t0 < 30


def test_run_ranks_watchdog():
    code = "import time; time.sleep(60)"
    t0 = time.time()
    assert bench.run_ranks(_plan(code), timeout_s=2) == 124
    assert time.time() - t0 < 30
