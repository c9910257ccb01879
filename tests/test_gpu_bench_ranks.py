"""bench.py's N-rank path end to end on ONE GPU (--rehearse-one-gpu): `python bench.py --gpus 2` starts
its two ranks itself (no torchrun), each on GPU 0 with its own NCCL_HOSTID so RCCL (the library's
communicator and torch's) runs over its socket transport. What the driver's multi-GPU run executes runs
here: the partition, the library's RCCL communicator, the overlapped halo residual, halo_parity (every
rank's owned rows bitwise against the one-GPU residual), the N-rank implicit step, the max-over-ranks
timing and rank 0's one JSON line. The times mean nothing (one shared GPU, sockets)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("numerics", ["headline", "config5"])
def test_bench_two_ranks_on_one_gpu(numerics):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--rehearse-one-gpu",
                          "--scale", "4", "--steps", "5", "--warmup", "2", "--no-cpu-baseline", "--no-fast",
                          "--preheat-ms", "20", "--launch-timeout", "400", "--numerics", numerics],
                         env=env, capture_output=True, text=True, timeout=450)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    print(json.dumps({k: d[k] for k in ("n_gpus", "value", "ms_per_step", "halo_parity")}),
          json.dumps(d["implicit_step"])[:600])
    assert d["n_gpus"] == 2 and d["config"]["rehearsal_one_gpu"]
    assert d["halo_parity"] is True, d["multi_gpu"]
    assert d["multi_gpu"]["layout_per_rank"][0]["neighbours"] == 1
    im = d["implicit_step"]
    assert "error" not in im and im["ranks"] == 2 and im["steps"] == 3, im
    assert im["first_order_start"]["resratio"] < 1.0


def test_bench_eight_ranks_on_one_gpu():
    """the driver's 8-GPU command shape (`bench.py --gpus 8`, strong scaling of the C4 O-grid) rehearsed with
    8 ranks on GPU 0 at --scale 4 (253,952 cells, 8 graph parts): every rank's owned rows bitwise the 1-GPU
    residual (halo_parity), the 8-rank implicit step (lines cut at rank boundaries, GMRES dots through
    ncclAllReduce) with its linear iterations reported, and the per-phase wall times in the line"""
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--rehearse-one-gpu",
                          "--scale", "4", "--steps", "5", "--warmup", "2", "--no-fast", "--preheat-ms", "20",
                          "--launch-timeout", "400", "--implicit-deadline", "240"],
                         env=env, capture_output=True, text=True, timeout=450)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    print(json.dumps({k: d[k] for k in ("n_gpus", "value", "ms_per_step", "halo_parity", "phases_s")}),
          json.dumps(d["implicit_step"])[:600])
    assert d["n_gpus"] == 8 and d["config"]["rehearsal_one_gpu"]
    assert d["halo_parity"] is True, d["multi_gpu"]
    lay = d["multi_gpu"]["layout_per_rank"]
    assert len(lay) == 8 and all(r["cells"] > 0 and r["neighbours"] >= 1 for r in lay), lay
    assert sum(r["cells"] for r in lay) == d["config"]["cells"]
    im = d["implicit_step"]
    assert "error" not in im and im["ranks"] == 8 and im["steps"] == 3, im
    assert im["lin_iters_per_step"] > 0 and im["first_order_start"]["resratio"] < 1.0, im
    for k in ("launch", "mesh", "partition", "path_staged", "path_primary", "halo_parity", "implicit", "total"):
        assert k in d["phases_s"], d["phases_s"]


@pytest.mark.parametrize("numerics,flux,operator", [("config2", "ROE", "assembled"), ("config3", "HLLC", "matrix-free")])
def test_bench_baseline_configs_one_gpu(numerics, flux, operator):
    """BASELINE configs 2 and 3 through bench.py on one GPU (reduced size): the fused instantiation their
    numerics select is the timed kernel, and config 3's implicit figure runs the matrix-free operator"""
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--numerics", numerics, "--scale", "4",
                          "--steps", "5", "--warmup", "2", "--no-cpu-baseline", "--no-fast", "--preheat-ms", "20"],
                         env=env, capture_output=True, text=True, timeout=400)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    print(json.dumps({k: d[k] for k in ("value", "ms_per_step", "roofline")}))
    assert d["n_gpus"] == 1 and d["value"] > 0
    assert d["roofline"]["kernel"] == "k_residual_wls<%s>" % flux, d["roofline"]
    im = d["implicit_step"]
    assert im["operator"] == operator and im["steps"] == 3, im
