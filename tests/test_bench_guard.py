"""bench.py's guarded implicit section on N ranks (CPU, gloo, world size 2): the ranks agree on an error
raised on one of them, and a rank stuck in a collective (its peer failed before joining) cannot lose the
measurement -- at the deadline rank 0 prints the line with the error and every process exits with
bench.GUARD_EXIT (not 0: the run did not finish)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = r"""
import json, os, sys, time
sys.path.insert(0, %(root)r)
import torch, torch.distributed as dist
import bench
mode = sys.argv[1]
dist.init_process_group("gloo", init_method="env://")
rank = dist.get_rank()
ctrl = dist.new_group(backend="gloo")

def section():
    if mode == "ok":
        return {"ranks": 2, "rank": rank}
    if mode == "raise":
        if rank == 1:
            raise RuntimeError("boom")
        return {"ranks": 2}
    # "hang": rank 1 fails before a collective that rank 0 enters (as a GMRES dot product would)
    if rank == 1:
        raise RuntimeError("left before the collective")
    t = torch.zeros(1)
    dist.all_reduce(t)
    return {"never": True}

res = bench.guarded_implicit(section, 6.0, dist, ctrl, rank,
                             lambda im: print(json.dumps({"deadline": im}), flush=True) if rank == 0 else None)
if rank == 0:
    print(json.dumps({"result": res}), flush=True)
dist.destroy_process_group()
"""


def _run(mode, tmp_path):
    script = tmp_path / "w.py"
    script.write_text(WORKER % {"root": ROOT})
    port = __import__("bench").free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, str(script), mode], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True, cwd=ROOT))
    outs = [p.communicate(timeout=120) for p in procs]
    return [p.returncode for p in procs], outs


@pytest.mark.parametrize("mode", ["ok", "raise", "hang"])
def test_guarded_implicit(mode, tmp_path):
    sys.path.insert(0, ROOT)
    import bench
    codes, outs = _run(mode, tmp_path)
    want = bench.GUARD_EXIT if mode == "hang" else 0
    assert codes == [want, want], (codes, [o[1][-1500:] for o in outs])
    lines = [json.loads(l) for l in outs[0][0].splitlines() if l.startswith("{")]
    assert len(lines) == 1, outs[0]
    d = lines[0]
    if mode == "ok":
        assert d["result"] == {"ranks": 2, "rank": 0}
    elif mode == "raise":
        assert "rank 1 failed" in d["result"]["error"], d
    else:
        assert "within 6 s" in d["deadline"]["error"], d
