#!/usr/bin/env python3
"""Benchmark: FVENS second-order residual sweep (FlowFV::compute_residual with local time steps)
on MI355X, Mfaces/s and achieved HBM GB/s of the dominant kernel.

Workload (BASELINE.json north_star target): the C4 mesh of SURVEY.md 8(d) — NACA0012 hybrid O-grid,
Ntheta = 2048, 256 quad + 864 triangle-split layers = 4,063,232 cells, 6,359,040 faces — with
Roe flux + weighted-least-squares gradients + MUSCL/Van Albada reconstruction, M 0.8, 1.25 deg.
One step = one full residual evaluation (primitive conversion, BC ghosts, WLS gradients, fused
reconstruction/flux/scatter/time-step sweep) with the state resident in HBM.
Multi-GPU (torchrun, one process per GPU): the mesh is partitioned (--partitioner graph: recursive
graph bisection of the cell dual graph, the stand-in for the reference's Scotch; or rcb), each rank holds
its cells plus a two-layer halo: ONE exchange of u per residual (both layers, RCCL ncclSend/ncclRecv
over xGMI with the library's own communicator) after which each rank computes its layer-1 ghosts'
gradients itself, overlapped with the patches that need no halo data.
--scaling strong (default): the C4 mesh itself is split N ways (BASELINE.json config 4); afterwards every
rank's owned residual is compared bit for bit with a 1-GPU residual of the whole mesh (halo_parity);
--scaling weak: the O-grid has N x 2048 cells around, so every GPU owns a C4-size part.
Launch: under torchrun (WORLD_SIZE set, it must equal --gpus), or `python bench.py --gpus N` alone, which
starts the N ranks itself (one child process per GPU, env:// rendezvous on 127.0.0.1, a wall-clock
watchdog, exit status of the first failing rank) before anything touches a GPU; --launch-dry-run prints
the plan.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

T_PROCESS = time.time()       # wall-clock phases of the run are reported from here (out["phases_s"])
ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)

# start of the implicit-step figure: first-order steps (expResidualRamp over init_cfl), then the timed
# second-order steps at a fixed CFL
# the implicit figure: a first-order start of 5 steps (timed), then 3 second-order steps timed from the free
# stream (a cold start, where the residual falls: profiles/r04/implicit_freestream.jsonl) and the same 3
# continuing from the start's state (where this O-grid's start-up transient makes it rise), CFL 25
IMPLICIT_START = dict(init_steps=5, cfl=25.0, init_cfl=None, second_from="freestream")


C4_WALL_SPACING = 1e-5
# far-field angles uniform in the surface parameter (generateNacaOgrid farmap 1): with the mid-chord
# direction map (0) the cosine-clustered trailing-edge points crowd the far field at angle 0, leaving
# sliver triangles (aspect ratio ~1e3) along the wake line where second-order solves blow up
C4_FARMAP = 1
# the viscous C5 family (config 5): the hybrid mesh of the visc-naca0012 grids' topology
# (testcases/visc-naca0012/grids/naca0012nasa-blcirc.geo, NACA0012_lam_hybrid_1.msh: quadrangles through the
# boundary layer, triangles outside it), built on the quadrangle C-grid's points (generateNacaHybrid): 3072
# columns round the body and 384 along each wake, 2048 rows from a 1e-5 wall spacing; quadrangles in the body's
# first 768 rows and in the wake blocks, near-isotropic triangles (each row resampled to its row distance)
# above the body's boundary layer: 8,054,644 cells (3,932,160 quadrangles, 4,122,484 triangles), 14,052,330
# faces. Round 5's quadrangle C-grid (generateNacaCgrid, ntri 0) stays available as topology "cgrid".
C5_DIMS = dict(nsurf=3072, nwake=384, nquad=768, nrows=2048)


def c4_mesh(fa, scale, mult=1, wall=None, farmap=None, topology="hybrid"):
    """C4 (mult 1): the O-grid; C5 (mult 2): the hybrid mesh of the visc-naca0012 grids' topology (or, with
    topology "cgrid", round 5's quadrangle C-grid: 4096 columns, 3072 round the body, 512 along each wake),
    unless an O-grid `farmap` is asked for"""
    nt = 2048 * mult // scale
    nq = 256 // scale
    ntri = 864 // scale
    ws = C4_WALL_SPACING if wall is None else wall
    if mult == 2 and farmap is None and topology == "hybrid":
        d = {k: v // scale for k, v in C5_DIMS.items()}
        return (fa.UMesh.naca_hybrid(d["nsurf"], d["nwake"], d["nquad"], d["nrows"], 20.0, ws),
                dict(topology="hybrid", **d, wall_spacing=ws))
    if mult == 2 and farmap is None:
        ns, nw, rows = 3 * nt // 4, nt // 8, nq + 2 * ntri
        return (fa.UMesh.naca_cgrid(ns, nw, rows, 0, 20.0, ws),
                dict(topology="cgrid", nsurf=ns, nwake=nw, rows=rows, wall_spacing=ws))
    fm = C4_FARMAP if farmap is None else farmap
    return (fa.UMesh.naca_ogrid(nt, nq, ntri, 20.0, ws, farmap=fm),
            dict(ntheta=nt, nquad=nq, ntri=ntri, wall_spacing=ws, farmap=fm))


def sweep_algorithmic_bytes(N, F, Fb):
    """32 B/face (L,R 8 + nx,ny,len 24) + 144 B/cell (prim 32 + grad 64 + centre 16
    + residual write 32) + 48 B/boundary face (ghost centre 16 + ghost state 32) + 8 B/cell for the
    time-step accumulation ("Time-step accumulation adds 8 B/cell")"""
    return 32 * F + 144 * N + 48 * Fb + 8 * N


def sweep_bytes_area_dt(N, F, Fb):
    """variant basis: the time step counted as area read 8 + dtm write 8 = 16 B/cell"""
    return sweep_algorithmic_bytes(N, F, Fb) + 8 * N


def residual_algorithmic_bytes(N, F, Fb):
    """Compulsory bytes of the one-launch residual k_residual_wls (gradients and WLS inverses computed
    in LDS / registers, never stored): 32 B/face (L,R 8 + nx,ny,len 24) + 96 B/cell (conserved state
    32 + centre 16 + area 8 read; residual 32 + time step 8 written) + 16 B/boundary face (ghost
    centre; the ghost state is computed in registers). Index data (packed 16-bit neighbour, slot and
    face codes) and the ring-1/ring-2 re-reads come on top and show in the PMC traffic."""
    return 32 * F + 96 * N + 16 * Fb


def prep_algorithmic_bytes(N, F, Fb):
    """k_prep_grad_wls: conserved state 32 + centre 16 + WLS inverse 32 + neighbour list 16 read,
    primitive state 32 + gradient 64 written per cell; boundary ghost states (conserved + primitive
    64) written and ghost centre 16 + normal 16 read per boundary face"""
    return (32 + 16 + 32 + 16 + 32 + 64) * N + 96 * Fb


def config4_algorithmic_bytes(N, F, Fb):
    """SURVEY.md 8(d), Roe + linear/Venkatakrishnan: the face centres are read too (48 B/face instead of
    32); + 8 B/cell time step. The limiter pass's own bytes (clength, phi), which the fused kernel never
    moves, are not counted (a lower figure than SURVEY's '+ limiter pass')"""
    return 48 * F + 144 * N + 48 * Fb + 8 * N


def kernel_bytes(label, N, F, Fb, numerics="headline"):
    """algorithmic bytes of one launch of the residual kernel `label` (profiling name): SURVEY.md 8(d)'s
    per-face figure for the second-order sweep (124.0 B/face on C4) plus the time-step bytes, the same
    for the one-launch residual and for the staged sweep -- they perform the same operation; the
    one-launch kernel's own compulsory traffic is lower (residual_algorithmic_bytes: gradients stay
    in LDS), which is why it is faster, not a different amount of algorithmic work"""
    if numerics in ("config3", "config4", "config5"):
        return config4_algorithmic_bytes(N, F, Fb)
    return sweep_algorithmic_bytes(N, F, Fb)


def kernel_symbol(label, numerics="headline"):
    """profiling label -> rocprofv3 kernel symbol suffix of the Roe/MUSCL/dt (headline, config2), HLLC/linear/
    Sutherland/dt (config3), Roe/linear/Venkatakrishnan/dt (config4) or Roe/linear/Sutherland/dt (config5: the
    visc-naca0012 deck's `limiter none`)
    instantiation (template arguments: include/fvhip.h's flux codes, kernels.hpp's SweepRec / SweepVisc)"""
    if label.startswith("k_residual_wls"):
        return {"headline": "k_residual_wls<4, 1, true, 0, 0>", "config2": "k_residual_wls<4, 1, true, 0, 0>",
                "config3": "k_residual_wls<6, 2, true, 1, 0>", "config4": "k_residual_wls<4, 2, true, 0, 2>",
                "config5": "k_residual_wls<4, 2, true, 1, 0>"}[numerics]
    return {"headline": "k_sweep<4, 1, 0, true, false>", "config2": "k_sweep<4, 1, 0, true, false>",
            "config3": "k_sweep<6, 2, 1, true, false>", "config4": "k_sweep<4, 2, 0, true, true>",
            "config5": "k_sweep<4, 2, 1, true, false>"}[numerics]


def pmc_traffic(kernel_symbol, workload_cells):
    """HBM bytes per launch of `kernel_symbol` from the newest committed rocprofv3 PMC summary
    (profiles/r*/pmc_traffic.json; pmc_schemes.json / pmc_config3.json / pmc_config5.json for the limited and viscous
    instantiations: FETCH_SIZE x2 + WRITE_SIZE, calibrated as MI355X_MICROARCH.md prescribes), if it was
    measured on the same workload; else None."""
    import glob
    best = None
    files = [f for r in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*")))
             for f in (os.path.join(r, n) for n in ("pmc_schemes.json", "pmc_config3.json", "pmc_config5.json",
                                                            "pmc_traffic.json"))
             if os.path.exists(f)]
    for f in files:
        try:
            d = json.load(open(f))
        except Exception:
            continue
        if str(workload_cells) not in d.get("workload", "").replace(",", ""):
            continue
        for k, v in d.get("kernels", {}).items():
            if k.endswith(kernel_symbol) and "hbm_bytes_corrected" in v:
                best = (v["hbm_bytes_corrected"], os.path.relpath(f, ROOT), v.get("SQ_INSTS_VALU"), v)
    return best


NUM_SIMDS = 256 * 4


def counter_bound(counters, kernel_ms):
    """which resource bounds the kernel, from its committed PMC counters: the fraction of time the
    vector ALUs issue (SQ_ACTIVE_INST_VALU quad-cycles x 4 over 1,024 SIMDs x the kernel's cycles,
    GRBM_GUI_ACTIVE / 8 XCDs) against the HBM fraction (PMC bytes / kernel time / 8 TB/s)"""
    if not counters or not counters.get("SQ_ACTIVE_INST_VALU") or not counters.get("GRBM_GUI_ACTIVE"):
        return None
    cycles = counters["GRBM_GUI_ACTIVE"] / 8.0
    valu = counters["SQ_ACTIVE_INST_VALU"] * 4.0 / (NUM_SIMDS * cycles)
    hbm = counters["hbm_bytes_corrected"] / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS
    return {"bound": "valu" if valu > hbm else "hbm", "valu_busy": round(valu, 3), "hbm_busy": round(hbm, 3)}


HBM_MEASURED_GBS = 6290.0          # MI355X_MICROARCH.md: float4 copy, 79 % of the spec
SCLK_MEASURED_HZ = 2.19e9         # the shader clock the chip holds under the residual kernels (DESIGN.md section 5:
                                   # s_memtime cycles over s_memrealtime, round 4), not the 2.4 GHz boost
FP64_LANE_OPS = 256 * 64 * SCLK_MEASURED_HZ   # FP64 VALU issue: 64 lanes/CU/clock (78.6 TFLOPS FMA spec at 2.4 GHz)


def valu_roofline(valu_wave_instrs, kernel_ms):
    """the face kernels are FP64-issue bound: VALU wave-instructions per launch (PMC SQ_INSTS_VALU of
    the committed profile) x 64 lanes / launch time, against the FP64 issue rate (every VALU
    instruction counted at the FP64 rate, so the fraction is a lower bound)"""
    if not valu_wave_instrs:
        return None
    a = valu_wave_instrs * 64 / (kernel_ms * 1e-3)
    return {"bound": "fp64-valu", "achieved": round(a / 1e12, 2), "peak": round(FP64_LANE_OPS / 1e12, 2),
            "unit": "T lane-ops/s", "frac": round(a / FP64_LANE_OPS, 4), "valu_wave_instrs": int(valu_wave_instrs)}


def host_cpu_info():
    """the cores this job may use: affinity CPUs / threads per core, capped by the cgroup CPU quota;
    lscpu model name (all physical cores, OMP_PROC_BIND=close OMP_PLACES=cores)"""
    import subprocess
    info = {}
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=20).stdout
        for line in out.splitlines():
            k, _, v = line.partition(":")
            info[k.strip()] = v.strip()
    except Exception:
        pass
    aff = len(os.sched_getaffinity(0))
    tpc = int(info.get("Thread(s) per core", "1") or 1)
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = int(q) // int(per)
    except Exception:
        pass
    cores = max(1, aff // max(tpc, 1))
    if quota:
        cores = min(cores, quota)
    return {"model": info.get("Model name"), "sockets": info.get("Socket(s)"),
            "cores_per_socket": info.get("Core(s) per socket"), "threads_per_core": tpc,
            "affinity_cpus": aff, "cgroup_cpu_quota": quota, "physical_cores_used": cores}


def cpu_baseline(mesh, u, nrep, rec="VANALBADA", kind="naca", flux="ROE"):
    """BASELINE.md's CPU baseline: the oracle's OpenMP restatement (the reference's omp parallel for /
    omp atomic structure) on this host's physical cores, in a child process so that OMP_PROC_BIND /
    OMP_PLACES take effect (torch has already loaded the OpenMP runtime here); median of `nrep` sweeps
    after 3 warm-ups on all cores, and on 1 thread"""
    import subprocess
    import tempfile
    hw = host_cpu_info()
    nt = int(os.environ.get("FVHIP_CPU_THREADS", "0")) or hw["physical_cores_used"]
    raw = mesh.raw()
    fd, path = tempfile.mkstemp(suffix=".npz", dir="/tmp")
    os.close(fd)
    try:
        np.savez(path, u=np.ascontiguousarray(u), **{k: np.asarray(v) for k, v in raw.items()})
        res = {}
        for threads, reps in ((nt, nrep), (1, max(3, nrep // 4))):
            env = dict(os.environ, OMP_NUM_THREADS=str(threads), OMP_PROC_BIND="close", OMP_PLACES="cores")
            out = subprocess.run([sys.executable, os.path.abspath(__file__), "--cpu-child", path, str(threads),
                                  str(reps), rec, kind, flux], env=env, capture_output=True, text=True, timeout=900)
            if out.returncode != 0:
                raise RuntimeError("cpu baseline child failed: " + out.stderr[-2000:])
            res[threads] = json.loads(out.stdout.strip().splitlines()[-1])
    finally:
        os.unlink(path)
    F = mesh.naface
    med_n, med_1 = res[nt]["median_s"], res[1]["median_s"]
    return {"value": F / med_n / 1e6, "unit": "Mfaces/s", "cores": nt, "kind": "port",
            "value_1_core": F / med_1 / 1e6, "host": hw,
            "sample": f"full second-order residual sweeps of the same {mesh.nelem}-cell mesh and state by the C++ "
                      f"restatement with the reference's omp parallel for / omp atomic structure (oracle/, -O2 "
                      f"-fopenmp, no FMA), OMP_PROC_BIND=close OMP_PLACES=cores: median of {nrep} sweeps after 3 "
                      f"warm-ups on {nt} threads = {med_n:.4f} s; median of {res[1]['nrep']} on 1 thread = "
                      f"{med_1:.3f} s"}


def cpu_child(path, threads, nrep, rec="VANALBADA", kind="naca", flux="ROE"):
    """child of cpu_baseline: builds the oracle from the saved mesh and times it (prints one JSON line)"""
    import _oracle as orc
    import cases
    d = np.load(path)
    raw = {k: (int(d[k]) if d[k].ndim == 0 else d[k]) for k in d.files if k != "u"}
    om = orc.OracleMesh.from_raw(raw)
    ref = orc.OracleSpatial(om, cases.physics(kind), cases.numerics(flux, "LEASTSQUARES", rec))
    med, times = ref.time_residual(np.ascontiguousarray(d["u"]), nrep, True, threads=threads, nwarm=3)
    print(json.dumps({"median_s": med, "nrep": nrep, "threads": threads, "min_s": float(times.min()),
                      "max_s": float(times.max())}))


def halo_parity(fa, torch, dist, mesh, p, n, u, part, rank, world, new_uid):
    """every rank's owned residual and time steps after one partitioned residual (RCCL halo), compared
    bit for bit with the 1-GPU residual of the whole mesh that rank 0 computes and broadcasts; returns
    True only if every owned row on every rank matches"""
    n.fast_math = False
    N = mesh.nelem
    full = torch.zeros((N, 5), dtype=torch.float64, device="cuda")
    if rank == 0:
        one = fa.FlowFV(mesh, p, n, device=torch.cuda.current_device())
        perm = one.permutation()
        du = torch.tensor(u[perm], device="cuda")
        dr = torch.zeros((N, 4), dtype=torch.float64, device="cuda")
        dt = torch.zeros(N, dtype=torch.float64, device="cuda")
        torch.cuda.synchronize()  # torch's stream vs the library's (non-blocking) streams
        one.compute_residual_device(du.data_ptr(), dr.data_ptr(), dt.data_ptr(), True, True)
        one.synchronize()
        idx = torch.tensor(perm, dtype=torch.int64, device="cuda")
        full[idx, :4] = dr
        full[idx, 4] = dt
        one.close()
        del du, dr, dt
    dist.broadcast(full, src=0)
    sp = fa.FlowFV(mesh, p, n, device=torch.cuda.current_device(), partition=part, rank=rank)
    sp.comm_init(world, rank, new_uid())
    owned = np.nonzero(part == rank)[0]
    gint = owned[sp.permutation()]
    du = torch.full((sp.nown + sp.nghost, 4), float("nan"), dtype=torch.float64, device="cuda")
    du[:sp.nown] = torch.tensor(u[gint], device="cuda")
    dr = torch.zeros((sp.nown, 4), dtype=torch.float64, device="cuda")
    dt = torch.zeros(sp.nown, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()  # torch's stream vs the library's (non-blocking) streams
    sp.compute_residual_device(du.data_ptr(), dr.data_ptr(), dt.data_ptr(), True, True)
    sp.synchronize()
    ref = full[torch.tensor(gint, dtype=torch.int64, device="cuda")]
    bad = torch.tensor([float((ref[:, :4] != dr).any(dim=1).sum().item() + (ref[:, 4] != dt).sum().item())],
                       dtype=torch.float64, device="cuda")
    dist.all_reduce(bad)
    sp.close()
    return bool(bad.item() == 0)


def free_port():
    """a TCP port on 127.0.0.1 that nothing listens on now (the children's rendezvous)"""
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_launch_plan(n, argv, port=None, rehearse=False):
    """the N child processes of `bench.py --gpus N` started without a torchrun environment: one rank per
    GPU, this script with the same arguments, the torch.distributed env:// variables set (rendezvous on
    127.0.0.1). Returns a list of (command, env additions)."""
    port = int(os.environ.get("MASTER_PORT") or 0) or port or free_port()
    cmd = [sys.executable, "-u", os.path.abspath(__file__)] + list(argv)
    # rehearsal on one GPU: RCCL refuses two ranks on one device unless each rank reports its own host
    extra = (lambda r: {"NCCL_HOSTID": "fvhip-rehearsal-%d" % r, "NCCL_SOCKET_IFNAME": "lo", "NCCL_IB_DISABLE": "1"}) \
        if rehearse else (lambda r: {})
    return [(cmd, {"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n), "LOCAL_WORLD_SIZE": str(n),
                   "GROUP_RANK": "0", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), **extra(r)})
            for r in range(n)]


def run_ranks(plan, timeout_s, poll_s=0.2):
    """start every child of `plan` in its own process group (this process touches no GPU), wait for all
    of them, and return the exit status: 0 if every child succeeded, else the first failing child's
    status (the others are killed); 124 when the wall-clock watchdog `timeout_s` expires (all killed).
    The children inherit stdout/stderr: rank 0 prints the JSON line."""
    import signal
    import subprocess
    procs = [subprocess.Popen(cmd, env=dict(os.environ, **env), start_new_session=True) for cmd, env in plan]

    def kill_all():
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGTERM)
                except ProcessLookupError:
                    pass
        t_end = time.time() + 10
        for p in procs:
            try:
                p.wait(timeout=max(t_end - time.time(), 0.1))
            except subprocess.TimeoutExpired:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
                p.wait()

    def on_signal(signum, frame):
        kill_all()
        sys.exit(128 + signum)
    old = {s: signal.signal(s, on_signal) for s in (signal.SIGTERM, signal.SIGINT)}
    try:
        t0 = time.time()
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                sys.stderr.write("bench.py launcher: a rank exited with status %d; stopping the others\n" % bad[0])
                kill_all()
                return bad[0] if bad[0] > 0 else 128 - bad[0]
            if all(c == 0 for c in codes):
                return 0
            if time.time() - t0 > timeout_s:
                sys.stderr.write("bench.py launcher: ranks still running after %.0f s; killed\n" % timeout_s)
                kill_all()
                return 124
            time.sleep(poll_s)
    finally:
        for s, h in old.items():
            signal.signal(s, h)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--launch-timeout", type=float, default=1500.0,
                    help="--gpus N without torchrun: wall-clock limit for the N ranks this script starts")
    ap.add_argument("--rehearse-one-gpu", action="store_true",
                    help="testing only: every rank on GPU 0, RCCL over its socket transport (NCCL_HOSTID per rank); "
                         "checks the N-rank code path on a one-GPU box, its times mean nothing")
    ap.add_argument("--launch-dry-run", action="store_true",
                    help="print the rank processes --gpus N would start (commands, environment) and exit")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--scale", type=int, default=1, help="divide the C4 mesh dimensions (debug)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sweeps", type=int, default=20, help="timed CPU-baseline sweeps (median)")
    ap.add_argument("--no-fast", action="store_true", help="skip the fast-math mode measurement")
    ap.add_argument("--scaling", choices=["weak", "strong"], default="strong")
    ap.add_argument("--partitioner", choices=["graph", "graph-faces", "graph-cells", "rcb"], default="graph",
                    help="graph: graph bisection balancing the fused residual's measured cost per cell (a quadrangle "
                         "costs ~1.44 triangles, fvens_amd.RESIDUAL_COST_WEIGHTS); graph-faces: balancing face counts; "
                         "graph-cells: balancing cell counts (the reference's unweighted Scotch graph); rcb: "
                         "coordinate bisection")
    ap.add_argument("--no-pipelined", action="store_true", help="skip the pipelined staged path")
    ap.add_argument("--no-implicit", action="store_true", help="skip the implicit-step figure (1 GPU only)")
    ap.add_argument("--implicit-deadline", type=float, default=300.0,
                    help="N GPUs: wall-clock seconds the implicit-step section may take; past it (or when any rank "
                         "fails in it) rank 0 prints the line with implicit_step = {'error': ...} and every rank exits, "
                         "so a rank stuck in a collective cannot lose the residual measurement")
    ap.add_argument("--preheat-ms", type=float, default=400.0,
                    help="untimed steps for this long (wall clock) after the warm-up steps of the primary path, "
                         "so the timed steps run at the clock the GPU holds under this load (reported)")
    ap.add_argument("--numerics", choices=["headline", "config2", "config3", "config4", "config5"], default="headline",
                    help="headline: Roe + WLS + MUSCL/Van Albada (north_star's sweep); config4: BASELINE config 4's "
                         "Roe + WLS + Venkatakrishnan (K = 20); config2: BASELINE config 2, the headline numerics on "
                         "SURVEY's C2 (229,376 cells); config3: BASELINE config 3, the laminar flat plate "
                         "(1024 x 1024 quads, M 0.2, Re 8.7e5), HLLC + WLS + unlimited linear + Sutherland viscous flux, "
                         "implicit figure matrix-free; config5: BASELINE config 5, the laminar NACA0012 "
                         "(M 0.5, Re 5000, alpha 0) on the 8.1M-cell hybrid C5 mesh (quadrangle boundary layer and wakes, "
                         "near-isotropic triangles outside: the visc-naca0012 grids' topology), Roe + WLS + "
                         "unlimited linear reconstruction (the deck's limiter none) + Sutherland viscous flux")
    args = ap.parse_args()

    # one process per GPU: under torchrun WORLD_SIZE must agree with --gpus; without it, --gpus N > 1
    # starts the N ranks here, before anything touches a GPU, and this process only waits for them
    env_world = os.environ.get("WORLD_SIZE")
    if args.gpus < 1:
        sys.exit("bench.py: --gpus must be >= 1")
    if env_world is not None and int(env_world) != args.gpus:
        sys.exit("bench.py: WORLD_SIZE=%s from the launcher differs from --gpus %d; refusing to run"
                 % (env_world, args.gpus))
    if env_world is None and (args.gpus > 1 or args.launch_dry_run):
        argv = [a for a in sys.argv[1:] if a != "--launch-dry-run"]
        plan = rank_launch_plan(args.gpus, argv, rehearse=args.rehearse_one_gpu) if args.gpus > 1 else []
        if args.launch_dry_run:
            print(json.dumps({"ranks": [{"cmd": c, "env": e} for c, e in plan],
                              "in_process": args.gpus == 1, "watchdog_s": args.launch_timeout}))
            return
        sys.exit(run_ranks(plan, args.launch_timeout))
    if args.launch_dry_run:
        print(json.dumps({"ranks": [], "in_process": True, "under_launcher": True, "world_size": int(env_world)}))
        return

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    phases = {"start_to_main": round(time.time() - T_PROCESS, 2)}

    def phase(name, t_start):
        phases[name] = round(time.time() - t_start, 2)

    tl = time.time()
    import torch
    ctrl = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(0 if args.rehearse_one_gpu else local_rank)
        dist.init_process_group("nccl", init_method="env://")
        # a host-side (gloo) group for agreeing on the implicit section's outcome: it does not queue
        # behind RCCL work a failed rank left half done
        ctrl = dist.new_group(backend="gloo")
    else:
        dist = None
        torch.cuda.set_device(0)
    phase("launch", tl)

    import fvens_amd as fa
    import cases

    t0 = time.time()
    tm = time.time()
    mult = world if (world > 1 and args.scaling == "weak") else 1
    if args.numerics == "config5":
        mult *= 2
    if args.numerics == "config3":       # BASELINE config 3: ~1M-cell laminar flat plate (tests/visc-flatplate)
        nx = 1024 * mult // args.scale
        ny = 1024 // args.scale
        mesh, dims = fa.UMesh.flat_plate(nx, ny), dict(nx=nx, ny=ny)
    elif args.numerics == "config2":     # 229,376 cells (the mesh of test_gpu_residual's naca_c2)
        nt, nq, ntri = 512 * mult // args.scale, 64 // args.scale, 192 // args.scale
        mesh = fa.UMesh.naca_ogrid(nt, nq, ntri)
        dims = dict(ntheta=nt, nquad=nq, ntri=ntri, wall_spacing=1e-4, farmap=0)
    else:
        mesh, dims = c4_mesh(fa, args.scale, mult)
    kind = {"config5": "visc", "config3": "plate"}.get(args.numerics, "naca")
    p = cases.physics(kind)
    # config 5 = testcases/visc-naca0012/laminar-implicit.ctrl: limiter none (:72), alpha 0 (:19, cases.physics)
    rec = {"config4": "VENKATAKRISHNAN", "config3": "NONE", "config5": "NONE"}.get(args.numerics, "VANALBADA")
    flux = "HLLC" if args.numerics == "config3" else "ROE"
    n = cases.numerics(flux, "LEASTSQUARES", rec)
    u = cases.state(mesh, p, seed=42)
    N, F, Fb = mesh.nelem, mesh.naface, mesh.nbface
    phase("mesh", tm)
    part = None
    partinfo = None
    if world > 1:
        tp = time.time()
        if args.partitioner == "rcb":
            part = fa.partition_rcb(mesh, world)
        else:
            part = fa.partition_graph(mesh, world, weights={"graph": "cost", "graph-faces": "faces",
                                                            "graph-cells": None}[args.partitioner])
        tp = time.time() - tp
        partinfo = {"partitioner": args.partitioner + {
                        "graph": " (recursive graph bisection, Scotch stand-in, cells weighted by their measured residual "
                                 "cost, triangle : quadrangle = 7 : 10)",
                        "graph-faces": " (recursive graph bisection, Scotch stand-in, cells weighted by face count)",
                        "graph-cells": " (recursive graph bisection, Scotch stand-in, equal cell counts)",
                        "rcb": " (coordinate bisection)"}[args.partitioner],
                    "edge_cut": fa.partition_edge_cut(mesh, part),
                    "edge_cut_rcb": fa.partition_edge_cut(mesh, fa.partition_rcb(mesh, world)),
                    "partition_s": round(tp, 2)}
        phases["partition"] = round(tp, 2)

    def new_uid():
        """a fresh RCCL unique id for every communicator (an id bootstraps exactly one)"""
        obj = [fa.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        return obj[0]

    def barrier(sp):
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        sp.synchronize()

    def measure(fast, path="default", preheat_ms=0.0):
        """ms per step (timed region bracketed by barrier + sync, max over ranks) and per-kernel ms;
        preheat_ms: after the warm-up steps, further untimed steps for that long (all ranks run the
        same count), outside the timed region"""
        n.fast_math = fast
        tlay = time.time()
        if world > 1:
            sp = fa.FlowFV(mesh, p, n, device=torch.cuda.current_device(), partition=part, rank=rank)
            sp.comm_init(world, rank, new_uid())
            owned = np.nonzero(part == rank)[0]
        else:
            sp = fa.FlowFV(mesh, p, n, device=torch.cuda.current_device())
            owned = np.arange(N)
        layout_s = round(time.time() - tlay, 2)
        gint = owned[sp.permutation()]
        du = torch.zeros((sp.nown + sp.nghost, 4), dtype=torch.float64, device="cuda")
        du[:sp.nown] = torch.tensor(u[gint], device="cuda")
        dr = torch.empty((sp.nown, 4), dtype=torch.float64, device="cuda")
        ddt = torch.empty(sp.nown, dtype=torch.float64, device="cuda")
        torch.cuda.synchronize()

        def step():
            sp.compute_residual_device(du.data_ptr(), dr.data_ptr(), ddt.data_ptr(), True, True,
                                       staged=path == "staged", pipelined=path == "pipelined")

        for _ in range(args.warmup):
            step()
        barrier(sp)
        pre = {"ms": 0.0, "steps": 0}
        if preheat_ms > 0:
            # step time from a short burst, then one batch of steps covering preheat_ms
            tb = time.perf_counter()
            for _ in range(10):
                step()
            sp.synchronize()
            est = max((time.perf_counter() - tb) / 10, 1e-5)
            k = int(preheat_ms * 1e-3 / est)
            if dist is not None:           # every rank the same count (the exchange pairs them)
                kt_ = torch.tensor([k], dtype=torch.int64, device="cuda")
                dist.all_reduce(kt_, op=dist.ReduceOp.MAX)
                k = int(kt_.item())
            for _ in range(k):
                step()
            barrier(sp)
            pre = {"ms": round((time.perf_counter() - tb) * 1e3, 1), "steps": k + 10}
        t1 = time.perf_counter()
        for _ in range(args.steps):
            step()
        sp.synchronize()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t1
        if dist is not None:
            t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
            dist.barrier()
        # per-kernel durations with HIP events on the library's stream (separate pass): an event pair around
        # every launch, and -- for a step that is one launch of one kernel -- one pair around all the steps
        # (the region average has no per-launch event overhead, which inflates kernels of ~20 us, but it
        # counts the dispatch gaps between launches: the smaller of the two is the tighter bound)
        sp.profile(True)
        for _ in range(args.steps):
            step()
        kt = sp.kernel_times()
        sp.profile(False)
        region = None
        if world == 1 and len(kt) == 1 and list(kt.values())[0][1] == args.steps:
            ext = torch.cuda.ExternalStream(sp.stream())
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            sp.synchronize()
            e0.record(ext)
            for _ in range(args.steps):
                step()
            e1.record(ext)
            e1.synchronize()
            region = e0.elapsed_time(e1) / args.steps
        measure.region_ms = region
        stats = dict(sp.layout_stats(), layout_s=layout_s)
        if dist is not None:
            dist.barrier()
        sp.close()
        # per step: a kernel launched several times per step (gradient chunks, sweep groups) is summed
        measure.preheat = pre
        return 1e3 * elapsed / args.steps, {k: v[0] / args.steps for k, v in kt.items()}, stats

    t_setup = time.time() - t0

    def dominant(km):
        k = max(km, key=km.get)
        return k, km[k]

    # every path is timed after the same wall-clock pre-heat (--preheat-ms, reported): kernel times
    # fall ~12 % over the first few hundred ms of a cold GPU, and handle set-up between the paths
    # leaves it idle for ~1 s; the primary (library default) path is timed last
    fast = None
    if not args.no_fast:
        tpa = time.time()
        fms, fk, stats = measure(True, preheat_ms=args.preheat_ms)
        phase("path_fast", tpa)
        cnt = (stats["cells"], stats["faces"], stats["bfaces"])
        fname, fsms = dominant(fk)
        fab = kernel_bytes(fname, *cnt, args.numerics) / (fsms * 1e-3) / 1e9
        ftr = pmc_traffic("fast::" + kernel_symbol(fname, args.numerics), N) if world == 1 else None
        fast = {"value": round(F / (fms * 1e-3) / 1e6, 3), "ms_per_step": round(fms, 5),
                "traffic": int(ftr[0]) if ftr else None,
                "kernels_ms": {k: round(v, 5) for k, v in fk.items()},
                "roofline_frac": round(fab / HBM_PEAK_GBS, 4), "achieved_GBs": round(fab, 1),
                "tolerance": "|dr| <= 1e-11 max|r| per variable, |d dt| <= 1e-12 |dt| "
                             "(tests/test_gpu_residual.py::test_fast_math_within_tolerance)"}
    # the two-kernel path (WLS gradient kernel + face sweep), same results bit for bit: one after
    # the other, and pipelined (gradient chunks overlapped with the sweep groups on a second stream)
    tpa = time.time()
    sms, sk, stats = measure(False, "staged", preheat_ms=args.preheat_ms)
    phase("path_staged", tpa)
    # this rank's algorithmic bytes (its owned cells, its faces incl. both copies of cut faces)
    cnt = (stats["cells"], stats["faces"], stats["bfaces"])
    sname, ssweep = [(k, v) for k, v in sk.items() if k.startswith("k_sweep")][0]
    staged = {"ms_per_step": round(sms, 5), "value": round(F / (sms * 1e-3) / 1e6, 3),
              "kernels_ms": {k: round(v, 5) for k, v in sk.items()},
              "sweep_roofline_frac": round(sweep_algorithmic_bytes(*cnt) / (ssweep * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
              "sweep_algorithmic_bytes": sweep_algorithmic_bytes(*cnt)}
    pipelined = None
    if world == 1 and not args.no_pipelined:
        tpa = time.time()
        pms, pk, _ = measure(False, "pipelined", preheat_ms=args.preheat_ms)
        phase("path_pipelined", tpa)
        pipelined = {"ms_per_step": round(pms, 5), "value": round(F / (pms * 1e-3) / 1e6, 3),
                     "kernels_ms_summed_over_chunks": {k: round(v, 5) for k, v in pk.items()},
                     "hbm_GBs_both_kernels": round((sweep_algorithmic_bytes(*cnt) + prep_algorithmic_bytes(*cnt))
                                                   / (pms * 1e-3) / 1e9, 1)}
    # the primary measurement: the library's default path for this configuration, after a wall-clock
    # pre-heat (untimed, reported): layout set-up between the secondary measurements leaves the GPU
    # idle for ~1 s, and a 20-step timed region (~6 ms) would otherwise run while the clocks ramp
    tpa = time.time()
    ms_per_step, kernels_ms, stats = measure(False, preheat_ms=args.preheat_ms)
    phase("path_primary", tpa)
    preheat = measure.preheat
    region_ms = measure.region_ms

    halo = None
    if world > 1:
        halo = {"layout_per_rank": None, "halo_parity": None, "halo_layers": 2,
                "exchange_rounds_per_residual": 1,
                "exchange": "one RCCL ncclSend/ncclRecv round of u rows (layer-1 + layer-2 ghosts); layer-1 "
                            "ghost gradients computed locally (k_grad_ghost), on a comm stream overlapped "
                            "with the interior patches"}
        allstats = [None] * world
        dist.all_gather_object(allstats, stats)
        halo["layout_per_rank"] = [{k: st[k] for k in ("cells", "ghosts", "neighbours", "send_rows",
                                                        "patches", "interior_patches", "layout_s")} for st in allstats]
        if args.scaling == "strong":
            thp = time.time()
            try:
                halo["halo_parity"] = halo_parity(fa, torch, dist, mesh, p, n, u, part, rank, world, new_uid)
            except Exception as e:          # report, do not lose the measurement
                halo["halo_parity"] = "error: %s" % e
            phase("halo_parity", thp)
    sweep_name, sweep_ms = dominant(kernels_ms)
    sweep_name = [sweep_name]
    pair_ms = sweep_ms
    if region_ms is not None:                        # one GPU only (a rank's step has several kernels)
        sweep_ms = min(pair_ms, region_ms)

    ab = kernel_bytes(sweep_name[0], *cnt, args.numerics)
    achieved = ab / (sweep_ms * 1e-3) / 1e9
    value = F / (ms_per_step * 1e-3) / 1e6       # every face of the (global) mesh once per step

    # recorded (NOT measured by this run): the committed full-size convergence runs of the same
    # device solver (~10 min each), kept apart from the measured figures
    recorded = None
    if world == 1 and not args.no_implicit and args.numerics in ("headline", "config4"):
        recorded = {"note": "read from committed profiles, not re-run here"}
        runs = (("c4_first_order_converged_bench_mesh.txt",
                 "first-order LLF, line-implicit preconditioner, GMRES(40), expResidualRamp CFL 5 -> 1000"),
                ("c4_first_order_converged.txt",
                 "first-order Roe, point-block Jacobi, GMRES(40), expResidualRamp CFL 5 -> 200"))
        for key, (fname, stage) in zip(("c4_converged_run", "c4_converged_run_wall1e-3"), runs):
            import glob
            found = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", fname)))   # the newest round's run
            if not found:
                continue
            conv = found[-1]
            last = json.loads(open(conv).read().strip().splitlines()[-1])
            st = last["stages"][0]
            recorded[key] = {
                "source": os.path.relpath(conv, ROOT), "cells": last["cells"], "mesh": last["dims"],
                "stage": stage, "steps": st["steps"], "seconds": st["seconds"], "ms_per_step": st["ms_per_step"],
                "drop_from_peak": st["drop_from_peak"], "drop_from_first": st["drop_from_first"]}

    # the C-ABI's host-pointer entry (fvhip_compute_residual: the reference's own calling convention, u, r
    # and dtm in host memory in reference order), PCIe and host work included -- reported, never `value`
    host_boundary = None
    if world == 1:
        n.fast_math = False
        hb = fa.FlowFV(mesh, p, n, device=torch.cuda.current_device())
        hr = np.zeros((N, 4))
        hdt = np.zeros(N)
        hb.compute_residual(u, hr, True, hdt)                       # warm-up: staging buffers
        reps = 5
        th = time.perf_counter()
        for _ in range(reps):
            hr[:] = 0.0
            hb.compute_residual(u, hr, True, hdt)
        hms = (time.perf_counter() - th) / reps * 1e3
        hb.close()
        del hr, hdt
        host_boundary = {"ms_per_call": round(hms, 3), "Mfaces_per_s": round(F / (hms * 1e-3) / 1e6, 3),
                         "calls": reps,
                         "note": "fvhip_compute_residual with host arrays in reference order (u, r in; r, dtm out): "
                                 "PCIe transfers and reordering included; the device-resident residual is `value`"}
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(mesh, u, args.cpu_sweeps, rec, kind, flux)

    # secondary figure: the device implicit pseudo-time step (BASELINE configs 3-5) on the
    # same mesh -- residual, analytic Jacobian, GMRES(30) with the line-implicit preconditioner, update --
    # with a first-order start, from the free stream and after that start (IMPLICIT_START); on N GPUs every
    # rank its partition's piece (lines cut at rank boundaries, GMRES dot products through ncclAllReduce), the
    # slowest rank's time. It runs last, after the line's other fields are final.
    def implicit_section():
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        from bench_implicit import implicit_steps
        kw = {}
        if world > 1:
            def allmax(x):
                t = torch.tensor([x], dtype=torch.float64, device="cuda")
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                return float(t.item())
            kw = dict(part=part, rank=rank, world=world, new_uid=new_uid, allmax=allmax)
        start = dict(IMPLICIT_START)
        if args.numerics == "config3":
            # the flat plate's free stream is a steady state of the density residual up to rounding (its
            # second-order residual there is ~1e-16): a ratio from it means nothing, so the steps are
            # timed after the first-order start (one step: its first-order residual is exactly 0)
            start["second_from"] = "start"
        im = next(implicit_steps(mesh, {"config5": "visc-c5", "config3": "plate"}.get(args.numerics, "naca"),
                                 steps=3, warmup=1, sweeps=1, lines=True,
                                 # BASELINE configs 3 and 5 name the matrix-free operator
                                 operators=((True,) if args.numerics in ("config3", "config5") else (False,)),
                                 **start, **kw))
        im.pop("faces", None)
        return im

    if rank == 0:
        # template of the timed sweep: k_residual_wls<FLUX=ROE(4), REC=MUSCL(1), DT, VISC=none(0), LIM=0>
        # (config4: REC=linear(2), LIM=Venkatakrishnan(2))
        tr = pmc_traffic("exact::" + kernel_symbol(sweep_name[0], args.numerics), N) if world == 1 else None
        cb = counter_bound(tr[3] if tr else None, sweep_ms)
        wl = {"headline": "C4 mesh, Roe + WLS gradients + MUSCL/Van Albada",
              "config2": "C2 mesh (SURVEY 8(d): 229,376-cell hybrid NACA0012 O-grid), Roe + WLS gradients + "
                         "MUSCL/Van Albada, BASELINE config 2's numerics",
              "config3": "flat plate (1024 x 1024 quads), laminar M 0.2 Re 8.7e5, HLLC + WLS gradients + unlimited "
                         "linear + Sutherland viscous flux, BASELINE config 3's numerics",
              "config4": "C4 mesh, Roe + WLS gradients + Venkatakrishnan (K = 20), BASELINE config 4's numerics",
              "config5": "C5 mesh (8.1M cells), laminar M 0.5 Re 5000 alpha 0, Roe + WLS gradients + unlimited linear "
                         "reconstruction + Sutherland viscous flux, BASELINE config 5's numerics "
                         "(visc-naca0012/laminar-implicit.ctrl)"}[args.numerics]
        out = {
            "metric": "Mfaces/s (flux+residual sweep) + achieved HBM GB/s, 1/2/4/8 MI355X",
            "value": round(value, 3),
            "unit": "Mfaces/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 5),
            "higher_is_better": True,
            # N = 1 is the first point of the same (default strong) series the multi-GPU runs extend
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f64",
            "data": ("synthetic (generated structured flat-plate quad mesh; seeded perturbed free stream)"
                     if args.numerics == "config3" else
                     "synthetic (generated NACA0012 hybrid mesh: quadrangle boundary layer and wakes, near-isotropic "
                     "triangles outside; seeded perturbed free stream)" if args.numerics == "config5" else
                     "synthetic (generated NACA0012 hybrid O-grid; seeded perturbed free stream)"),
            "config": {"workload": f"{wl}, 2nd-order residual sweep with local time steps "
                                   "(explicit pseudo-time step)",
                       "cells": N, "faces": F, "boundary_faces": Fb, **dims,
                       "parallelism": (f"dp{world}: {args.partitioner} {world}-way partition, two-layer halo, one RCCL "
                                       f"p2p exchange of u per residual"
                                       if world > 1 else "single GPU"),
                       "layout": stats, "setup_s": round(t_setup, 2),
                       **({"rehearsal_one_gpu": "all ranks on GPU 0, RCCL over sockets: times are not a measurement"}
                          if args.rehearse_one_gpu else {})},
            "preheat": {**preheat, "note": "untimed steps of the primary path after its warm-up, outside the "
                                           "timed region (--preheat-ms)"},
            "roofline": {"bound": cb["bound"] if cb else None,
                         "bound_basis": ({**cb, "source": tr[1], "rule": "valu if SQ_ACTIVE_INST_VALU x 4 / "
                                          "(1024 SIMDs x GRBM_GUI_ACTIVE / 8) exceeds PMC bytes / time / 8 TB/s"}
                                         if cb else "no committed PMC profile of this kernel on this workload"),
                         "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": int(tr[0]) if tr else None,
                         "traffic_source": tr[1] if tr else None,
                         "kernel": sweep_name[0] if sweep_name else None,
                         "kernel_ms": round(sweep_ms, 5),
                         "kernel_ms_event_pairs": round(pair_ms, 5),
                         "kernel_ms_region": round(region_ms, 5) if region_ms is not None else None,
                         "kernel_ms_method": ("min(HIP event pair per launch, HIP event pair around the timed steps / "
                                              "steps) on the library's stream" if region_ms is not None else
                                              "HIP event pair per launch on the library's stream"),
                         "algorithmic_bytes": ab,
                         "bytes_basis": ("SURVEY.md 8(d) 32F + 144N + 48Fb (124.0 B/face) + 8N time step"
                                         if args.numerics not in ("config3", "config4", "config5") else
                                         "SURVEY.md 8(d) linear reconstruction (config4: + Venkatakrishnan): "
                                         "48F + 144N + 48Fb + 8N time step"),
                         "frac_area_dt_basis": round(sweep_bytes_area_dt(*cnt) / (sweep_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                         "area_dt_basis": "same + 8N (time step as area read 8 + dtm write 8 = 16 B/cell)",
                         "compulsory_bytes_one_launch": residual_algorithmic_bytes(*cnt),
                         "frac_of_measured_peak": round(achieved / HBM_MEASURED_GBS, 4)},
            "valu_roofline": valu_roofline(tr[2] if tr else None, sweep_ms),
            "kernels_ms": {k: round(v, 5) for k, v in kernels_ms.items()},
            "multi_gpu": ({**partinfo, **halo} if world > 1 else None),
            "halo_parity": (halo["halo_parity"] if world > 1 else None),
            "cpu_baseline": cpu,
            "host_boundary": host_boundary,
            "fast_math": fast,
            "staged_path": staged,
            "pipelined_path": pipelined,
            "implicit_step": None,
            "recorded": recorded,
            "build": fa._ffi.build_info(),
        }
    ti = time.time()
    if args.no_implicit:
        implicit = None
    elif world == 1:
        implicit = implicit_section()
    else:
        implicit = guarded_implicit(implicit_section, args.implicit_deadline, dist, ctrl, rank,
                                    lambda im: emit(out, im, phases, ti) if rank == 0 else None)
    if not args.no_implicit:
        phase("implicit", ti)
    if rank == 0:
        emit(out, implicit, phases, None)
    if dist is not None:
        dist.destroy_process_group()


def emit(out, implicit, phases, t_implicit):
    """rank 0's one JSON line: the measurement with the implicit figure (or its error) and the wall-clock
    phases of this process (t_implicit: start of an implicit section cut short by its deadline)"""
    if t_implicit is not None:
        phases = dict(phases, implicit=round(time.time() - t_implicit, 2))
    out["implicit_step"] = implicit
    out["phases_s"] = dict(phases, total=round(time.time() - T_PROCESS, 2))
    print(json.dumps(out), flush=True)


GUARD_EXIT = 3     # exit status of a rank whose implicit section missed the deadline


def guarded_implicit(section, deadline_s, dist, ctrl, rank, on_deadline):
    """N ranks: run the implicit section (collectives over RCCL) so that its failure cannot lose the line.
    A rank whose section raises keeps the error; the ranks then agree over the host-side gloo group `ctrl`
    (an error anywhere is an error everywhere). A rank stuck in a collective -- its peer failed, or a
    transport hangs -- never reaches the agreement: when `deadline_s` passes, every rank's timer fires,
    rank 0 prints the line with the error (on_deadline) and every process exits at once with status
    GUARD_EXIT (the run did not finish). A lock orders the timer against the agreement: once the ranks have
    agreed the timer can no longer fire, so exactly one line is printed."""
    import threading
    import torch
    lock = threading.Lock()
    state = {"agreed": False}

    def expire():
        with lock:
            if state["agreed"]:
                return
            try:
                on_deadline({"error": "implicit section did not finish on every rank within %.0f s" % deadline_s})
            finally:
                sys.stdout.flush()
                sys.stderr.flush()
                os._exit(GUARD_EXIT)
    timer = threading.Timer(deadline_s, expire)
    timer.daemon = True
    timer.start()
    try:
        im, err = section(), None
    except Exception as e:
        im, err = None, "rank %d: %s" % (rank, e)
    flag = torch.tensor([0.0 if err is None else 1.0 + rank], dtype=torch.float64)
    dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=ctrl)
    with lock:
        state["agreed"] = True
    timer.cancel()
    if err is not None:
        return {"error": err}
    if flag.item() > 0:
        return {"error": "rank %d failed in the implicit section" % (int(flag.item()) - 1)}
    return im


if __name__ == "__main__":
    if len(sys.argv) == 8 and sys.argv[1] == "--cpu-child":
        cpu_child(sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), sys.argv[5], sys.argv[6], sys.argv[7])
    else:
        main()
