#!/usr/bin/env python3
"""One rank of tests/test_gpu_rccl_ranks.py: N processes on ONE GPU drive the library's own RCCL
communicator through its real multi-rank legs (ncclSend/ncclRecv halo exchange inside
ncclGroupStart/End, ncclAllReduce of the Krylov dot products and norms, ncclMin of the TVD-RK step).

RCCL refuses two ranks on one device ("Duplicate GPU detected", keyed by host hash and bus id), so each
rank sets its own NCCL_HOSTID: RCCL then sees N hosts and moves the data over its socket transport on
the loopback interface -- slow, but the library's calls, their pairing and their ordering are exactly
those of the one-GPU-per-rank run. torch.distributed (gloo) only rendezvouses the ranks and carries the
RCCL unique id and the results; the single-GPU reference results are computed by every rank itself.

usage (set by the test): RANK, WORLD_SIZE, MASTER_ADDR, MASTER_PORT, NCCL_HOSTID in the environment;
argv: <out.json> <mesh key> <partitioner> [numerics]  (numerics: "visc" = laminar Roe + WLS + Van Albada +
Sutherland, "venkat" = Roe + WLS + Venkatakrishnan)
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)


def main():
    out_path, meshkey, partitioner = sys.argv[1], sys.argv[2], sys.argv[3]
    mode = sys.argv[4] if len(sys.argv) > 4 else ""

    def mark(msg):
        print("[rank %s] %s" % (os.environ["RANK"], msg), flush=True)
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method="env://")
    torch.cuda.set_device(0)
    import fvens_amd as fa
    import cases
    from test_gpu_residual import get_mesh

    m, _ = get_mesh(meshkey)
    p = cases.physics("visc" if mode == "visc" else "naca")
    n = cases.numerics("ROE", "LEASTSQUARES", "VENKATAKRISHNAN" if mode == "venkat" else "VANALBADA")
    part = fa.partition_graph(m, world, weights="cost") if partitioner == "graph" else fa.partition_rcb(m, world)

    def uid():
        obj = [fa.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        return obj[0]

    if os.environ.get("FVHIP_CRASHTRACE"):
        # diagnostic: native backtrace of a crash (tools/probes/crashtrace.c), installed after every
        # library that might set its own handlers has loaded
        import ctypes
        ctypes.CDLL(os.environ["FVHIP_CRASHTRACE"])
        mark("crash tracer installed")
    rep = {"rank": rank, "world": world}
    owned = np.nonzero(part == rank)[0]
    mark("mesh and partition ready")

    # 1. residuals: five back-to-back partitioned residuals on changing states, each owned row bitwise
    #    the single-GPU residual (ghost rows start as NaN: a missed exchange cannot pass)
    one = fa.FlowFV(m, p, n)
    sp = fa.FlowFV(m, p, n, partition=part, rank=rank)
    sp.comm_init(world, rank, uid())
    g = owned[sp.permutation()]
    p1 = one.permutation()
    bad = 0
    for k in range(5):
        u = cases.state(m, p, seed=20 + k)
        du1 = torch.tensor(u[p1], device="cuda")
        dr1 = torch.zeros_like(du1)
        dt1 = torch.zeros(m.nelem, dtype=torch.float64, device="cuda")
        torch.cuda.synchronize()  # torch's stream vs the library's (non-blocking) streams
        one.compute_residual_device(du1.data_ptr(), dr1.data_ptr(), dt1.data_ptr(), True, True)
        one.synchronize()                 # the library's stream, not torch's
        r1 = np.empty((m.nelem, 4))
        t1 = np.empty(m.nelem)
        r1[p1] = dr1.cpu().numpy()
        t1[p1] = dt1.cpu().numpy()
        du = torch.full((sp.nown + sp.nghost, 4), float("nan"), dtype=torch.float64, device="cuda")
        du[:sp.nown] = torch.tensor(u[g], device="cuda")
        dr = torch.zeros((sp.nown, 4), dtype=torch.float64, device="cuda")
        dt = torch.zeros(sp.nown, dtype=torch.float64, device="cuda")
        torch.cuda.synchronize()
        sp.compute_residual_device(du.data_ptr(), dr.data_ptr(), dt.data_ptr(), True, True)
        sp.synchronize()
        bad += int((dr.cpu().numpy() != r1[g]).any(axis=1).sum() + (dt.cpu().numpy() != t1[g]).sum())
    rep["residual_mismatched_rows"] = bad
    rep["layout"] = sp.layout_stats()
    mark("residuals done")

    # 2. implicit steps (GMRES dot products and norms through ncclAllReduce; block-Jacobi across ranks
    #    for the line preconditioner): the same steps as a one-process group of the same partition
    u0 = cases.state(m, p, seed=8)
    for lines in (False, True):
        cfg = fa.ImplicitConfig(cflinit=10.0, cflfin=200.0, tol=0.0, maxiter=3, lin_rtol=1e-4, lin_maxit=60,
                                restart=20, prec_sweeps=2 if not lines else 1, min_relax=0.2, prec_lines=lines)
        du = torch.full((sp.nown + sp.nghost, 4), float("nan"), dtype=torch.float64, device="cuda")
        du[:sp.nown] = torch.tensor(u0[g], device="cuda")
        torch.cuda.synchronize()
        st, hist = sp.steady_backward_euler_device(du.data_ptr(), cfg)
        sp.synchronize()
        ur = du[:sp.nown].cpu().numpy()
        # the in-process group of the same partition (device copies, host sums), on rank 0's view
        sps = [fa.FlowFV(m, p, n, partition=part, rank=k) for k in range(world)]
        dus = []
        for k, s_ in enumerate(sps):
            gk = np.nonzero(part == k)[0][s_.permutation()]
            d = torch.full((s_.nown + s_.nghost, 4), float("nan"), dtype=torch.float64, device="cuda")
            d[:s_.nown] = torch.tensor(u0[gk], device="cuda")
            dus.append(d)
        torch.cuda.synchronize()
        grp = fa.FlowFVGroup(sps)
        stg, histg = grp.steady_backward_euler_device([d.data_ptr() for d in dus], cfg)
        for s_ in sps:
            s_.synchronize()
        ug = dus[rank][:sps[rank].nown].cpu().numpy()
        grp.close()
        for s_ in sps:
            s_.close()
        scale = np.abs(u0[g] - ug).max()
        key = "implicit_lines" if lines else "implicit_pbj"
        rep[key] = {"steps": st["steps"], "lin_iters": st["lin_iters"], "group_lin_iters": stg["lin_iters"],
                    "hist_rel": float(np.max(np.abs(np.asarray(hist) - np.asarray(histg)) / np.abs(histg))),
                    "u_rel": float(np.abs(ur - ug).max() / scale)}
        mark("implicit %s done" % key)

    # 3. TVD-RK: the global dtmin through ncclMin, bitwise the one-GPU steps
    mark("tvdrk")
    u0 = cases.state(m, p, seed=9)
    du1 = torch.tensor(u0[p1], device="cuda")
    torch.cuda.synchronize()
    s1, t1 = one.tvdrk_device(du1.data_ptr(), 3, 0.4, 1e9, 3)
    one.synchronize()
    uo = np.empty_like(u0)
    uo[p1] = du1.cpu().numpy()
    du = torch.full((sp.nown + sp.nghost, 4), float("nan"), dtype=torch.float64, device="cuda")
    du[:sp.nown] = torch.tensor(u0[g], device="cuda")
    torch.cuda.synchronize()
    s, t = sp.tvdrk_device(du.data_ptr(), 3, 0.4, 1e9, 3)
    sp.synchronize()
    rep["tvdrk"] = {"steps": s, "time_equal": t == t1,
                    "mismatched_rows": int((du[:sp.nown].cpu().numpy() != uo[g]).any(axis=1).sum())}
    sp.close()
    one.close()
    with open(out_path, "w") as f:
        json.dump(rep, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
