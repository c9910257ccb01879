"""probe: where the residual of the stalled second-order solve on a C4-family grid sits"""
import sys
sys.path.insert(0, "."); sys.path.insert(0, "tests")
import numpy as np
import torch
import fvens_amd as fa
import cases

p = cases.physics("naca")
m = fa.UMesh.naca_ogrid(256, 32, 108, 20.0, 1e-3)
rc = m.rc
for rec in ("VANALBADA", "NONE"):
    sp = fa.FlowFV(m, p, cases.numerics("ROE", "LEASTSQUARES", rec))
    perm = sp.permutation()
    du = torch.tensor(np.tile(cases.freestream(p), (m.nelem, 1))[perm], device="cuda")
    try:
        steps, ratio, hist = sp.steady_forward_euler_device(du.data_ptr(), 0.5, 1e-12, 150000)
    except RuntimeError as e:
        print(rec, e); continue
    u = np.empty((m.nelem, 4)); u[perm] = du.cpu().numpy()
    r = np.zeros((m.nelem, 4)); dt = np.zeros(m.nelem)
    sp.compute_residual(u, r, True, dt)
    a = m.area
    e = np.abs(r[:, 3])                              # energy residual (flux balance, not / area)
    idx = np.argsort(e)[::-1][:12]
    tot = np.sqrt((r[:, 3]**2 * a).sum())
    print(rec, "steps", steps, "norm", tot, "share of the top 12 cells", np.sqrt((r[idx, 3]**2 * a[idx]).sum()) / tot, flush=True)
    for c in idx:
        print("   cell %7d rc (%.4f, %.4f) r_E %.2e area %.2e rho %.4f" % (c, rc[c, 0], rc[c, 1], r[c, 3], a[c], u[c, 0]))
    # distribution by radius
    rad = np.hypot(rc[:, 0] - 0.5, rc[:, 1])
    for lo, hi in ((0, 0.6), (0.6, 2), (2, 10), (10, 30)):
        s = (rad >= lo) & (rad < hi)
        print("   radius [%g,%g): %d cells, norm share %.3f" % (lo, hi, s.sum(), np.sqrt((r[s, 3]**2 * a[s]).sum()) / tot))
    sp.close()
