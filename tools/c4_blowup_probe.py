"""probe: where and when does the unlimited / Venkatakrishnan second-order explicit solve on a
C4-family grid lose positivity? Chunks of explicit steps; per chunk the cell of minimum pressure
and of maximum |residual|."""
import sys
sys.path.insert(0, "."); sys.path.insert(0, "tests")
import numpy as np
import torch
import fvens_amd as fa
import cases

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 8
rec = sys.argv[2] if len(sys.argv) > 2 else "NONE"
p = cases.physics("naca")
farmap = int(sys.argv[3]) if len(sys.argv) > 3 else 0
m = fa.UMesh.naca_ogrid(2048 // scale, 256 // scale, 864 // scale, 20.0, 1e-3, farmap=farmap)
sp = fa.FlowFV(m, p, cases.numerics("ROE", "LEASTSQUARES", rec, K=5.0))
perm = np.asarray(sp.permutation())
du = torch.tensor(np.tile(cases.freestream(p), (m.nelem, 1))[perm], device="cuda")
rc = np.asarray(m.rc[:m.nelem])[perm]
g = p.gamma
done = 0
for chunk in [1]*5 + [5]*4 + [20]*10 + [100]*20 + [1000]*30:
    try:
        steps, ratio, hist = sp.steady_forward_euler_device(du.data_ptr(), 0.5, 1e-30, chunk)
    except RuntimeError as e:
        print("diverged in chunk after", done, e, flush=True)
        break
    done += chunk
    u = du.cpu().numpy()
    rho = u[:, 0]; pr = (g - 1) * (u[:, 3] - 0.5 * (u[:, 1]**2 + u[:, 2]**2) / rho)
    i = int(np.argmin(pr)); j = int(np.argmax(pr)); vm = np.hypot(u[:, 1], u[:, 2]) / rho; k = int(np.argmax(vm))
    print(f"step {done}: res {hist[steps-1]:.3e} min p {pr[i]:.4e} at ({rc[i,0]:.4f},{rc[i,1]:.4f}) max p {pr[j]:.4e} at ({rc[j,0]:.4f},{rc[j,1]:.4f}) max |v| {vm[k]:.3f} at ({rc[k,0]:.4f},{rc[k,1]:.4f})", flush=True)
