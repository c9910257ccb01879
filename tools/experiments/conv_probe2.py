"""probe: LS+HLLC cylinder entropy convergence on all four meshes under several linear-solver settings:
finest slopes and the residual drop each main solve reached"""
import sys
sys.path.insert(0, "."); sys.path.insert(0, "tests")
import numpy as np
import test_gpu_convergence as t

case = sys.argv[1] if len(sys.argv) > 1 else "ls_hllc_implicit"
SETS = [dict(prec_sweeps=1), dict(prec_sweeps=1, lin_rtol=1e-2), dict(prec_sweeps=1, lin_maxit=100, restart=100),
        dict(prec_sweeps=2, prec_gs=True, lin_rtol=1e-2), dict(prec_sweeps=1, lin_rtol=1e-2, lin_maxit=100, restart=100),
        dict(prec_sweeps=2, prec_gs=True, lin_maxit=100, restart=100, lin_rtol=1e-2), dict(prec_sweeps=3, prec_gs=True),
        dict(prec_sweeps=1, min_relax=0.5), dict(prec_sweeps=1, lin_rtol=3e-2)]
grad, flux, imp, init, main, nmesh, drop, _ = t.CASES[case]
for sett in SETS:
    lh, le, rr = [], [], []
    import fvens_amd as fa
    orig = fa.ImplicitConfig.__init__
    def patched(self, *a, **k):
        k.update(sett)
        orig(self, *a, **k)
    fa.ImplicitConfig.__init__ = patched
    for i in range(nmesh):
        n, err, erro, st, conv = t.solve_entropy("2dcylinder%d" % i, grad, flux, imp, init, main, drop)
        lh.append(np.log10(1/np.sqrt(n))); le.append(np.log10(err)); rr.append(st["resratio"])
    fa.ImplicitConfig.__init__ = orig
    sl = [(le[i]-le[i-1])/(lh[i]-lh[i-1]) for i in range(1, nmesh)]
    print(sett, "slopes", np.round(sl, 4), "errs", np.round(le, 5), "ratios", ["%.1e" % x for x in rr], flush=True)
