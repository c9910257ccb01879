"""probe: LS+HLLC cylinder entropy convergence on all four meshes under several linear-solver settings"""
import sys
sys.path.insert(0, "."); sys.path.insert(0, "tests")
import numpy as np
import test_gpu_convergence as t

for sw, gs in ((1, False), (4, False), (2, True)):
    grad, flux, imp, init, main, nmesh, drop, _ = t.CASES["ls_hllc_implicit"]
    lh, le, rr = [], [], []
    import fvens_amd as fa
    orig = fa.ImplicitConfig.__init__
    def patched(self, *a, **k):
        orig(self, *a, **k)
        self.prec_sweeps, self.prec_gs = sw, gs
    fa.ImplicitConfig.__init__ = patched
    for i in range(4):
        n, err, erro, st, conv = t.solve_entropy("2dcylinder%d" % i, grad, flux, imp, init, main, drop)
        lh.append(np.log10(1/np.sqrt(n))); le.append(np.log10(err)); rr.append(st["resratio"])
    fa.ImplicitConfig.__init__ = orig
    sl = [(le[i]-le[i-1])/(lh[i]-lh[i-1]) for i in range(1, 4)]
    print(sw, gs, "slopes", np.round(sl, 4), "errs", np.round(le, 5), "ratios", ["%.1e" % x for x in rr], flush=True)
