"""Shared test cases: meshes (reference fixtures + synthetic), configurations mirroring the
reference's control files, and seeded flow states."""
import os

import numpy as np

import fvens_amd as fa
from fvens_amd import FlowBCConfig, FlowNumericsConfig, FlowPhysicsConfig

HERE = os.path.dirname(os.path.abspath(__file__))
MESHDIR = os.path.join(HERE, "fixtures", "meshes")


def fixture_mesh(name):
    return os.path.join(MESHDIR, name + ".msh")


def physics(kind, aoa_deg=0.0, Minf=None):
    """Physics + BCs of the reference test decks.
    'cyl'   inviscid cylinder, tests/inv-2dcyl/inv-cyl-base.ctrl (slipwall 2, farfield 4, M 0.38)
    'naca'  transonic NACA0012, testcases/naca0012/transonic-sanity-test-muscl.ctrl (M 0.8, 1.25 deg)
    'visc'  laminar NACA0012, testcases/visc-naca0012/laminar-implicit.ctrl (Re 5000, M 0.5, alpha 0: :19-31)
    'plate' flat plate, tests/visc-flatplate/flatplate.ctrl (M 0.2, Re 8.7e5, T 290.19 K, Pr 0.708)
    'wall'  tests/flow-general/test.ctrl (farfield 4, adiabatic 2, isothermal 3; M 0.5, Re 5000);
            the deck's wall temperature 290 is used as a non-dimensional value by abc.cpp:349-366,
            which makes the ghost state non-physical, so 1.1 (x free-stream T) is used here
    """
    d2r = np.pi / 180.0
    if kind == "cyl":
        return FlowPhysicsConfig(gamma=1.4, Minf=Minf or 0.38, aoa=aoa_deg * d2r,
                                 bcconf=[FlowBCConfig("slipwall", 2), FlowBCConfig("farfield", 4)])
    if kind == "naca":
        return FlowPhysicsConfig(gamma=1.4, Minf=Minf or 0.8, aoa=1.25 * d2r,
                                 bcconf=[FlowBCConfig("slipwall", 2), FlowBCConfig("farfield", 4)])
    if kind == "visc":
        return FlowPhysicsConfig(gamma=1.4, Minf=Minf or 0.5, Tinf=288.15, Reinf=5000.0, Pr=0.72,
                                 aoa=aoa_deg * d2r, viscous_sim=True,
                                 bcconf=[FlowBCConfig("adiabaticwall", 2, [0.0]),
                                         FlowBCConfig("inflowoutflow", 4)])
    if kind == "viscconst":
        p = physics("visc")
        p.const_visc = True
        return p
    if kind == "plate":
        return FlowPhysicsConfig(gamma=1.4, Minf=Minf or 0.2, Tinf=290.19, Reinf=8.7e5, Pr=0.708,
                                 viscous_sim=True,
                                 bcconf=[FlowBCConfig("slipwall", 3), FlowBCConfig("adiabaticwall", 2, [0.0]),
                                         FlowBCConfig("farfield", 4), FlowBCConfig("inflowoutflow", 5)])
    if kind == "plate_inviscid":
        return FlowPhysicsConfig(gamma=1.4, Minf=Minf or 0.2,
                                 bcconf=[FlowBCConfig("slipwall", 3), FlowBCConfig("extrapolation", 2),
                                         FlowBCConfig("farfield", 4), FlowBCConfig("inflowoutflow", 5)])
    if kind == "wall":
        return FlowPhysicsConfig(gamma=1.4, Minf=0.5, Tinf=288.15, Reinf=5000.0, Pr=0.72, viscous_sim=True,
                                 bcconf=[FlowBCConfig("farfield", 4), FlowBCConfig("adiabaticwall", 2, [0.0]),
                                         FlowBCConfig("isothermalwall", 3, [0.0, 1.1])])
    raise ValueError(kind)


def numerics(flux="ROE", grad="LEASTSQUARES", rec="VANALBADA", order2=True, jac=None, K=20.0):
    return FlowNumericsConfig(conv_numflux=flux, conv_numflux_jac=jac or flux, gradientscheme=grad,
                              reconstruction=rec, limiter_param=K, order2=order2)


def freestream(p):
    g, M, a = p.gamma, p.Minf, p.aoa
    pinf = 1.0 / (g * M * M)
    return np.array([1.0, np.cos(a), np.sin(a), pinf / (g - 1.0) + 0.5])


def state(mesh, p, seed=42, amp=0.05):
    """Free stream perturbed smoothly: rho, p *(1+amp sin), v += amp sin, seeded."""
    rng = np.random.default_rng(seed)
    x = mesh.rc[:mesh.nelem, 0]
    y = mesh.rc[:mesh.nelem, 1]
    g, M, a = p.gamma, p.Minf, p.aoa
    pinf = 1.0 / (g * M * M)

    def wave():
        k = rng.integers(1, 5, size=2)
        ph = rng.random(2)
        return np.sin(2 * np.pi * (k[0] * x / 3.0 + ph[0])) * np.cos(2 * np.pi * (k[1] * y / 3.0 + ph[1]))
    rho = 1.0 * (1 + amp * wave())
    pr = pinf * (1 + amp * wave())
    vx = np.cos(a) + amp * wave()
    vy = np.sin(a) + amp * wave()
    u = np.empty((mesh.nelem, 4))
    u[:, 0] = rho
    u[:, 1] = rho * vx
    u[:, 2] = rho * vy
    u[:, 3] = pr / (g - 1.0) + 0.5 * rho * (vx * vx + vy * vy)
    return np.ascontiguousarray(u)
