"""Solver counterparts (callers of the operator layer): the operator applies of
Solvers/ConvectionDiffusion_Solver.py and Solvers/NavierStokes_Solver.py on the GPU, and the OpenMDAO Boussinesq coupling of the two."""
from .convection_diffusion import ConvectionDiffusionSolver  # noqa: F401
from .navier_stokes import NavierStokesSolver  # noqa: F401
from .boussinesq import BoussinesqCoupler, ParallelBoussinesqCoupler  # noqa: F401
from .components import ConvectionDiffusion_Component, NavierStokes_Component  # noqa: F401

__all__ = ["ConvectionDiffusionSolver", "NavierStokesSolver", "BoussinesqCoupler", "ParallelBoussinesqCoupler",
           "ConvectionDiffusion_Component", "NavierStokes_Component"]
