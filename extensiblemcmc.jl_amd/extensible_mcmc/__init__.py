"""extensible_mcmc — Python host mirror of ExtensibleMCMC.jl's API over the
MI355X many-chain engine (libemcmc.so, include/emcmc.h).

Names follow the reference's exports (src/ExtensibleMCMC.jl:31-41); Julia's
``run!``/``reschedule!`` become ``run``/``reschedule``.  Indices (coords,
mcmciter, pidx) stay 1-based as in the reference.
"""
from .callbacks import Callback, REPLCallback, SavingCallback
from .diagnostics import allgather_moments, merge as merge_moments, rhat_from_moments
from .engine import Engine, EngineConfig
from .kernels import (AdaptationUnifRW, GaussianRandomWalk, GaussianRandomWalkMix, HaarioTypeAdaptation,
                      HamiltonianMCUpdate, ImproperPosPrior, ImproperPrior, MALAUpdate, MCMCBackend,
                      MCMCParamUpdate, MCMCUpdate, NoAdaptation, ProductPrior, RandomWalkUpdate, StandardPrior,
                      UniformRandomWalk, UnsupportedPlugin, isdecorator, isequal_except, Normal, Uniform,
                      Exponential, Gamma, Product, LogNormal, Beta, InverseGamma, Cauchy, Laplace, TDist,
                      MvNormal, UserUpdate)
from .mcmc import (MCMC, GenericMCMCBackend, MI355XBackend, MI355XGlobalWorkspace, MI355XLocalWorkspace,
                   create_workspaces, get_decorators, init, run, run_)
from .schedule import JRange, MCMCSchedule, Step, reschedule, reschedule_
from .targets import GsnTargetLaw, LogisticRegressionLaw, UserTargetLaw, make_data
from ._lib import EMCMCError, device_count

__all__ = [
    "MCMC", "UniformRandomWalk", "GaussianRandomWalk", "GaussianRandomWalkMix", "AdaptationUnifRW",
    "HaarioTypeAdaptation", "NoAdaptation", "RandomWalkUpdate", "GenericMCMCBackend", "MI355XBackend",
    "GsnTargetLaw", "run", "run_", "get_decorators", "isdecorator", "ImproperPosPrior", "ImproperPrior",
    "SavingCallback", "REPLCallback", "MCMCSchedule", "JRange", "reschedule", "Engine", "EngineConfig",
    "EMCMCError", "device_count", "rhat_from_moments", "allgather_moments", "merge_moments", "MALAUpdate", "LogisticRegressionLaw",
    "StandardPrior", "ProductPrior", "Normal", "Uniform", "Exponential", "Gamma", "Product",
    "LogNormal", "Beta", "InverseGamma", "Cauchy", "Laplace", "TDist", "MvNormal", "UserUpdate", "UserTargetLaw",
]
