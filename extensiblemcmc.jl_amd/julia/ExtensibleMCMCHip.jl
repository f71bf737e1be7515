#===============================================================================
    ExtensibleMCMCHip.jl — MI355X backend for ExtensibleMCMC.jl over libemcmc.so

    Adds `MI355XBackend <: MCMCBackend` (the extension point of
    src/types.jl:110-117) with the global/local workspace constructors the
    reference dispatches on (src/workspaces.jl:38, :280) and a `run!` method
    for `MCMC` objects built with this backend.  The hot loop (__run!,
    src/run.jl:64-83) executes on the GPU through the C ABI declared in
    include/emcmc.h; the schedule (src/schedule.jl) stays in Julia and is
    handed over as a list of (mcmciter, pidx) steps.

    Not executed in this repository's CI (no Julia in the build image); the
    Python twin (extensible_mcmc/_lib.py) exercises the same entry points.
===============================================================================#
module ExtensibleMCMCHip

using ExtensibleMCMC
import Distributions
const eMCMC = ExtensibleMCMC

const LIB = get(ENV, "EMCMC_LIB", joinpath(@__DIR__, "..", "lib", "libemcmc.so"))
const ABI_VERSION = UInt32(2)

# ---- C structs (include/emcmc.h) ---------------------------------------------
struct EmcmcConfig
    abi_version::UInt32
    dim::UInt32
    num_chains::UInt64
    first_chain_id::UInt64
    num_mcmc_steps::UInt64
    seed::UInt64
    device::Int32
    history_mode::UInt32
    roll_window::UInt32
    lanes_per_chain::UInt32
    steps_per_launch::UInt32
    kernel_variant::UInt32
    chain_moments::UInt32
    history_ring::UInt32
    reserved::NTuple{4,UInt32}
end

struct EmcmcUpdateDesc
    kernel::UInt32
    prior::UInt32
    adaptation::UInt32
    num_coords::UInt32
    coords::Ptr{UInt32}
    sigma::Ptr{Float64}
    epsilon::Ptr{Float64}
    pos::Ptr{UInt8}
    adaptation_params::Ptr{Cvoid}
    sigma_b::Ptr{Float64}
    prior_params::Ptr{Cvoid}          # const emcmc_prior_desc* (ProductPrior / StandardPrior)
    user_update::Ptr{Cvoid}           # const emcmc_user_update_desc* (EMCMC_USER_UPDATE)
    mix_lambda::Float64
    reserved_f64::NTuple{3,Float64}
end

struct EmcmcHaarioAdaptation
    adapt_every_k_steps::UInt32
    reserved::UInt32
    scale::Float64
end

struct EmcmcTargetDesc
    kind::UInt32
    dim::UInt32
    mu::Ptr{Float64}
    sigma::Ptr{Float64}
    num_obs::UInt64
    obs::Ptr{Float64}
    ll_mode::UInt32
    reserved::UInt32
    labels::Ptr{Float64}              # EMCMC_TARGET_LOGISTIC: y
end

# include/emcmc.h emcmc_user_target_desc: a user law compiled at run time (hiprtc)
struct EmcmcUserTargetDesc
    dim::UInt32
    obs_dim::UInt32
    theta0::Ptr{Float64}
    num_obs::UInt64
    obs::Ptr{Float64}
    num_params::UInt64
    params::Ptr{Float64}
    source::Cstring
    options::Cstring
end

struct EmcmcPriorFactor
    family::UInt32
    count::UInt32
    a::Float64
    b::Float64
    components::Ptr{EmcmcPriorFactor}   # EMCMC_DIST_PRODUCT: count univariate components
    mu::Ptr{Float64}                    # EMCMC_DIST_MVNORMAL: μ
    sigma::Ptr{Float64}                 # EMCMC_DIST_MVNORMAL: Σ, column-major
end

struct EmcmcPriorDesc
    num_factors::UInt32
    reserved::UInt32
    factors::Ptr{EmcmcPriorFactor}
end

struct EmcmcStep
    mcmciter::UInt32
    pidx::UInt32
end

struct EmcmcUserUpdateDesc
    source::Cstring
    options::Cstring
    num_params::UInt64
    params::Ptr{Float64}
end

const RW_GAUSSIAN = UInt32(2)
const RW_GAUSSIAN_MIX = UInt32(3)
const MALA = UInt32(4)
const USER_UPDATE = UInt32(5)
const ADPT_HAARIO = UInt32(2)
const PRIOR_IMPROPER, PRIOR_IMPROPER_POS, PRIOR_PRODUCT, PRIOR_STANDARD = UInt32(0), UInt32(1), UInt32(2), UInt32(3)
const DIST_NORMAL, DIST_UNIFORM, DIST_EXPONENTIAL, DIST_GAMMA = UInt32(1), UInt32(2), UInt32(3), UInt32(4)
const DIST_LOGNORMAL, DIST_BETA, DIST_INVERSE_GAMMA = UInt32(5), UInt32(6), UInt32(7)
const DIST_CAUCHY, DIST_LAPLACE, DIST_TDIST = UInt32(8), UInt32(9), UInt32(10)
const DIST_PRODUCT, DIST_MVNORMAL = UInt32(32), UInt32(33)
const ADPT_NONE = UInt32(0)
const TARGET_GSN = UInt32(1)
const H_STATE, H_PROPOSAL, H_LL, H_ACCEPT = UInt32(0), UInt32(1), UInt32(2), UInt32(3)

"""
    HipTargetLaw(source, θ; params = Float64[], options = "")

A user-defined target law for `MI355XBackend`: the law's parameter vector θ
(`set_parameters!(P, idx, θ)` writes into it, as for any law of the reference,
src/example/gsn_target.jl:15-21) and its `loglikelihood(P, obs)` written as an
`EMCMC_USER_LOGLIK { … }` body — plus, for `HipMALAUpdate`, its gradient as an
`EMCMC_USER_GRAD { … }` body (the law's `compute_gradients_and_momenta!`) —
(include/emcmc.h emcmc_user_target_desc), which the
engine compiles for the device.  `obs` is the `data.obs` vector of observation
vectors (all of one length).
"""
struct HipTargetLaw{T}
    θ::Vector{T}
    source::String
    params::Vector{Float64}
    options::String
end
HipTargetLaw(source::String, θ::Vector{T}; params = Float64[], options = "") where {T} =
    HipTargetLaw{T}(copy(θ), source, Float64.(params), options)
function eMCMC.set_parameters!(P::HipTargetLaw, loc2glob_idx, θ)
    P.θ[loc2glob_idx] .= θ
end

function _set_user_target(h, P::HipTargetLaw, obs)
    X = isempty(obs) ? zeros(0, 1) : reduce(vcat, permutedims.(obs))   # n×w
    Xrm = permutedims(X)                                                # row-major for the ABI
    θ0 = Float64.(P.θ)
    GC.@preserve X Xrm θ0 P begin
        t = Ref(EmcmcUserTargetDesc(UInt32(length(θ0)), UInt32(size(X, 2)), pointer(θ0), UInt64(size(X, 1)),
                                    isempty(Xrm) ? Ptr{Float64}(C_NULL) : pointer(Xrm), UInt64(length(P.params)),
                                    isempty(P.params) ? Ptr{Float64}(C_NULL) : pointer(P.params),
                                    Base.unsafe_convert(Cstring, P.source), Base.unsafe_convert(Cstring, P.options)))
        check(ccall((:emcmc_set_user_target, LIB), Cint, (Ptr{Cvoid}, Ref{EmcmcUserTargetDesc}), h, t),
              h, "emcmc_set_user_target")
    end
end

"""
    HipUpdate(source, coords; params = Float64[], prior = ImproperPrior(), options = "")

A user-defined `MCMCParamUpdate` for `MI355XBackend`.  The reference's update
plugin surface — `proposal!(updt, global_ws, ws, step)` and
`log_transition_density(updt, θ, θ°)` (src/updates.jl:42-93) — written once as an
`EMCMC_USER_PROPOSAL { … } EMCMC_USER_LTD { … }` source (include/emcmc.h
emcmc_user_update_desc) that the engine compiles for the device, with `params`
as its constants and draws from the engine's stream (`em_randn(j)`,
`em_rand(j)`).  `set_parameters!` is the generic `P°.θ[coords] ← θ°`
(updates.jl:198-205); the prior enters the ratio as for any update.
"""
struct HipUpdate{K,P} <: eMCMC.MCMCParamUpdate
    source::String
    coords::K
    invcoords::Dict{Int,Int}
    params::Vector{Float64}
    prior::P
    adpt::eMCMC.NoAdaptation
    options::String
end
HipUpdate(source::String, coords; params = Float64[], prior = eMCMC.ImproperPrior(), options = "") =
    HipUpdate(source, coords, Dict(c => i for (i, c) in enumerate(coords)), Float64.(params), prior,
              eMCMC.NoAdaptation(), options)

function _update_desc(updt::HipUpdate, keep)
    coords = UInt32.(collect(updt.coords) .- 1)
    pk, pp = _prior_desc(updt.prior, length(coords), keep)
    ud = Ref(EmcmcUserUpdateDesc(Base.unsafe_convert(Cstring, updt.source), Base.unsafe_convert(Cstring, updt.options),
                                 UInt64(length(updt.params)),
                                 isempty(updt.params) ? Ptr{Float64}(C_NULL) : pointer(updt.params)))
    push!(keep, coords, ud, updt)
    EmcmcUpdateDesc(USER_UPDATE, pk, ADPT_NONE, UInt32(length(coords)), pointer(coords), C_NULL, C_NULL, C_NULL,
                    C_NULL, C_NULL, pp, Base.unsafe_convert(Ptr{Cvoid}, ud), 0.0, (0.0, 0.0, 0.0))
end

"""
    HipMALAUpdate(ϵ, coords; prior = ImproperPrior())

MALA for `MI355XBackend`: the reference declares `MALAUpdate <: MCMCGradientBasedUpdate`
without fields or methods (src/updates.jl:216-218) and gives gradient-based
updates one hook, `compute_gradients_and_momenta!` (updates.jl:123-133, called at
run.jl:110 and run.jl:259).  The engine's definition (DESIGN.md §2): θ° = θ +
(ϵ²/2)∇ℓ + ϵz, MvNormal(·, ϵ²I) transition densities both ways, the prior in the
ratio.  ∇ℓ is the target's: the built-in GsnTargetLaw's, or a `HipTargetLaw`
whose source also defines `EMCMC_USER_GRAD { … }` (include/emcmc.h); on the
logistic-regression target the fused MFMA kernel runs it.
"""
struct HipMALAUpdate{K,P} <: eMCMC.MCMCGradientBasedUpdate
    ϵ::Float64
    coords::K
    invcoords::Dict{Int,Int}
    prior::P
    adpt::eMCMC.NoAdaptation
end
HipMALAUpdate(ϵ::Real, coords; prior = eMCMC.ImproperPrior()) =
    HipMALAUpdate(Float64(ϵ), coords, Dict(c => i for (i, c) in enumerate(coords)), prior, eMCMC.NoAdaptation())

function _update_desc(updt::HipMALAUpdate, keep)
    coords = UInt32.(collect(updt.coords) .- 1)
    pk, pp = _prior_desc(updt.prior, length(coords), keep)
    eps = [updt.ϵ]
    push!(keep, coords, eps, updt)
    EmcmcUpdateDesc(MALA, pk, ADPT_NONE, UInt32(length(coords)), pointer(coords), C_NULL, pointer(eps), C_NULL,
                    C_NULL, C_NULL, pp, C_NULL, 0.0, (0.0, 0.0, 0.0))
end

function check(st, h, where)
    st == 0 && return nothing
    msg = h == C_NULL ? "" : unsafe_string(ccall((:emcmc_last_error, LIB), Cstring, (Ptr{Cvoid},), h))
    error("$where failed with emcmc_status $st: $msg")
end

# ---- backend -------------------------------------------------------------------
"""
    MI355XBackend(; num_chains=1, seed=0, first_chain_id=0, device=0,
                  history=:full, ll_mode=:per_obs)

Many-chain GPU backend: each of the `num_chains` chains is an independent
replica of the reference's single-chain sampler, keyed by its global id.
"""
Base.@kwdef struct MI355XBackend <: eMCMC.MCMCBackend
    num_chains::Int = 1
    seed::UInt64 = 0
    first_chain_id::Int = 0
    device::Int = 0
    history::Symbol = :full
    ll_mode::Symbol = :per_obs
    chain_moments::Bool = false   # GenericChainStats mean/cov on device (chain_statistics.jl:46-49)
    callback_chain::Int = 1       # the chain the reference's callbacks (SavingCallback, REPLCallback) observe
end

mutable struct MI355XGlobalWorkspace{T} <: eMCMC.GlobalWorkspace{T}
    handle::Ptr{Cvoid}
    backend::MI355XBackend
    num_mcmc_steps::Int
    dim::Int
    num_updates::Int
    num_locals::Int
    num_coords::Vector{Int}        # per update: length(updt.coords)
    coords::Vector{Vector{Int}}    # per update: updt.coords (1-based)
    names::Vector{String}          # per update: string(remove_curly(typeof(updt))) (workspaces.jl:474)
    last_iter::Vector{Int}         # per update: the last mcmciter __run! handed to the device (0: none)
    θinit::Vector{T}
end

struct MI355XLocalWorkspace{T} <: eMCMC.LocalWorkspace{T}
    gws::MI355XGlobalWorkspace{T}
    pidx::Int
end

struct EmcmcUnifRWAdaptation
    adapt_every_k_steps::UInt32
    reserved::UInt32
    target_accpt_rate::Float64
    scale::Float64
    min::Float64
    max::Float64
    offset::Float64
end

# include/emcmc.h emcmc_unifrw_adaptation_vec: the per-coordinate form
struct EmcmcUnifRWAdaptationVec
    adapt_every_k_steps::UInt32
    reserved::UInt32
    target_accpt_rate::Float64
    scale::Ptr{Float64}
    min::Ptr{Float64}
    max::Ptr{Float64}
    offset::Ptr{Float64}
end

const RW_UNIFORM = UInt32(1)
const ADPT_UNIF_RW = UInt32(1)
const ADPT_UNIF_RW_VEC = UInt32(3)

# priors.jl:18-88 → (EMCMC_PRIOR_*, emcmc_prior_desc pointer or C_NULL).
# Every factor goes with its `dims` entry as count; the engine rebuilds the
# constructor's index list (priors.jl:64-79: dims 1 → θ[1], dims k → a range).
_uf(fam, a, b) = EmcmcPriorFactor(fam, UInt32(1), Float64(a), Float64(b), C_NULL, C_NULL, C_NULL)
_dist_factor(d::Distributions.Normal, k, keep) = _uf(DIST_NORMAL, d.μ, d.σ)
_dist_factor(d::Distributions.Uniform, k, keep) = _uf(DIST_UNIFORM, d.a, d.b)
_dist_factor(d::Distributions.Exponential, k, keep) = _uf(DIST_EXPONENTIAL, d.θ, 0.0)
_dist_factor(d::Distributions.Gamma, k, keep) = _uf(DIST_GAMMA, d.α, d.θ)
_dist_factor(d::Distributions.LogNormal, k, keep) = _uf(DIST_LOGNORMAL, d.μ, d.σ)
_dist_factor(d::Distributions.Beta, k, keep) = _uf(DIST_BETA, d.α, d.β)
_dist_factor(d::Distributions.InverseGamma, k, keep) = _uf(DIST_INVERSE_GAMMA, Distributions.shape(d), Distributions.scale(d))
_dist_factor(d::Distributions.Cauchy, k, keep) = _uf(DIST_CAUCHY, d.μ, d.σ)
_dist_factor(d::Distributions.Laplace, k, keep) = _uf(DIST_LAPLACE, d.μ, d.θ)
_dist_factor(d::Distributions.TDist, k, keep) = _uf(DIST_TDIST, d.ν, 0.0)
function _dist_factor(d::Distributions.Product, k, keep)
    comps = EmcmcPriorFactor[_dist_factor(c, 1, keep) for c in d.v]
    push!(keep, comps)
    EmcmcPriorFactor(DIST_PRODUCT, UInt32(k), 0.0, 0.0, pointer(comps), C_NULL, C_NULL)
end
function _dist_factor(d::Distributions.MvNormal, k, keep)
    μ, Σ = Vector{Float64}(Distributions.mean(d)), Matrix{Float64}(Distributions.cov(d))
    push!(keep, μ, Σ)
    EmcmcPriorFactor(DIST_MVNORMAL, UInt32(k), 0.0, 0.0, C_NULL, pointer(μ), pointer(Σ))
end
_dist_factor(d, k, keep) = error("no device plugin for prior distribution $(typeof(d))")

function _prior_desc(prior, n, keep)
    prior isa eMCMC.ImproperPrior && return PRIOR_IMPROPER, C_NULL
    prior isa eMCMC.ImproperPosPrior && return PRIOR_IMPROPER_POS, C_NULL
    if prior isa eMCMC.ProductPrior
        # prior.idx holds 1 for a dims-1 factor and a range otherwise (priors.jl:68-73)
        fs = EmcmcPriorFactor[_dist_factor(d, ix isa Integer ? 1 : length(ix), keep)
                              for (d, ix) in zip(prior.dists, prior.idx)]
        kind = PRIOR_PRODUCT
    elseif prior isa eMCMC.StandardPrior && prior.dist isa Distributions.MultivariateDistribution
        fs = EmcmcPriorFactor[_dist_factor(prior.dist, length(prior.dist), keep)]
        kind = PRIOR_STANDARD
    else
        error("no device plugin for $(typeof(prior)) on $n coordinates")
    end
    pd = Ref(EmcmcPriorDesc(UInt32(length(fs)), UInt32(0), pointer(fs)))
    push!(keep, fs, pd)
    kind, Base.unsafe_convert(Ptr{Cvoid}, pd)
end

function _update_desc(updt::eMCMC.RandomWalkUpdate, keep)
    coords = UInt32.(collect(updt.coords) .- 1)                 # 0-based across the ABI
    pk, pp = _prior_desc(updt.prior, length(coords), keep)
    push!(keep, coords)
    adpt, adptp = ADPT_NONE, C_NULL
    if updt.rw isa eMCMC.GaussianRandomWalk
        updt.adpt isa eMCMC.NoAdaptation || error("no device plugin for $(typeof(updt.adpt)) with GaussianRandomWalk")
        Σ = Matrix{Float64}(updt.rw.Σ)                         # column-major already
        pos = UInt8.(updt.rw.pos)                               # log-scale coordinates (random_walk.jl:136-171)
        push!(keep, Σ, pos)
        return EmcmcUpdateDesc(RW_GAUSSIAN, pk, ADPT_NONE, UInt32(length(coords)), pointer(coords),
                               pointer(Σ), C_NULL, pointer(pos), C_NULL, C_NULL, pp, C_NULL, 0.0,
                               (0.0, 0.0, 0.0))
    elseif updt.rw isa eMCMC.GaussianRandomWalkMix                # random_walk.jl:193-232
        ΣA = Matrix{Float64}(updt.rw.gsn_A.Σ)
        ΣB = Matrix{Float64}(updt.rw.gsn_B.Σ)
        pos = UInt8.(updt.rw.gsn_A.pos)                           # both components share pos (:198-205)
        push!(keep, ΣA, ΣB, pos)
        if updt.adpt isa eMCMC.HaarioTypeAdaptation              # adaptation.jl:372-426 (fλ must be identity)
            p = Ref(EmcmcHaarioAdaptation(UInt32(updt.adpt.adapt_every_k_steps), UInt32(0), updt.adpt.scale))
            push!(keep, p)
            adpt, adptp = ADPT_HAARIO, Base.unsafe_convert(Ptr{Cvoid}, p)
        elseif !(updt.adpt isa eMCMC.NoAdaptation)
            error("no device plugin for $(typeof(updt.adpt)) with GaussianRandomWalkMix")
        end
        return EmcmcUpdateDesc(RW_GAUSSIAN_MIX, pk, adpt, UInt32(length(coords)), pointer(coords),
                               pointer(ΣA), C_NULL, pointer(pos), adptp, pointer(ΣB), pp, C_NULL, updt.rw.λ,
                               (0.0, 0.0, 0.0))
    elseif updt.rw isa eMCMC.UniformRandomWalk                      # random_walk.jl:45-94, pos included
        ϵ = Float64.(collect(updt.rw.ϵ))
        pos = UInt8.(collect(updt.rw.pos) .!= 0)
        push!(keep, ϵ, pos)
        if updt.adpt isa eMCMC.AdaptationUnifRW{Float64}      # scalar form (adaptation.jl:162-169)
            a = updt.adpt
            p = Ref(EmcmcUnifRWAdaptation(UInt32(a.adapt_every_k_steps), UInt32(0), a.target_accpt_rate, a.scale,
                                          a.min, a.max, a.offset))
            push!(keep, p)
            adpt, adptp = ADPT_UNIF_RW, Base.unsafe_convert(Ptr{Cvoid}, p)
        elseif updt.adpt isa eMCMC.AdaptationUnifRW              # Vector / SVector form (adaptation.jl:171-188)
            a = updt.adpt
            v = [Float64.(collect(a.scale)), Float64.(collect(a.min)), Float64.(collect(a.max)),
                 Float64.(collect(a.offset))]
            p = Ref(EmcmcUnifRWAdaptationVec(UInt32(a.adapt_every_k_steps), UInt32(0), a.target_accpt_rate,
                                             pointer(v[1]), pointer(v[2]), pointer(v[3]), pointer(v[4])))
            push!(keep, v, p)
            adpt, adptp = ADPT_UNIF_RW_VEC, Base.unsafe_convert(Ptr{Cvoid}, p)
        elseif !(updt.adpt isa eMCMC.NoAdaptation)
            error("no device plugin for $(typeof(updt.adpt))")
        end
        return EmcmcUpdateDesc(RW_UNIFORM, pk, adpt, UInt32(length(coords)), pointer(coords), C_NULL,
                               pointer(ϵ), pointer(pos), adptp, C_NULL, pp, C_NULL, 0.0, (0.0, 0.0, 0.0))
    end
    error("no device plugin for $(typeof(updt.rw))")
end

# Field reads that only a RandomWalkUpdate has (`rw`, its λ, the Haario `adpt`)
# go through these predicates: HipUpdate and HipMALAUpdate have no `rw`
# (updates.jl:42-93 and :129-133 define no such field for a plugin update).
_mix(u) = u isa eMCMC.RandomWalkUpdate && u.rw isa eMCMC.GaussianRandomWalkMix
_haario_mix(u) = _mix(u) && u.adpt isa eMCMC.HaarioTypeAdaptation

# emcmc_lambda_fn trampoline: ctx is a HaarioTypeAdaptation, kept alive by the
# MCMC object for the whole run!
function _flam_trampoline(λ::Float64, N::Int64, it::Int64, ctx::Ptr{Cvoid})::Float64
    adpt = unsafe_pointer_to_objref(ctx)::eMCMC.HaarioTypeAdaptation
    Float64(adpt.fλ(λ, N, it))
end
_flam_cfunction() = @cfunction(_flam_trampoline, Float64, (Float64, Int64, Int64, Ptr{Cvoid}))

# workspaces.jl:38 — init_global_workspace(::MCMCBackend, …)
function eMCMC.init_global_workspace(be::MI355XBackend, num_mcmc_steps,
                                     updates::Vector{<:eMCMC.MCMCUpdate}, data, θinit::Vector{T};
                                     kwargs...) where T
    D = length(θinit)
    cfg = Ref(EmcmcConfig(ABI_VERSION, UInt32(D), UInt64(be.num_chains), UInt64(be.first_chain_id),
                          UInt64(num_mcmc_steps), be.seed, Int32(be.device),
                          be.history === :full ? UInt32(0) : UInt32(1), UInt32(100), UInt32(0),
                          UInt32(0), UInt32(0), UInt32(be.chain_moments), UInt32(0), ntuple(_ -> UInt32(0), 4)))
    h = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:emcmc_create, LIB), Cint, (Ref{Ptr{Cvoid}}, Ref{EmcmcConfig}), h, cfg), C_NULL, "emcmc_create")
    keep = Any[]
    GC.@preserve keep begin
        for (i, u) in enumerate(updates)
            desc = Ref(_update_desc(u, keep))
            check(ccall((:emcmc_add_update, LIB), Cint, (Ptr{Cvoid}, Ref{EmcmcUpdateDesc}), h[], desc),
                  h[], "emcmc_add_update")
            if _haario_mix(u)
                # fλ (adaptation.jl:425) runs in Julia at every readjust: the library
                # calls back with (λ, N, mcmc_iter); ctx is the (mutable) adaptation
                check(ccall((:emcmc_set_mix_lambda_fn, LIB), Cint, (Ptr{Cvoid}, UInt32, Ptr{Cvoid}, Ptr{Cvoid}),
                            h[], UInt32(i), _flam_cfunction(), pointer_from_objref(u.adpt)),
                      h[], "emcmc_set_mix_lambda_fn")
            end
        end
    end
    P = data.P
    if P isa HipTargetLaw
        _set_user_target(h[], P, data.obs)
    else
    d = length(P.θ) == 0 ? 0 : Int(round((sqrt(1 + 4length(P.θ)) - 1) / 2))  # θ = [μ; vec Σ]
    μ = P.θ[1:d]
    Σ = reshape(P.θ[(d+1):end], d, d)
    X = reduce(vcat, permutedims.(data.obs))                     # n×d
    Xrm = permutedims(X)                                           # row-major view for the ABI
    GC.@preserve μ Σ Xrm begin
        t = Ref(EmcmcTargetDesc(TARGET_GSN, UInt32(d), pointer(μ), pointer(Σ), UInt64(size(X, 1)),
                                pointer(Xrm), be.ll_mode === :per_obs ? UInt32(0) : UInt32(1), UInt32(0),
                                Ptr{Float64}(C_NULL)))
        check(ccall((:emcmc_set_target, LIB), Cint, (Ptr{Cvoid}, Ref{EmcmcTargetDesc}), h[], t),
              h[], "emcmc_set_target")
    end
    end
    θ0 = repeat(Float64.(θinit), be.num_chains)                     # [C][D] row-major
    check(ccall((:emcmc_set_state, LIB), Cint, (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}), h[], θ0, C_NULL),
          h[], "emcmc_set_state")
    ws = MI355XGlobalWorkspace{T}(h[], be, num_mcmc_steps, D, length(updates), 0,
                                  [length(u.coords) for u in updates], [collect(Int, u.coords) for u in updates],
                                  [string(eMCMC.remove_curly(typeof(u))) for u in updates],
                                  zeros(Int, length(updates)), copy(θinit))
    finalizer(w -> ccall((:emcmc_destroy, LIB), Cvoid, (Ptr{Cvoid},), w.handle), ws)
    ws
end

# workspaces.jl:280 — create_workspace(::MCMCBackend, mcmcupdate, global_ws, num_mcmc_steps);
# the per-update state lives on the device, the local workspace only names it.
function eMCMC.create_workspace(::MI355XBackend, updt, gws::MI355XGlobalWorkspace{T},
                                num_mcmc_steps) where T
    gws.num_locals += 1
    MI355XLocalWorkspace{T}(gws, gws.num_locals)
end

# run.jl:64-83 — __run!(global_ws, local_wss, updates, schedule, callbacks).
# run!() (run.jl:34) dispatches here through the workspace type: the schedule is
# walked in Julia, cut at callback boundaries, and each slice runs on the GPU.
function eMCMC.__run!(gws::MI355XGlobalWorkspace, local_wss, updates, schedule, callbacks)
    h = gws.handle
    steps = EmcmcStep[]
    flush!() = begin
        if !isempty(steps)
            check(ccall((:emcmc_run, LIB), Cint, (Ptr{Cvoid}, Ptr{EmcmcStep}, UInt64), h, steps,
                        length(steps)), h, "emcmc_run")
            empty!(steps)
        end
        check(ccall((:emcmc_synchronize, LIB), Cint, (Ptr{Cvoid},), h), h, "emcmc_synchronize")
    end
    pre, post = eMCMC.PreMCMCStep(), eMCMC.PostMCMCStep()
    wants(step, flag) = any(cb -> eMCMC.check_if_execute(cb, step, flag), callbacks)
    for step in schedule
        # callbacks observe device state only at the steps they ask for
        # (callbacks.jl:33-45); everything between two such steps is one slice
        if wants(step, pre)
            flush!()
            eMCMC.update_callbacks!(callbacks, gws, local_wss, step, pre)
        end
        push!(steps, EmcmcStep(UInt32(step.mcmciter), UInt32(step.pidx)))   # both 1-based across the ABI
        gws.last_iter[step.pidx] = step.mcmciter
        if wants(step, post)
            flush!()
            eMCMC.update_callbacks!(callbacks, gws, local_wss, step, post)
        end
    end
    flush!()
    for (i, u) in enumerate(updates)   # readjust! mutates rw.λ (adaptation.jl:425)
        if _mix(u)
            λ = Ref(0.0)
            check(ccall((:emcmc_get_mix_lambda, LIB), Cint, (Ptr{Cvoid}, UInt32, Ref{Float64}), h, UInt32(i), λ),
                  h, "emcmc_get_mix_lambda")
            u.rw.λ = λ[]
        end
    end
    nothing
end

"""
    state(gws::MI355XGlobalWorkspace) -> Matrix{Float64} (C × D)

Current θ of every chain (`state(global_ws)` of the reference, per chain).
"""
function eMCMC.state(gws::MI355XGlobalWorkspace)
    out = Matrix{Float64}(undef, gws.dim, gws.backend.num_chains)      # column-major = row-major [C][D]
    check(ccall((:emcmc_get_state, LIB), Cint, (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}), gws.handle, out, C_NULL),
          gws.handle, "emcmc_get_state")
    permutedims(out)
end

"""
    state_history(gws, iter_first, n) -> Array{Float64,4} (D, C, P, n)

`state_history[iter][pidx]` of every chain for iterations iter_first:iter_first+n-1.
"""
function state_history(gws::MI355XGlobalWorkspace, iter_first::Integer, n::Integer)
    out = Array{Float64}(undef, gws.dim, gws.backend.num_chains, gws.num_updates, n)
    check(ccall((:emcmc_get_history, LIB), Cint,
                (Ptr{Cvoid}, UInt32, UInt64, UInt64, Ptr{Cvoid}, Csize_t),
                gws.handle, H_STATE, iter_first, n, out, sizeof(out)), gws.handle, "emcmc_get_history")
    out
end

function _history(gws::MI355XGlobalWorkspace, which, out, iter_first, n)
    check(ccall((:emcmc_get_history, LIB), Cint,
                (Ptr{Cvoid}, UInt32, UInt64, UInt64, Ptr{Cvoid}, Csize_t),
                gws.handle, which, iter_first, n, out, sizeof(out)), gws.handle, "emcmc_get_history")
    out
end

"""
    proposal_history(gws, iter_first, n) -> Array{Float64,4} (D, C, P, n)

`state_proposal_history[iter][pidx]` (run.jl:237-239) of every chain.
"""
proposal_history(gws::MI355XGlobalWorkspace, iter_first::Integer, n::Integer) =
    _history(gws, H_PROPOSAL, Array{Float64}(undef, gws.dim, gws.backend.num_chains, gws.num_updates, n),
             iter_first, n)

"""
    ll_history(gws, iter_first, n) -> Array{Float64,3} (C, P, n)

`local_wss[pidx].sub_ws.ll_history` (run.jl:333) of every chain.
"""
ll_history(gws::MI355XGlobalWorkspace, iter_first::Integer, n::Integer) =
    _history(gws, H_LL, Array{Float64}(undef, gws.backend.num_chains, gws.num_updates, n), iter_first, n)

"""
    acceptance_history(gws, iter_first, n) -> Array{Bool,3} (C, P, n)

`local_wss[pidx].acceptance_history` (run.jl:334) of every chain, unpacked
from the device's one-bit-per-chain rows.
"""
function acceptance_history(gws::MI355XGlobalWorkspace, iter_first::Integer, n::Integer)
    C = gws.backend.num_chains
    words = _history(gws, H_ACCEPT, Array{UInt64}(undef, cld(C, 64), gws.num_updates, n), iter_first, n)
    [((words[(c - 1) >> 6 + 1, p, i] >> ((c - 1) & 63)) & 1) == 1 for c in 1:C, p in 1:gws.num_updates, i in 1:n]
end

"""
    rolling_acceptance(gws) -> (rolling_ar::Matrix{Float64} (C, P), accepted::Matrix{UInt64} (C, P))

Current `GenericChainStats.rolling_ar[last iteration][pidx]` (chain_statistics.jl:51-65)
and accepted counts of every chain.
"""
function rolling_acceptance(gws::MI355XGlobalWorkspace)
    ra = Matrix{Float64}(undef, gws.backend.num_chains, gws.num_updates)
    acc = Matrix{UInt64}(undef, gws.backend.num_chains, gws.num_updates)
    check(ccall((:emcmc_get_chain_stats, LIB), Cint, (Ptr{Cvoid}, Ptr{Float64}, Ptr{UInt64}), gws.handle, ra, acc),
          gws.handle, "emcmc_get_chain_stats")
    ra, acc
end

"""
    adaptation_state(gws, pidx) -> (ϵ::Matrix{Float64} (C, k), proposed::Vector{UInt32}, accepted::Vector{UInt32})

UniformRandomWalk ϵ as adapted and AdaptationUnifRW's counters
(adaptation.jl:51-70, 273-329) of update `pidx` for every chain.
"""
function adaptation_state(gws::MI355XGlobalWorkspace, pidx::Integer)
    C, k = gws.backend.num_chains, gws.num_coords[pidx]
    ϵ = Matrix{Float64}(undef, k, C)
    prop, acc = Vector{UInt32}(undef, C), Vector{UInt32}(undef, C)
    check(ccall((:emcmc_get_update_state, LIB), Cint, (Ptr{Cvoid}, UInt32, Ptr{Float64}, Ptr{UInt32}, Ptr{UInt32}),
                gws.handle, UInt32(pidx), ϵ, prop, acc), gws.handle, "emcmc_get_update_state")
    permutedims(ϵ), prop, acc
end

"""
    chain_moments(gws) -> (mean::Matrix{Float64} (C, D), cov::Array{Float64,3} (D, D, C))

GenericChainStats running mean/cov of every chain (chain_statistics.jl:46-49).
"""
function chain_moments(gws::MI355XGlobalWorkspace)
    C, D = gws.backend.num_chains, gws.dim
    m = Matrix{Float64}(undef, D, C)
    cov = Array{Float64}(undef, D, D, C)   # symmetric blocks: row- and column-major agree
    check(ccall((:emcmc_get_chain_moments, LIB), Cint, (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}), gws.handle, m, cov),
          gws.handle, "emcmc_get_chain_moments")
    permutedims(m), cov
end

"""
    mix_state(gws, pidx) -> (L_B::Array{Float64,3} (D, D, C), M::Int)

GaussianRandomWalkMix: lower Cholesky factor of every chain's Σ_B and
HaarioTypeAdaptation's own-turn count since the last readjust (adaptation.jl:399-426).
"""
function mix_state(gws::MI355XGlobalWorkspace, pidx::Integer)
    C, D = gws.backend.num_chains, gws.num_coords[pidx]
    L = Array{Float64}(undef, D, D, C)     # [C][D][D] row-major, transposed below
    M = Ref{UInt32}(0)                     # the same for every chain
    check(ccall((:emcmc_get_mix_state, LIB), Cint, (Ptr{Cvoid}, UInt32, Ptr{Float64}, Ref{UInt32}),
                gws.handle, UInt32(pidx), L, M), gws.handle, "emcmc_get_mix_state")
    permutedims(L, (2, 1, 3)), Int(M[])
end

"""
    adaptation_moments(gws, pidx) -> (mean::Matrix{Float64} (C, n), cov::Array{Float64,3} (n, n, C))

HaarioTypeAdaptation's own running mean/cov of update `pidx` (adaptation.jl:406-414):
the update's coordinates, log scale where pos, registered after every update step.
"""
function adaptation_moments(gws::MI355XGlobalWorkspace, pidx::Integer)
    C, n = gws.backend.num_chains, gws.num_coords[pidx]
    m = Matrix{Float64}(undef, n, C)
    cov = Array{Float64}(undef, n, n, C)
    check(ccall((:emcmc_get_adaptation_moments, LIB), Cint, (Ptr{Cvoid}, UInt32, Ptr{Float64}, Ptr{Float64}),
                gws.handle, UInt32(pidx), m, cov), gws.handle, "emcmc_get_adaptation_moments")
    permutedims(m), cov
end

"""
    faults(gws) -> Vector{UInt32}

Per-chain fault bits: 1 non-finite proposal log-likelihood, 2 RNG retry cap,
4 Haario readjust not positive definite.
"""
function faults(gws::MI355XGlobalWorkspace)
    f = Vector{UInt32}(undef, gws.backend.num_chains)
    check(ccall((:emcmc_get_faults, LIB), Cint, (Ptr{Cvoid}, Ptr{UInt32}), gws.handle, f), gws.handle,
          "emcmc_get_faults")
    f
end

struct EmcmcMoments
    num_chains::UInt64
    num_draws::UInt64
    accepted::UInt64
    proposed::UInt64
end

"""
    moments_window(gws, iter_first, n; split=true) -> (moments::Matrix{Float64} (D, 3), info::EmcmcMoments)

Per-dimension moments over this shard's (split) chains of the window means and
variances: columns m̄ (mean of the chain means), M2 = Σ(m_c − m̄)² and Σ var_c,
the input of split-R̂.  Shards combine by Chan's pairwise merge of (count, m̄, M2)
after an all-gather (extensible_mcmc/diagnostics.py).
"""
function moments_window(gws::MI355XGlobalWorkspace, iter_first::Integer, n::Integer; split::Bool=true)
    out = Matrix{Float64}(undef, gws.dim, 3)
    info = Ref{EmcmcMoments}()
    check(ccall((:emcmc_moments_window, LIB), Cint, (Ptr{Cvoid}, UInt64, UInt64, Cint, Ptr{Float64}, Ref{EmcmcMoments}),
                gws.handle, iter_first, n, Cint(split), out, info), gws.handle, "emcmc_moments_window")
    out, info[]
end

# ---- cross-chain diagnostics over every rank (emcmc_comm_*, emcmc_diagnostics) ------------
# One handle per GPU holds a shard of the chains; an HipComm joins the ranks of a job.
# `HipComm(nranks, rank, device, id)` is RCCL over xGMI (rank 0 draws `rccl_unique_id()`,
# the caller broadcasts the 128 bytes, e.g. MPI.Bcast!); `HipComm(nranks, rank, allgather!)`
# wraps the caller's own all-gather of Float64 vectors (e.g. MPI.Allgather!), called by
# the library through a @cfunction.  `diagnostics(gws, comm, iter_first, n)` all-gathers
# the shards' moments and merges them in rank order (Chan), then split-R̂ — the same bits
# on every rank and in extensible_mcmc/diagnostics.py.

struct EmcmcDiag
    num_chains::UInt64
    num_draws::UInt64
    accepted::UInt64
    proposed::UInt64
    accept_rate::Float64
    max_rhat::Float64
    dim::UInt32
    nranks::UInt32
    mean::Ptr{Float64}
    m2::Ptr{Float64}
    sum_var::Ptr{Float64}
    W::Ptr{Float64}
    B::Ptr{Float64}
    rhat::Ptr{Float64}
end

mutable struct HipComm
    ptr::Ptr{Cvoid}
    allgather!::Any   # the host form's Julia all-gather (kept alive with the comm), else nothing
    err::Any          # an exception the all-gather raised (a Julia exception cannot cross the C ABI)
end

function rccl_unique_id()
    id = Vector{UInt8}(undef, 128)
    check(ccall((:emcmc_comm_unique_id, LIB), Cint, (Ptr{UInt8},), id), C_NULL, "emcmc_comm_unique_id")
    id
end

function _comm_check(st, c::HipComm, where)
    if c.err !== nothing
        e, c.err = c.err, nothing
        throw(e)
    end
    st == 0 && return nothing
    error("$where failed with emcmc_status $st: " *
          unsafe_string(ccall((:emcmc_comm_last_error, LIB), Cstring, (Ptr{Cvoid},), c.ptr)))
end

function HipComm(nranks::Integer, rank::Integer, device::Integer, id::AbstractVector{UInt8})
    length(id) == 128 || throw(ArgumentError("an RCCL unique id has 128 bytes"))
    p = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:emcmc_comm_init, LIB), Cint, (Ref{Ptr{Cvoid}}, Cint, Cint, Cint, Ptr{UInt8}),
                p, nranks, rank, device, Vector{UInt8}(id)), C_NULL, "emcmc_comm_init")
    c = HipComm(p[], nothing, nothing)
    finalizer(c -> (c.ptr != C_NULL && ccall((:emcmc_comm_destroy, LIB), Cvoid, (Ptr{Cvoid},), c.ptr);
                    c.ptr = C_NULL), c)
end

# emcmc_allgather_fn: ctx is the HipComm; recv gets nranks·count doubles in rank order
function _allgather_trampoline(send::Ptr{Float64}, recv::Ptr{Float64}, count::UInt64, ctx::Ptr{Cvoid})::Cint
    c = unsafe_pointer_to_objref(ctx)::HipComm
    try
        s = copy(unsafe_wrap(Array, send, Int(count)))
        r = c.allgather!(s)
        dst = unsafe_wrap(Array, recv, length(r))
        dst .= r
        return Cint(0)
    catch e
        c.err = e
        return Cint(1)
    end
end

"""
    HipComm(nranks, rank, allgather!)

A host communicator: `allgather!(send::Vector{Float64}) -> Vector{Float64}` returns every
rank's `send`, concatenated in rank order (e.g. `MPI.Allgather(send, comm)`).
"""
function HipComm(nranks::Integer, rank::Integer, allgather!::Function)
    c = HipComm(C_NULL, allgather!, nothing)
    p = Ref{Ptr{Cvoid}}(C_NULL)
    fp = @cfunction(_allgather_trampoline, Cint, (Ptr{Float64}, Ptr{Float64}, UInt64, Ptr{Cvoid}))
    check(ccall((:emcmc_comm_init_host, LIB), Cint, (Ref{Ptr{Cvoid}}, Cint, Cint, Ptr{Cvoid}, Ptr{Cvoid}),
                p, nranks, rank, fp, pointer_from_objref(c)), C_NULL, "emcmc_comm_init_host")
    c.ptr = p[]
    finalizer(c -> (c.ptr != C_NULL && ccall((:emcmc_comm_destroy, LIB), Cvoid, (Ptr{Cvoid},), c.ptr);
                    c.ptr = C_NULL), c)
end

"""
    diagnostics(gws, comm, iter_first, n; split=true) -> NamedTuple

Cross-chain diagnostics of θ over iterations iter_first … iter_first+n−1 over every rank
of `comm` (`nothing`: this shard alone): `rhat` (split-R̂ per coordinate), `mean`, `W`,
`B`, `m2`, `sum_var`, `max_rhat`, `accept_rate`, `num_chains`, `num_draws`.  Collective.
"""
function diagnostics(gws::MI355XGlobalWorkspace, comm::Union{HipComm,Nothing}, iter_first::Integer, n::Integer;
                     split::Bool=true)
    D = gws.dim
    a = [Vector{Float64}(undef, D) for _ in 1:6]
    d = Ref(EmcmcDiag(0, 0, 0, 0, 0.0, 0.0, 0, 0, pointer(a[1]), pointer(a[2]), pointer(a[3]), pointer(a[4]),
                      pointer(a[5]), pointer(a[6])))
    cp = comm === nothing ? C_NULL : comm.ptr
    st = GC.@preserve a comm ccall((:emcmc_diagnostics, LIB), Cint,
                                   (Ptr{Cvoid}, Ptr{Cvoid}, UInt64, UInt64, Cint, Ref{EmcmcDiag}),
                                   gws.handle, cp, iter_first, n, Cint(split), d)
    comm === nothing || comm.err === nothing || _comm_check(st, comm, "emcmc_diagnostics")
    check(st, gws.handle, "emcmc_diagnostics")
    r = d[]
    (rhat=a[6], mean=a[1], W=a[4], B=a[5], m2=a[2], sum_var=a[3], max_rhat=r.max_rhat, accept_rate=r.accept_rate,
     num_chains=Int(r.num_chains), num_draws=Int(r.num_draws), accepted=Int(r.accepted), proposed=Int(r.proposed),
     nranks=Int(r.nranks))
end

"""
    kernel_name(gws) -> String

The device kernel variant `__run!` dispatches to.
"""
function kernel_name(gws::MI355XGlobalWorkspace)
    buf = Vector{UInt8}(undef, 256)
    check(ccall((:emcmc_kernel_name, LIB), Cint, (Ptr{Cvoid}, Ptr{UInt8}, Csize_t), gws.handle, buf, length(buf)),
          gws.handle, "emcmc_kernel_name")
    unsafe_string(pointer(buf))
end

function device_count()
    n = Ref{Cint}(0)
    check(ccall((:emcmc_device_count, LIB), Cint, (Ref{Cint},), n), C_NULL, "emcmc_device_count")
    Int(n[])
end


# ---- the reference's workspace accessors, for its own callbacks -----------------
# SavingCallback reads ws.sub_ws.state_history[i][j], ws.sub_ws.state_proposal_history[i][j],
# local_wss[j].sub_ws.ll_history[i], local_wss[j].sub_ws°.ll_history[i] and
# local_wss[j].acceptance_history[i] (callbacks.jl:246-256); REPLCallback calls
# summary(ws), name_of_update, ll, ll°, llr, accepted, state and state° (callbacks.jl:
# 276-319, workspaces.jl:244-385).  With many chains these observe one chain,
# MI355XBackend.callback_chain, through lazy views that copy single slots from the
# device (emcmc_get_history_chains, emcmc_get_proposal_ll).

_cbchain(gws::MI355XGlobalWorkspace) = gws.backend.callback_chain

# θ of the callback chain at (iter, pidx) from history `which` (EMCMC_H_STATE / H_PROPOSAL)
function _hist_slot(gws::MI355XGlobalWorkspace, which, iter::Integer, pidx::Integer)
    out = Array{Float64}(undef, gws.dim, 1, gws.num_updates)        # [1][P][1][D] row-major
    check(ccall((:emcmc_get_history_chains, LIB), Cint,
                (Ptr{Cvoid}, UInt32, UInt64, UInt64, UInt64, UInt64, Ptr{Cvoid}, Csize_t),
                gws.handle, which, iter, 1, _cbchain(gws) - 1, 1, out, sizeof(out)),
          gws.handle, "emcmc_get_history_chains")
    out[:, 1, pidx]
end
function _ll_slot(gws::MI355XGlobalWorkspace, iter::Integer, pidx::Integer)
    out = Array{Float64}(undef, 1, gws.num_updates)
    check(ccall((:emcmc_get_history_chains, LIB), Cint,
                (Ptr{Cvoid}, UInt32, UInt64, UInt64, UInt64, UInt64, Ptr{Cvoid}, Csize_t),
                gws.handle, H_LL, iter, 1, _cbchain(gws) - 1, 1, out, sizeof(out)),
          gws.handle, "emcmc_get_history_chains")
    out[1, pidx]
end

"`state_history` / `state_proposal_history` of the callback chain: h[i][j] is a Vector (workspaces.jl:157-160)."
struct HistoryView{T}
    gws::MI355XGlobalWorkspace{T}
    which::UInt32
end
struct HistoryRow{T}
    gws::MI355XGlobalWorkspace{T}
    which::UInt32
    iter::Int
end
Base.getindex(h::HistoryView, i::Integer) = HistoryRow(h.gws, h.which, Int(i))
Base.length(h::HistoryView) = h.gws.num_mcmc_steps
Base.getindex(r::HistoryRow, j::Integer) = _hist_slot(r.gws, r.which, r.iter, j)
Base.length(r::HistoryRow) = r.gws.num_updates
Base.iterate(r::HistoryRow, j=1) = j > length(r) ? nothing : (r[j], j + 1)

"The global sub-workspace view: ws.sub_ws.state, .state_history, .state_proposal_history."
struct GlobalSubView{T}
    gws::MI355XGlobalWorkspace{T}
end
function Base.getproperty(v::GlobalSubView, s::Symbol)
    gws = getfield(v, :gws)
    s === :state && return _chain_state(gws)
    s === :state_history && return HistoryView(gws, H_STATE)
    s === :state_proposal_history && return HistoryView(gws, H_PROPOSAL)
    s === :gws && return gws
    error("MI355X global sub-workspace has no field $s")
end

function Base.getproperty(gws::MI355XGlobalWorkspace, s::Symbol)
    s === :sub_ws && return GlobalSubView(gws)
    getfield(gws, s)
end

# θ of the callback chain, now
_chain_state(gws::MI355XGlobalWorkspace) = eMCMC.state(gws)[_cbchain(gws), :]

"ll_history views: sub_ws.ll_history[i] = [ll] of (i, pidx); sub_ws°.ll_history[i] stays zeros (never written, run.jl:333)."
struct LLHistoryView{T}
    lws::MI355XLocalWorkspace{T}
    proposal::Bool
end
Base.getindex(h::LLHistoryView, i::Integer) =
    h.proposal ? zeros(Float64, 1) : [_ll_slot(h.lws.gws, i, h.lws.pidx)]
Base.length(h::LLHistoryView) = h.lws.gws.num_mcmc_steps

struct LocalSubView{T}
    lws::MI355XLocalWorkspace{T}
    proposal::Bool
end
function Base.getproperty(v::LocalSubView, s::Symbol)
    lws, prop = getfield(v, :lws), getfield(v, :proposal)
    s === :ll && return prop ? [_proposal_ll(lws)] : [_current_ll(lws)]
    s === :ll_history && return LLHistoryView(lws, prop)
    s === :state && return prop ? _proposal_state(lws) : _chain_state(lws.gws)[lws.gws.coords[lws.pidx]]
    error("MI355X local sub-workspace has no field $s")
end

struct AcceptanceView{T}
    lws::MI355XLocalWorkspace{T}
end
function Base.getindex(a::AcceptanceView, i::Integer)
    gws, c = a.lws.gws, _cbchain(a.lws.gws)
    words = _history(gws, H_ACCEPT, Array{UInt64}(undef, cld(gws.backend.num_chains, 64), gws.num_updates, 1), i, 1)
    ((words[(c - 1) >> 6 + 1, a.lws.pidx, 1] >> ((c - 1) & 63)) & 1) == 1
end
Base.length(a::AcceptanceView) = a.lws.gws.num_mcmc_steps

function Base.getproperty(lws::MI355XLocalWorkspace, s::Symbol)
    s === :sub_ws && return LocalSubView(lws, false)
    s === :sub_ws° && return LocalSubView(lws, true)
    s === :acceptance_history && return AcceptanceView(lws)
    s === :updt_name && return getfield(lws, :gws).names[getfield(lws, :pidx)]
    getfield(lws, s)
end

function _current_ll(lws::MI355XLocalWorkspace)
    ll = Vector{Float64}(undef, lws.gws.backend.num_chains)
    check(ccall((:emcmc_get_state, LIB), Cint, (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}), lws.gws.handle, C_NULL, ll),
          lws.gws.handle, "emcmc_get_state")
    ll[_cbchain(lws.gws)]
end
function _proposal_ll(lws::MI355XLocalWorkspace)
    gws = lws.gws
    out = Matrix{Float64}(undef, gws.backend.num_chains, gws.num_updates)     # [P][C] row-major
    check(ccall((:emcmc_get_proposal_ll, LIB), Cint, (Ptr{Cvoid}, Ptr{Float64}), gws.handle, out),
          gws.handle, "emcmc_get_proposal_ll")
    out[_cbchain(gws), lws.pidx]
end
# sub_ws°.state: θ° of the update's latest proposal (its coordinates of the proposal history slot)
function _proposal_state(lws::MI355XLocalWorkspace)
    gws = lws.gws
    it = gws.last_iter[lws.pidx]
    it == 0 && return gws.θinit[gws.coords[lws.pidx]]
    _hist_slot(gws, H_PROPOSAL, it, lws.pidx)[gws.coords[lws.pidx]]
end

# workspaces.jl:91-136, 294-385 for this backend
eMCMC.num_mcmc_steps(gws::MI355XGlobalWorkspace) = gws.num_mcmc_steps
eMCMC.num_updt(gws::MI355XGlobalWorkspace) = gws.num_updates
eMCMC.state(gws::MI355XGlobalWorkspace, step) = _hist_slot(gws, H_STATE, step.mcmciter, step.pidx)
eMCMC.state°(gws::MI355XGlobalWorkspace, step) = _hist_slot(gws, H_PROPOSAL, step.mcmciter, step.pidx)
function eMCMC.estim_mean(gws::MI355XGlobalWorkspace)
    gws.backend.chain_moments || error("estim_mean needs MI355XBackend(chain_moments=true)")
    chain_moments(gws)[1][_cbchain(gws), :]
end
function eMCMC.estim_cov(gws::MI355XGlobalWorkspace)
    gws.backend.chain_moments || error("estim_cov needs MI355XBackend(chain_moments=true)")
    chain_moments(gws)[2][:, :, _cbchain(gws)]
end
eMCMC.accepted(lws::MI355XLocalWorkspace, i::Int) = lws.acceptance_history[i]
eMCMC.ll(lws::MI355XLocalWorkspace) = lws.sub_ws.ll
eMCMC.ll°(lws::MI355XLocalWorkspace) = lws.sub_ws°.ll
eMCMC.ll(lws::MI355XLocalWorkspace, i::Int) = lws.sub_ws.ll_history[i]
eMCMC.ll°(lws::MI355XLocalWorkspace, i::Int) = lws.sub_ws°.ll      # workspaces.jl:337 reads the current ll°
eMCMC.state(lws::MI355XLocalWorkspace) = lws.sub_ws.state
eMCMC.state°(lws::MI355XLocalWorkspace) = lws.sub_ws°.state
eMCMC.name_of_update(lws::MI355XLocalWorkspace) = lws.updt_name

export MI355XBackend, state_history, proposal_history, ll_history, acceptance_history, rolling_acceptance,
       adaptation_state, chain_moments, adaptation_moments, mix_state, faults, moments_window, kernel_name, device_count,
       HipComm, rccl_unique_id, diagnostics, HipTargetLaw, HipUpdate, HipMALAUpdate

end # module
