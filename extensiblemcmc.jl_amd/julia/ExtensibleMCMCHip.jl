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
const eMCMC = ExtensibleMCMC

const LIB = get(ENV, "EMCMC_LIB", joinpath(@__DIR__, "..", "lib", "libemcmc.so"))
const ABI_VERSION = UInt32(1)

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
    reserved_ptr::NTuple{2,Ptr{Cvoid}}
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
end

struct EmcmcStep
    mcmciter::UInt32
    pidx::UInt32
end

const RW_GAUSSIAN = UInt32(2)
const RW_GAUSSIAN_MIX = UInt32(3)
const ADPT_HAARIO = UInt32(2)
const PRIOR_IMPROPER = UInt32(0)
const ADPT_NONE = UInt32(0)
const TARGET_GSN = UInt32(1)
const H_STATE, H_PROPOSAL, H_LL, H_ACCEPT = UInt32(0), UInt32(1), UInt32(2), UInt32(3)

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
end

mutable struct MI355XGlobalWorkspace{T} <: eMCMC.GlobalWorkspace{T}
    handle::Ptr{Cvoid}
    backend::MI355XBackend
    num_mcmc_steps::Int
    dim::Int
    num_updates::Int
    num_locals::Int
    num_coords::Vector{Int}   # per update: length(updt.coords)
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

const RW_UNIFORM = UInt32(1)
const ADPT_UNIF_RW = UInt32(1)

function _update_desc(updt::eMCMC.RandomWalkUpdate, keep)
    updt.prior isa eMCMC.ImproperPrior || error("no device plugin for $(typeof(updt.prior))")
    coords = UInt32.(collect(updt.coords) .- 1)                 # 0-based across the ABI
    push!(keep, coords)
    adpt, adptp = ADPT_NONE, C_NULL
    if updt.rw isa eMCMC.GaussianRandomWalk
        updt.adpt isa eMCMC.NoAdaptation || error("no device plugin for $(typeof(updt.adpt)) with GaussianRandomWalk")
        Σ = Matrix{Float64}(updt.rw.Σ)                         # column-major already
        pos = UInt8.(updt.rw.pos)                               # log-scale coordinates (random_walk.jl:136-171)
        push!(keep, Σ, pos)
        return EmcmcUpdateDesc(RW_GAUSSIAN, PRIOR_IMPROPER, ADPT_NONE, UInt32(length(coords)), pointer(coords),
                               pointer(Σ), C_NULL, pointer(pos), C_NULL, C_NULL, (C_NULL, C_NULL), 0.0,
                               (0.0, 0.0, 0.0))
    elseif updt.rw isa eMCMC.GaussianRandomWalkMix                # random_walk.jl:193-232
        (any(updt.rw.gsn_A.pos) || any(updt.rw.gsn_B.pos)) &&
            error("positivity-restricted coordinates are not on device yet")
        ΣA = Matrix{Float64}(updt.rw.gsn_A.Σ)
        ΣB = Matrix{Float64}(updt.rw.gsn_B.Σ)
        push!(keep, ΣA, ΣB)
        if updt.adpt isa eMCMC.HaarioTypeAdaptation              # adaptation.jl:372-426 (fλ must be identity)
            p = Ref(EmcmcHaarioAdaptation(UInt32(updt.adpt.adapt_every_k_steps), UInt32(0), updt.adpt.scale))
            push!(keep, p)
            adpt, adptp = ADPT_HAARIO, Base.unsafe_convert(Ptr{Cvoid}, p)
        elseif !(updt.adpt isa eMCMC.NoAdaptation)
            error("no device plugin for $(typeof(updt.adpt)) with GaussianRandomWalkMix")
        end
        return EmcmcUpdateDesc(RW_GAUSSIAN_MIX, PRIOR_IMPROPER, adpt, UInt32(length(coords)), pointer(coords),
                               pointer(ΣA), C_NULL, C_NULL, adptp, pointer(ΣB), (C_NULL, C_NULL), updt.rw.λ,
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
        elseif !(updt.adpt isa eMCMC.NoAdaptation)
            error("no device plugin for $(typeof(updt.adpt))")
        end
        return EmcmcUpdateDesc(RW_UNIFORM, PRIOR_IMPROPER, adpt, UInt32(length(coords)), pointer(coords), C_NULL,
                               pointer(ϵ), pointer(pos), adptp, C_NULL, (C_NULL, C_NULL), 0.0, (0.0, 0.0, 0.0))
    end
    error("no device plugin for $(typeof(updt.rw))")
end

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
        for u in updates
            desc = Ref(_update_desc(u, keep))
            check(ccall((:emcmc_add_update, LIB), Cint, (Ptr{Cvoid}, Ref{EmcmcUpdateDesc}), h[], desc),
                  h[], "emcmc_add_update")
        end
    end
    P = data.P
    d = length(P.θ) == 0 ? 0 : Int(round((sqrt(1 + 4length(P.θ)) - 1) / 2))  # θ = [μ; vec Σ]
    μ = P.θ[1:d]
    Σ = reshape(P.θ[(d+1):end], d, d)
    X = reduce(vcat, permutedims.(data.obs))                     # n×d
    Xrm = permutedims(X)                                           # row-major view for the ABI
    GC.@preserve μ Σ Xrm begin
        t = Ref(EmcmcTargetDesc(TARGET_GSN, UInt32(d), pointer(μ), pointer(Σ), UInt64(size(X, 1)),
                                pointer(Xrm), be.ll_mode === :per_obs ? UInt32(0) : UInt32(1), UInt32(0)))
        check(ccall((:emcmc_set_target, LIB), Cint, (Ptr{Cvoid}, Ref{EmcmcTargetDesc}), h[], t),
              h[], "emcmc_set_target")
    end
    θ0 = repeat(Float64.(θinit), be.num_chains)                     # [C][D] row-major
    check(ccall((:emcmc_set_state, LIB), Cint, (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}), h[], θ0, C_NULL),
          h[], "emcmc_set_state")
    ws = MI355XGlobalWorkspace{T}(h[], be, num_mcmc_steps, D, length(updates), 0,
                                  [length(u.coords) for u in updates])
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
        if wants(step, post)
            flush!()
            eMCMC.update_callbacks!(callbacks, gws, local_wss, step, post)
        end
    end
    flush!()
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
    C, D = gws.backend.num_chains, gws.dim
    L = Array{Float64}(undef, D, D, C)     # [C][D][D] row-major, transposed below
    M = Ref{UInt32}(0)                     # the same for every chain
    check(ccall((:emcmc_get_mix_state, LIB), Cint, (Ptr{Cvoid}, UInt32, Ptr{Float64}, Ref{UInt32}),
                gws.handle, UInt32(pidx), L, M), gws.handle, "emcmc_get_mix_state")
    permutedims(L, (2, 1, 3)), Int(M[])
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
    moments_window(gws, iter_first, n; split=true) -> (sums::Matrix{Float64} (D, 3), info::EmcmcMoments)

Per-dimension sums over this shard's (split) chains of the window means, squared
means and variances: the input of split-R̂.  Shards combine by summation
(MPI/RCCL all-reduce across processes).
"""
function moments_window(gws::MI355XGlobalWorkspace, iter_first::Integer, n::Integer; split::Bool=true)
    out = Matrix{Float64}(undef, gws.dim, 3)
    info = Ref{EmcmcMoments}()
    check(ccall((:emcmc_moments_window, LIB), Cint, (Ptr{Cvoid}, UInt64, UInt64, Cint, Ptr{Float64}, Ref{EmcmcMoments}),
                gws.handle, iter_first, n, Cint(split), out, info), gws.handle, "emcmc_moments_window")
    out, info[]
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

export MI355XBackend, state_history, proposal_history, ll_history, acceptance_history, rolling_acceptance,
       adaptation_state, chain_moments, mix_state, faults, moments_window, kernel_name, device_count

end # module
