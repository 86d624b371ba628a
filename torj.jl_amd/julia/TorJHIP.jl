# TorJHIP.jl -- drop-in GPU back end for TorJ.jl's ray-tracing path (make_ray /
# make_beam, src/solve.jl) on AMD MI355X, through the C ABI of libtorj_hip.so
# (include/torj_hip.h).  Kept deliberately thin: argument marshalling only.
#
# Usage (see INTEGRATION.md):
#     using TorJ, TorJHIP
#     TorJHIP.abs_Al_init(24)
#     plasma = TorJ.Plasma(R, Z, psi_norm, psi_prof, ne, Te, Br, Bz, Bphi, eq_psi, eq_vol)
#     s, u, P, dP_dV, P_dep = TorJHIP.make_ray(plasma, x0, N0, f, 1, 0.4, psi_dP_dV)
#     out = TorJHIP.make_beam(plasma, r, phi, z, tor, pol, spot, inv_curv, f, 1, 1.0,
#                             psi_dP_dV; N_rings=92, min_azimuthal_points=11, n_gpus=8)
# A TorJ.Plasma is converted once (GPUPlasma(plasma): its Interpolations.jl
# B-spline coefficients go to the GPU as they are) and cached per object.
#
# Untested in this repository's container (no Julia toolchain); the same ABI is
# exercised by the Python ctypes mirror in torj.jl_amd/torj_hip.
module TorJHIP

import TorJ

const libtorj = get(ENV, "TORJ_HIP_LIB", joinpath(@__DIR__, "..", "build", "libtorj_hip.so"))
const ABI_VERSION = 8  # include/torj_hip.h TORJ_ABI_VERSION

function __init__()
    v = ccall((:torj_abi_version, libtorj), Cint, ())
    v == ABI_VERSION || error("libtorj_hip.so at $libtorj has ABI version $v, TorJHIP expects $ABI_VERSION")
end

struct TraceCfg              # torj_trace_cfg
    omega::Float64
    mode::Cint
    ds::Float64
    n_steps::Cint
    chunk_steps::Cint
    psi_exit::Float64
    P_min::Float64
    absorption::Cint         # 0 none, 1 abs_Albajar_fast, 2 / 3 warm alpha (iwarm 1 / 3)
    traj_stride::Cint
    deposition::Cint         # 0: binned, 1: power_deposition_profile (src/plasma.jl:91-151)
    integrator::Cint         # 0: fixed RK4; 1: the reference's adaptive solve() (Tsit5)
    abstol::Float64
    reltol::Float64
    s_max::Float64
    n_chunks::Cint
end

check(rc) = rc == 0 || error(unsafe_string(ccall((:torj_last_error, libtorj), Cstring, ())))

"""abs_Al_init(N) -- src/absorption.jl:1-7"""
abs_Al_init(n::Integer) = check(ccall((:torj_abs_al_init, libtorj), Cint, (Cint,), n))

mutable struct GPUPlasma
    h::Ptr{Cvoid}
    psi_prof_max::Float64
    function GPUPlasma(h::Ptr{Cvoid}, psi_prof_max::Float64)
        p = new(h, psi_prof_max)
        finalizer(x -> ccall((:torj_plasma_destroy, libtorj), Cint, (Ptr{Cvoid},), x.h), p)
        return p
    end
end

"""GPUPlasma from the raw maps -- the arguments of TorJ.Plasma (src/plasma.jl:30-32);
the B-spline prefilter runs in the library."""
function GPUPlasma(R::Vector{Float64}, Z::Vector{Float64}, psi_norm::Matrix{Float64},
                   psi_prof::Vector{Float64}, ne::Vector{Float64}, Te::Vector{Float64},
                   Br::Matrix{Float64}, Bz::Matrix{Float64}, Bphi::Matrix{Float64},
                   eq_psi::Vector{Float64}, eq_vol::Vector{Float64}; device::Integer=0)
    h = Ref{Ptr{Cvoid}}(C_NULL)
    # Julia matrices are (nR, nZ) column-major: exactly the ABI layout
    check(ccall((:torj_plasma_create, libtorj), Cint,
                (Cint, Cint, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Cint, Ptr{Float64},
                 Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Cint,
                 Ptr{Float64}, Ptr{Float64}, Cint, Ptr{Ptr{Cvoid}}),
                length(R), length(Z), R, Z, psi_norm, length(psi_prof), psi_prof, ne, Te,
                Br, Bz, Bphi, length(eq_psi), eq_psi, eq_vol, device, h))
    return GPUPlasma(h[], maximum(psi_prof))
end

# Interpolations.jl: cubic_spline_interpolation(ranges, A; extrapolation_bc=Line())
# is extrapolate(scale(interpolate(A, BSpline(Cubic(Line(OnGrid())))), ranges...), Line());
# .itp is the ScaledInterpolation (its .ranges), .itp.itp the BSplineInterpolation
# whose padded coefficient OffsetArray has parent (n+2) x (m+2).
_coefs(spl) = Array{Float64}(parent(spl.itp.itp.coefs))
_ranges(spl) = spl.itp.ranges

"""GPUPlasma(plasma::TorJ.Plasma) -- the TorJ object itself (src/plasma.jl:2-14): its six
2-D splines' coefficients (psi, ln ne, ln Te, Br, Bz, Bphi) and the 1-D volume spline
go to the GPU unchanged (torj_plasma_create_from_coefs), so the GPU evaluates exactly
the splines TorJ built."""
function GPUPlasma(p::TorJ.Plasma; device::Integer=0)
    rR, rZ = _ranges(p.psi_norm_spline)
    c = [_coefs(getfield(p, f)) for f in (:psi_norm_spline, :ne_spline, :Te_spline,
                                           :Br_spline, :Bz_spline, :Bϕ_spline)]
    all(size(x) == (length(rR) + 2, length(rZ) + 2) for x in c) ||
        throw(ArgumentError("TorJ.Plasma splines are not on one (R, Z) grid"))
    rv = _ranges(p.volume_psi_spline)[1]
    cv = _coefs(p.volume_psi_spline)
    h = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:torj_plasma_create_from_coefs, libtorj), Cint,
                (Cint, Cint, Float64, Float64, Float64, Float64, Ptr{Float64}, Ptr{Float64},
                 Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Cint, Float64, Float64,
                 Ptr{Float64}, Float64, Cint, Ptr{Ptr{Cvoid}}),
                length(rR), length(rZ), first(rR), last(rR), first(rZ), last(rZ), c[1], c[2],
                c[3], c[4], c[5], c[6], length(rv), first(rv), last(rv), cv,
                Float64(p.psi_prof_max), device, h))
    return GPUPlasma(h[], Float64(p.psi_prof_max))
end

# one GPU copy per TorJ.Plasma object (make_ray / make_beam on TorJ's own type)
const _gpu_cache = IdDict{Any,GPUPlasma}()
const _gpu_lock = ReentrantLock()
gpu_plasma(p::TorJ.Plasma) = lock(() -> get!(() -> GPUPlasma(p), _gpu_cache, p), _gpu_lock)

"""first_point + vacuum_plasma_refraction for n rays (x0, N0: n x 3), on the GPU."""
function ray_entry(p::GPUPlasma, x0::Matrix{Float64}, N0::Matrix{Float64}, omega, mode)
    n = size(x0, 1)
    xp, Np, s0, st = zeros(n, 3), zeros(n, 3), zeros(n), zeros(Cint, n)
    check(ccall((:torj_ray_entry_gpu, libtorj), Cint,
                (Ptr{Cvoid}, Cint, Ptr{Float64}, Ptr{Float64}, Float64, Cint, Ptr{Float64},
                 Ptr{Float64}, Ptr{Float64}, Ptr{Cint}),
                p.h, n, x0, N0, omega, mode, xp, Np, s0, st))
    return xp, Np, s0, st
end

function trace(p::GPUPlasma, cfg::TraceCfg, x0::Matrix{Float64}, N0::Matrix{Float64},
               w::Vector{Float64}, psi_grid::Vector{Float64}, x_launch::Matrix{Float64},
               s0::Vector{Float64}; n_gpus::Integer=1, n_shards::Integer=0)
    n = size(x0, 1)
    n_save = cfg.traj_stride > 0 ? cfg.n_steps ÷ cfg.traj_stride : 0
    state, status, steps = zeros(n, 7), zeros(Cint, n), zeros(Cint, n)
    dP, Pdep = zeros(length(psi_grid) + 1), zeros(n)
    traj = n_save > 0 ? zeros(n, 5, n_save) : zeros(0, 5, 0)
    GC.@preserve x0 N0 w psi_grid x_launch s0 begin
        # make_beam's fan-out over n_gpus devices + the RCCL reduce of dP_shell
        check(ccall((:torj_trace_beam, libtorj), Cint,
                    (Ptr{Cvoid}, Ref{TraceCfg}, Cint, Ptr{Float64}, Ptr{Float64}, Ptr{Float64},
                     Cint, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Cint},
                     Ptr{Cint}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Cint, Cint),
                    p.h, cfg, n, x0, N0, w, length(psi_grid), psi_grid, x_launch, s0, state,
                    status, steps, dP, Pdep, n_save > 0 ? traj : C_NULL, n_gpus, n_shards))
    end
    return state, status, steps, dP, Pdep, traj
end

# who took part in the last make_beam reduce over n_gpus replicas (ABI 8): each
# replica's HIP device and its RCCL communicator's rank count and rank (0 / -1
# where no communicator exists)
function beam_comm_info(p::GPUPlasma, n_gpus::Integer)
    dev, nranks, rank = zeros(Cint, n_gpus), zeros(Cint, n_gpus), zeros(Cint, n_gpus)
    check(ccall((:torj_beam_comm_info, libtorj), Cint,
                (Ptr{Cvoid}, Cint, Ptr{Cint}, Ptr{Cint}, Ptr{Cint}), p.h, n_gpus, dev, nranks, rank))
    return (device=dev, rccl_nranks=nranks, rccl_rank=rank)
end

function shell_volumes(p::GPUPlasma, g::Vector{Float64})
    dV = zeros(length(g) - 1)
    check(ccall((:torj_shell_volumes, libtorj), Cint, (Ptr{Cvoid}, Cint, Ptr{Float64}, Ptr{Float64}),
                p.h, length(g), g, dV))
    return dV
end

"""power_deposition_profile -- same signature and return tuple as
TorJ.power_deposition_profile (src/plasma.jl:91-151), on the GPU: psi at x from the
plasma's spline, the not-a-knot fits, Dierckx.roots (maxn = 8) pairing and the
outside-in walk.  Returns (dP_dV, P)."""
function power_deposition_profile(p::GPUPlasma, s::Vector{Float64}, x::Vector{Vector{Float64}},
                                  dP_ds::Vector{Float64}, psi_dP_dV::Vector{Float64})
    n = length(s)
    (length(x) == n && length(dP_ds) == n) || throw(DimensionMismatch("s, x, dP_ds lengths differ"))
    xm = Matrix{Float64}(undef, n, 3)  # n x 3 column-major = the ABI's component-major 3 x n
    for i in 1:n, c in 1:3
        xm[i, c] = x[i][c]
    end
    dP_dV, P = zeros(length(psi_dP_dV)), zeros(1)
    np = Cint[n]
    check(ccall((:torj_power_deposition_profile, libtorj), Cint,
                (Ptr{Cvoid}, Cint, Ptr{Cint}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Cint,
                 Ptr{Float64}, Ptr{Float64}, Ptr{Float64}),
                p.h, 1, np, s, xm, dP_ds, length(psi_dP_dV), psi_dP_dV, dP_dV, P))
    return dP_dV, P[1]
end
power_deposition_profile(p::TorJ.Plasma, args...) = power_deposition_profile(gpu_plasma(p), args...)

"""make_ray -- same signature and return tuple as TorJ.make_ray (src/solve.jl:135-181)."""
function make_ray(p::GPUPlasma, x0::AbstractVector, N_vacuum::AbstractVector, f::Real,
                  mode::Integer, s_max::Float64, psi_dP_dV::AbstractVector; ds::Float64=1e-4,
                  deposition::Integer=1, integrator::Integer=0, absorption::Integer=1)
    ω = 2π * f
    xp, Np, s0, st = ray_entry(p, reshape(collect(Float64, x0), 1, 3),
                               reshape(collect(Float64, N_vacuum), 1, 3), ω, mode)
    st[1] == 0 || throw(AssertionError("ray entry failed (status $(st[1]))"))
    n_steps = max(1, round(Int, s_max / ds))
    cap = integrator == 1 ? 2n_steps + 400 : n_steps
    cfg = TraceCfg(ω, mode, ds, cap, max(1, n_steps ÷ 100), 1.0, 1e-6, absorption, 1, deposition,
                   integrator, 1e-6, 1e-6, s_max, 100)
    g = collect(Float64, psi_dP_dV)
    xl = reshape(collect(Float64, x0), 1, 3)
    state, status, steps, dP, Pdep, traj = trace(p, cfg, xp, Np, ones(1), g, xl, s0)
    k = steps[1]
    s = vcat(0.0, s0[1], traj[1, 5, 1:k])
    u = vcat([collect(Float64, x0)], [xp[1, :]], [traj[1, 1:3, i] for i in 1:k])
    P_beam = vcat(1.0, 1.0, exp.(-traj[1, 4, 1:k]))
    dP_dV = zeros(length(g))
    dP_dV[1:end-1] .= dP[1:end-2] ./ shell_volumes(p, g)
    return s, u, P_beam, dP_dV, Pdep[1]
end
make_ray(p::TorJ.Plasma, args...; kw...) = make_ray(gpu_plasma(p), args...; kw...)

"""make_beam -- same signature and return tuple as TorJ.make_beam (src/solve.jl:209-242);
the launch fan and IMAS angles on the host, every ray on the GPU(s): n_gpus devices of
this process (torj_trace_beam), dP_shell summed across them by RCCL.  traj_stride keeps
every traj_stride-th step of each ray (1 = all, as the reference) plus its final state."""
function make_beam(p::GPUPlasma, r, phi, z, tor, pol, spot, inv_curv, f, mode::Integer,
                   s_max::Float64, psi_dP_dV::Vector{Float64}; ds::Float64=1e-4,
                   N_rings::Integer=3, min_azimuthal_points::Integer=5,
                   normalize_weight_sum::Bool=true, deposition::Integer=1,
                   integrator::Integer=0, absorption::Integer=1, traj_stride::Integer=1,
                   n_gpus::Integer=1)
    N0 = zeros(3)
    ccall((:torj_pol_tor_angles_2_vector, libtorj), Cvoid, (Float64, Float64, Ptr{Float64}),
          pol, tor, N0)
    x0 = [r * cos(phi), r * sin(phi), z]
    nr = Ref{Cint}(0)
    check(ccall((:torj_launch_peripheral_rays, libtorj), Cint,
                (Ptr{Float64}, Ptr{Float64}, Float64, Float64, Float64, Cint, Cint, Cint, Ref{Cint},
                 Ptr{Float64}, Ptr{Float64}, Ptr{Float64}),
                x0, N0, spot, inv_curv, f, N_rings, min_azimuthal_points, normalize_weight_sum, nr,
                C_NULL, C_NULL, C_NULL))
    n = nr[]
    pos, dirs, w = zeros(n, 3), zeros(n, 3), zeros(n)
    check(ccall((:torj_launch_peripheral_rays, libtorj), Cint,
                (Ptr{Float64}, Ptr{Float64}, Float64, Float64, Float64, Cint, Cint, Cint, Ref{Cint},
                 Ptr{Float64}, Ptr{Float64}, Ptr{Float64}),
                x0, N0, spot, inv_curv, f, N_rings, min_azimuthal_points, normalize_weight_sum, nr,
                pos, dirs, w))
    ω = 2π * f
    xp, Np, s0, st = ray_entry(p, pos, dirs, ω, mode)
    all(st .== 0) || throw(AssertionError("ray entry failed for $(count(st .!= 0)) rays"))
    n_steps = max(1, round(Int, s_max / ds))
    cap = integrator == 1 ? 2n_steps + 400 : n_steps
    traj_stride >= 1 || throw(ArgumentError("traj_stride must be >= 1"))
    # checked before tracing: the adaptive integrator's final state is no saved sample
    (integrator == 1 && traj_stride > 1) &&
        throw(ArgumentError("integrator = 1 (adaptive) needs traj_stride = 1"))
    cfg = TraceCfg(ω, mode, ds, cap, max(1, n_steps ÷ 100), 1.0, 1e-6, absorption, traj_stride,
                   deposition, integrator, 1e-6, 1e-6, s_max, 100)
    state, status, steps, dP, Pdep, traj = trace(p, cfg, xp, Np, w, psi_dP_dV, pos, s0;
                                                 n_gpus=n_gpus)
    dP_dV = zeros(length(psi_dP_dV))
    dP_dV[1:end-1] .= dP[1:end-2] ./ shell_volumes(p, psi_dP_dV)
    arc_lengths, trajectories, ray_powers = Vector{Vector{Float64}}(), Vector{Vector{Vector{Float64}}}(), Vector{Vector{Float64}}()
    for i in 1:n
        k = steps[i] ÷ traj_stride
        s_i, x_i, τ_i = traj[i, 5, 1:k], [traj[i, 1:3, j] for j in 1:k], traj[i, 4, 1:k]
        if steps[i] % traj_stride != 0  # the final state is not a saved sample
            # fma: the single-rounding s0 + steps ds the trajectory kernel stores
            push!(s_i, fma(Float64(steps[i]), ds, s0[i])); push!(x_i, state[i, 1:3]); push!(τ_i, state[i, 7])
        end
        push!(arc_lengths, vcat(0.0, s0[i], s_i))
        push!(trajectories, vcat([pos[i, :]], [xp[i, :]], x_i))
        push!(ray_powers, vcat(1.0, 1.0, exp.(-τ_i)))
    end
    return arc_lengths, trajectories, ray_powers, dP_dV, dP[end], w
end
make_beam(p::TorJ.Plasma, args...; kw...) = make_beam(gpu_plasma(p), args...; kw...)

"""alpha(...) of src/general_absorption.jl:1328-1337 (repaired, DESIGN.md §3.6) at n
points on the GPU: iwarm 1 (weakly) or 3 (fully relativistic); inv_dDdN = 1/|dD/dN|.
Returns (alpha, N_perp^2)."""
function alpha_warm(omega::Vector{Float64}, X::Vector{Float64}, Y::Vector{Float64},
                    N_abs::Vector{Float64}, N_par::Vector{Float64}, Te::Vector{Float64},
                    inv_dDdN::Vector{Float64}, mode::Integer, iwarm::Integer)
    n = length(X)
    alpha, n2 = zeros(n), zeros(2n)
    check(ccall((:torj_alpha_warm, libtorj), Cint,
                (Cint, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64},
                 Ptr{Float64}, Ptr{Float64}, Cint, Cint, Ptr{Float64}, Ptr{Float64}),
                n, omega, X, Y, N_abs, N_par, Te, inv_dDdN, mode, iwarm, alpha, n2))
    return alpha, complex.(n2[1:2:end], n2[2:2:end])
end

end # module
