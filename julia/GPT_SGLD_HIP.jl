# GPT_SGLD_HIP — drop-in replacement of the reference's `GPT_SGLD` module entry points on the
# MI355X path, via `ccall` into libgptsgld.so (include/gptsgld.h).  Julia is not on the image:
# tests/test_julia_shim.py checks every ccall against the C prototypes, and the Python binding
# gpt_amd/GPT_SGLD.py (tested on the GPU) makes the identical C calls.
#
#   kin40kExperiment.jl:  `@everywhere using GPT_SGLD`  ->  `@everywhere using GPT_SGLD_HIP`
#
# Arrays are passed zero-copy (Julia column-major == the C ABI layout); outputs are allocated here,
# exactly as the reference functions allocate and return them.
module GPT_SGLD_HIP

export datawhitening, feature, featureNotensor, samplenz, GPTregression, GPTregression_chains,
       GPT_SGLDERM, pred, RMSE,
       GPNT_SGLD, GPT_SGLDERM_RMSprop, GPT_SGLDERMw, GPTclassification, GPT_GMC, pred_mean_x,
       init_state

const LIB = get(ENV, "GPTSGLD_LIB", joinpath(@__DIR__, "..", "gpt_amd", "libgptsgld.so"))

struct SGLDConfig          # gpt_sgld_config
    n::Int64; D::Int64; N::Int64; r::Int64; Q::Int64; m::Int64
    epsw::Float64; epsU::Float64; signal_var::Float64; sigma_w::Float64
    burnin::Int64; maxepoch::Int64; seed::UInt64
    langevin::Int32; stiefel::Int32; store_every::Int64; max_steps::Int64
end

lasterr() = unsafe_string(ccall((:gpt_last_error, LIB), Cstring, ()))
check(rc) = rc == 0 ? nothing : error("gptsgld error $rc: " * lasterr())

# GPT_SGLD.jl:62-67 (host data prep, unchanged semantics)
function datawhitening(X::Array)
    X = copy(X)
    for i = 1:size(X, 2)
        X[:, i] = (X[:, i] .- sum(X[:, i]) / size(X, 1)) ./ sqrt(sum(abs2, X[:, i] .- sum(X[:, i]) / size(X, 1)) / (size(X, 1) - 1))
    end
    return X
end

# feature(X,length_scale,sigma_RBF,phi_scale,Z,b)  GPT_SGLD.jl:71
function feature(X::Array{Float64,2}, length_scale, sigma_RBF::Real, phi_scale::Real,
                 Z::Array{Float64,2}, b::Array{Float64})
    N, D = size(X); n = size(Z, 1)
    ls = collect(Float64, length_scale isa Real ? [length_scale] : length_scale)
    phi = Array{Float64}(undef, n, D, N)
    check(ccall((:gpt_feature, LIB), Cint,
                (Ptr{Float64}, Int64, Int64, Ptr{Float64}, Int64, Float64, Float64, Ptr{Float64},
                 Ptr{Float64}, Int64, Ptr{Float64}),
                X, N, D, ls, length(ls), sigma_RBF, phi_scale, Z, b, n, phi))
    return phi
end

# Generation-C seeded form used by kin40kExperiment.jl:71: feature(X,n,ls,σ,seed,scale)
function feature(X::Array{Float64,2}, n::Integer, length_scale, sigma_RBF::Real, seed::Integer,
                 scale::Real)
    D = size(X, 2)
    Z = Array{Float64}(undef, n, D); b = Array{Float64}(undef, n, D)
    check(ccall((:gpt_feature_inputs, LIB), Cint, (Int64, Int64, UInt64, Ptr{Float64}, Ptr{Float64}),
                n, D, seed, Z, b))
    return feature(X, length_scale, sigma_RBF, scale, Z, b)
end

# Generation-A seeded form feature(X,n,length_scale,seed) (GPT_SGLD_p.jl:40-54): Z = randn(n,D)
# / length_scale, b = randn(n,D), phi = sqrt(2/n)·cos(X[i,k]·Z[j,k] + b[j,k]) — no sigma_RBF, no
# scale (gpt_feature_inputs_a draws Z and b on the framework's Philox contract)
function feature(X::Array{Float64,2}, n::Integer, length_scale::Real, seed::Integer)
    D = size(X, 2)
    Z = Array{Float64}(undef, n, D); b = Array{Float64}(undef, n, D)
    check(ccall((:gpt_feature_inputs_a, LIB), Cint, (Int64, Int64, UInt64, Ptr{Float64}, Ptr{Float64}),
                n, D, seed, Z, b))
    return feature(X, 1.0, 1.0, 1.0, Z ./ length_scale, b)
end

# featureNotensor(X,length_scale,sigma_RBF,Z,b)  GPT_SGLD.jl:109
function featureNotensor(X::Array{Float64,2}, length_scale, sigma_RBF::Real, Z::Array{Float64,2},
                         b::Array{Float64})
    N, D = size(X); n = size(Z, 1)
    ls = collect(Float64, length_scale isa Real ? [length_scale] : length_scale)
    phi = Array{Float64}(undef, n, N)
    check(ccall((:gpt_feature_notensor, LIB), Cint,
                (Ptr{Float64}, Int64, Int64, Ptr{Float64}, Int64, Float64, Ptr{Float64},
                 Ptr{Float64}, Int64, Ptr{Float64}),
                X, N, D, ls, length(ls), sigma_RBF, Z, b, n, phi))
    return phi
end

# Generation-C seeded form featureNotensor(X,n,length_scale,sigma_RBF,seed), the call of
# PowerPlantNoTensorExperiment.jl:32-33, kin40kNoTensorExperiment.jl:35-36 and
# PowerPlantDataExperiment.jl:159: Z = randn(n,D), b = 2π·rand(n) drawn by gpt_feature_inputs on
# the framework's Philox contract (column 1 of its b), then the Gen-D map above
function featureNotensor(X::Array{Float64,2}, n::Integer, length_scale, sigma_RBF::Real,
                         seed::Integer)
    D = size(X, 2)
    Z = Array{Float64}(undef, n, D); b = Array{Float64}(undef, n, D)
    check(ccall((:gpt_feature_inputs, LIB), Cint, (Int64, Int64, UInt64, Ptr{Float64}, Ptr{Float64}),
                n, D, seed, Z, b))
    return featureNotensor(X, length_scale, sigma_RBF, Z, b[:, 1])
end

# samplenz(r,D,Q,seed)  GPT_SGLD_p.jl:57
function samplenz(r::Integer, D::Integer, Q::Integer, seed::Integer=0)
    I = Array{Int32}(undef, Q, D)
    check(ccall((:gpt_samplenz, LIB), Cint, (Int64, Int64, Int64, UInt64, Ptr{Int32}), r, D, Q, seed, I))
    return I
end

# GPTregression(phi,y,signal_var,I,r,Q,m,epsw,epsU,burnin,maxepoch,param_seed;langevin,stiefel)
# GPT_SGLD.jl:345 — returns (w_store, U_store); NaN in the geodesic -> message + zeros (:422-424).
function GPTregression(phi::Array{Float64,3}, y::Array{Float64}, signal_var::Real, I::Array{Int32,2},
                       r::Integer, Q::Integer, m::Integer, epsw::Real, epsU::Real, burnin::Integer,
                       maxepoch::Integer, param_seed::Integer=0; langevin=true, stiefel=true,
                       sigma_w::Real=1.0, store_every::Integer=1)
    n, D, N = size(phi)
    numbatches = cld(N, m)
    T = div(maxepoch * numbatches, store_every)
    cfg = Ref(SGLDConfig(n, D, N, r, Q, m, epsw, epsU, signal_var, sigma_w, burnin, maxepoch,
                         UInt64(param_seed), Int32(langevin), Int32(stiefel), store_every, 0))
    w_store = zeros(Q, T); U_store = zeros(n, r, D, T)
    rc = ccall((:gpt_sgld_regression, LIB), Cint,
               (Ref{SGLDConfig}, Ptr{Float64}, Ptr{Float64}, Ptr{Int32}, Ptr{Float64}, Ptr{Float64},
                Ptr{Float64}, Ptr{Float64}, Ptr{Float64}),
               cfg, phi, vec(y), I, C_NULL, C_NULL, w_store, U_store, C_NULL)
    if rc == 1
        println("Get NaN when moving along Geodesic. Try smaller epsU")
        return zeros(Q, T), zeros(n, r, D, T)
    end
    check(rc)
    return w_store, U_store
end

# The sweep block of kin40kExperiment.jl:67-74 (`@parallel for j=1:10`, one GPTregression per sweep
# on that sweep's phitrain) as one call: chain j runs on phis[j] with param_seeds[j] (epsw, epsU,
# signal_var: one value, or one per chain) in one device session (gpt_sgld_regression_chains: the
# chain engine at r <= 5, the wave engine at kin40k's r = 20).  Returns [(w_store, U_store, status)]
# per chain; status 1 = the geodesic NaN bail-out (message + zero stores, :422-424).
function GPTregression_chains(phis::Vector{Array{Float64,3}}, y::Array{Float64}, signal_var,
                              I::Array{Int32,2}, r::Integer, Q::Integer, m::Integer, epsw, epsU,
                              burnin::Integer, maxepoch::Integer, param_seeds::Vector{<:Integer};
                              sigma_w::Real=1.0, store_every::Integer=1)
    C = length(param_seeds)
    length(phis) == C || error("one phi per chain")
    n, D, N = size(phis[1])
    T = div(maxepoch * cld(N, m), store_every)
    perchain(v) = v isa Real ? fill(Float64(v), C) : collect(Float64, v)
    ew, eu, sv = perchain(epsw), perchain(epsU), perchain(signal_var)
    cfg = Ref(SGLDConfig(n, D, N, r, Q, m, ew[1], eu[1], sv[1], sigma_w, burnin, maxepoch,
                         UInt64(0), Int32(1), Int32(1), store_every, 0))
    ws = [zeros(Q, T) for c = 1:C]; Us = [zeros(n, r, D, T) for c = 1:C]
    yv = vec(y); status = zeros(Int32, C); seeds = UInt64.(param_seeds)
    GC.@preserve phis yv ws Us begin
        check(ccall((:gpt_sgld_regression_chains, LIB), Cint,
                    (Ref{SGLDConfig}, Int32, Ptr{UInt64}, Ptr{Ptr{Float64}}, Ptr{Ptr{Float64}},
                     Ptr{Int32}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Ptr{Float64}},
                     Ptr{Ptr{Float64}}, Ptr{Int32}),
                    cfg, Int32(C), seeds, pointer.(phis), fill(pointer(yv), C), I, ew, eu, sv,
                    pointer.(ws), pointer.(Us), status))
    end
    for c = 1:C
        status[c] == 1 && println("Get NaN when moving along Geodesic. Try smaller epsU")
    end
    return [(ws[c], Us[c], Int(status[c])) for c = 1:C]
end

# GPT_SGLDERM(phi,y,sigma,I,r,Q,m,epsw,epsU,burnin,maxepoch)  GPT_SGLD_p.jl:146 (σ_w=√(nᴰ/Q))
function GPT_SGLDERM(phi::Array{Float64,3}, y::Array{Float64}, sigma::Real, I::Array{Int32,2},
                     r::Integer, Q::Integer, m::Integer, epsw::Real, epsU::Real, burnin::Integer,
                     maxepoch::Integer, param_seed::Integer=0)
    n, D, _ = size(phi)
    return GPTregression(phi, y, sigma^2, I, r, Q, m, epsw, epsU, burnin, maxepoch, param_seed;
                         sigma_w=sqrt(Float64(n)^D / Q))
end

# GPT_SGLDERM_RMSprop(phi,y,signal_var,I,r,Q,m,epsilon,alpha,burnin,maxepoch)  GPT_SGLD.jl:1121
function GPT_SGLDERM_RMSprop(phi::Array{Float64,3}, y::Array{Float64}, signal_var::Real,
                             I::Array{Int32,2}, r::Integer, Q::Integer, m::Integer, epsilon::Real,
                             alpha::Real, burnin::Integer, maxepoch::Integer, param_seed::Integer=0)
    n, D, N = size(phi)
    T = maxepoch * cld(N, m)
    cfg = Ref(SGLDConfig(n, D, N, r, Q, m, epsilon, epsilon, signal_var, 1.0, burnin, maxepoch,
                         UInt64(param_seed), Int32(1), Int32(1), 1, 0))
    w_store = zeros(Q, T); U_store = zeros(n, r, D, T)
    rc = ccall((:gpt_sgld_rmsprop, LIB), Cint,
               (Ref{SGLDConfig}, Float64, Float64, Ptr{Float64}, Ptr{Float64}, Ptr{Int32},
                Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}),
               cfg, epsilon, alpha, phi, vec(y), I, C_NULL, C_NULL, w_store, U_store, C_NULL)
    if rc == 1
        return zeros(Q, T), zeros(n, r, D, T)
    end
    check(rc)
    return w_store, U_store
end

# pred(w,U,I,phitest)  GPT_SGLD.jl:233
# GPT_SGLD.jl:1065-1118 (w-only SGLD, U fixed at its Stiefel draw)
function GPT_SGLDERMw(phi::Array{Float64,3}, y::Array{Float64}, signal_var::Real, I::Array{Int32,2},
                      r::Integer, Q::Integer, m::Integer, epsw::Real, burnin::Integer, maxepoch::Integer,
                      param_seed::Integer=0)
    n, D, N = size(phi)
    cfg = SGLDConfig(n, D, N, r, Q, m, epsw, 0.0, signal_var, 1.0, burnin, maxepoch, param_seed, 1, 1, 1, 0)
    w_store = Array{Float64}(undef, Q, maxepoch * cld(N, m))
    U = Array{Float64}(undef, n, r, D)
    check(ccall((:gpt_sgld_wonly, LIB), Cint,
                (Ref{SGLDConfig}, Ptr{Float64}, Ptr{Float64}, Ptr{Int32}, Ptr{Float64}, Ptr{Float64},
                 Ptr{Float64}, Ptr{Float64}, Ptr{Float64}),
                cfg, phi, vec(y), I, C_NULL, C_NULL, w_store, U, C_NULL))
    return w_store, U
end

# GPT_SGLD.jl:452-680 (labels y in 1..C)
function GPTclassification(phi::Array{Float64,3}, y::Array, I::Array{Int32,2}, r::Integer, Q::Integer,
                           m::Integer, epsw::Real, epsU::Real, burnin::Integer, maxepoch::Integer,
                           param_seed::Integer; langevin=true, stiefel=true)
    n, D, N = size(phi)
    C = Int(maximum(y) - minimum(y) + 1)
    cfg = SGLDConfig(n, D, N, r, Q, m, epsw, epsU, 1.0, 1.0, burnin, maxepoch, param_seed,
                     Int32(langevin), Int32(stiefel), 1, 0)
    T = maxepoch * cld(N, m)
    w_store = Array{Float64}(undef, Q, C, T); U_store = Array{Float64}(undef, n, r, D, C, T)
    rc = ccall((:gpt_sgld_classification, LIB), Cint,
               (Ref{SGLDConfig}, Ptr{Float64}, Ptr{Float64}, Ptr{Int32}, Ptr{Float64}, Ptr{Float64},
                Ptr{Float64}, Ptr{Float64}, Ptr{Float64}),
               cfg, phi, Float64.(vec(y)), I, C_NULL, C_NULL, w_store, U_store, C_NULL)
    if rc == 1
        println("Get NaN when moving along Geodesic. Try smaller epsU")
        return zeros(Q, C, T), zeros(n, r, D, C, T)
    end
    check(rc)
    return w_store, U_store
end

# GPT_SGLD.jl:684-805 (geodesic Monte Carlo)
function GPT_GMC(phi::Array{Float64,3}, y::Array{Float64}, signal_var::Real, I::Array{Int32,2},
                 r::Integer, Q::Integer, epsw::Real, epsU::Real, burnin::Integer, maxepoch::Integer,
                 L::Integer, param_seed::Integer)
    n, D, N = size(phi)
    w_store = Array{Float64}(undef, Q, maxepoch); U_store = Array{Float64}(undef, n, r, D, maxepoch)
    accept_prob = Array{Float64}(undef, maxepoch + burnin)
    rc = ccall((:gpt_gmc, LIB), Cint,
               (Ptr{Float64}, Ptr{Float64}, Int64, Int64, Int64, Int64, Int64, Ptr{Int32}, Float64,
                Float64, Float64, Int64, Int64, Int64, UInt64, Ptr{Float64}, Ptr{Float64},
                Ptr{Float64}, Ptr{Float64}, Ptr{Float64}),
               phi, vec(y), n, D, N, r, Q, I, signal_var, epsw, epsU, burnin, maxepoch, L, param_seed,
               C_NULL, C_NULL, w_store, U_store, accept_prob)
    rc == 1 && println("Get NaN when moving along Geodesic. Try smaller epsU")
    rc in (0, 1) || check(rc)
    return w_store, U_store, accept_prob
end

function pred(w::Array{Float64}, U::Array{Float64,3}, I::Array{Int32,2}, phitest::Array{Float64,3})
    n, D, Nt = size(phitest); r = size(U, 2); Q = length(w)
    f = Array{Float64}(undef, Nt)
    check(ccall((:gpt_pred, LIB), Cint,
                (Ptr{Float64}, Ptr{Float64}, Ptr{Int32}, Ptr{Float64}, Int64, Int64, Int64, Int64, Int64,
                 Ptr{Float64}), vec(w), U, I, phitest, n, D, Nt, r, Q, f))
    return f
end

# RMSE(w_store,U_store,I,phitest,ytest)  GPT_SGLD_p.jl:124 — mean prediction over all samples
function RMSE(w_store::Array{Float64,2}, U_store::Array{Float64,4}, I::Array{Int32,2},
              phitest::Array{Float64,3}, ytest::Array{Float64})
    n, D, Nt = size(phitest); r = size(U_store, 2); Q, S = size(w_store)
    meanf = Array{Float64}(undef, Nt); out = Ref(0.0)
    check(ccall((:gpt_pred_mean, LIB), Cint,
                (Ptr{Float64}, Ptr{Float64}, Ptr{Int32}, Ptr{Float64}, Ptr{Float64}, Int64, Int64, Int64,
                 Int64, Int64, Int64, Float64, Ptr{Float64}, Ref{Float64}),
                w_store, U_store, I, phitest, vec(ytest), n, D, Nt, r, Q, S, 1.0, meanf, out))
    return out[]
end

# The per-epoch evaluation of kin40kExperiment.jl:78-87 with the test features formed inside the
# prediction kernel (no n·D·Ntest phitest array): returns (meanfhat, scale·RMSE of the mean,
# per-sample scale·RMSE = the testRMSE curve when the samples are the epoch ends)
function pred_mean_x(w_store::Array{Float64,2}, U_store::Array{Float64,4}, I::Array{Int32,2},
                     Xtest::Array{Float64,2}, ytest::Array{Float64}, length_scale,
                     sigma_RBF::Real, phi_scale::Real, Z::Array{Float64,2}, b::Array{Float64};
                     scale::Real=1.0)
    Nt, D = size(Xtest); n = size(Z, 1); r = size(U_store, 2); Q, S = size(w_store)
    ls = collect(Float64, length_scale isa Real ? [length_scale] : length_scale)
    meanf = Array{Float64}(undef, Nt); out = Ref(0.0); curve = Array{Float64}(undef, S)
    check(ccall((:gpt_pred_mean_x, LIB), Cint,
                (Ptr{Float64}, Ptr{Float64}, Ptr{Int32}, Ptr{Float64}, Ptr{Float64}, Int64, Int64,
                 Ptr{Float64}, Int64, Float64, Float64, Ptr{Float64}, Ptr{Float64}, Int64, Int64,
                 Int64, Int64, Float64, Ptr{Float64}, Ref{Float64}, Ptr{Float64}),
                w_store, U_store, I, Xtest, vec(ytest), Nt, D, ls, length(ls), sigma_RBF,
                phi_scale, Z, b, n, r, Q, S, scale, meanf, out, curve))
    return meanf, out[], curve
end

# The initial draws of GPTregression for param_seed (GPT_SGLD.jl:357-369): (w, U)
function init_state(n::Integer, r::Integer, D::Integer, Q::Integer, param_seed::Integer;
                    stiefel=true, sigma_w::Real=1.0)
    cfg = Ref(SGLDConfig(n, D, 1, r, Q, 1, 0.0, 0.0, 1.0, sigma_w, 0, 1, UInt64(param_seed),
                         Int32(1), Int32(stiefel), 1, 0))
    w = Array{Float64}(undef, Q); U = Array{Float64}(undef, n, r, D)
    check(ccall((:gpt_sgld_init, LIB), Cint, (Ref{SGLDConfig}, Ptr{Float64}, Ptr{Float64}), cfg, w, U))
    return w, U
end

# GPNT_SGLD(phi,y,signal_var,sigma_theta,m,eps_theta,decay_rate,burnin,maxepoch,param_seed)
# GPT_SGLD.jl:809
function GPNT_SGLD(phi::Array{Float64,2}, y::Array{Float64}, signal_var::Real, sigma_theta::Real,
                   m::Integer, eps_theta::Real, decay_rate::Real, burnin::Integer, maxepoch::Integer,
                   param_seed::Integer)
    n, N = size(phi)
    store = Array{Float64}(undef, n, (maxepoch + burnin) * cld(N, m))
    rc = ccall((:gpt_gpnt_sgld, LIB), Cint,
               (Ptr{Float64}, Ptr{Float64}, Int64, Int64, Float64, Float64, Int64, Float64, Float64,
                Int64, Int64, UInt64, Ptr{Float64}),
               phi, vec(y), n, N, signal_var, sigma_theta, m, eps_theta, decay_rate, burnin, maxepoch,
               param_seed, store)
    if rc == 4
        println("Get NaN in theta. Try smaller epsilon")
        return zeros(n)
    end
    check(rc)
    return store
end

end # module
