# MovieLens_HIP — the tensor CF samplers of 100k_movielensExperiment.jl on libgptsgld.so
# (include/gptsgld.h: gpt_cf_*).  Julia is not on the image: tests/test_julia_shim.py checks every
# ccall below against the C prototypes; the same entry points are exercised through
# gpt_amd/movielens.py by the GPU tests.  In the script, replace the `@everywhere function
# GPT_fixw(...)` .. `GPT_fullw_gibbs(...)` definitions with `using MovieLens_HIP`; the data
# processing (:553-586) is unchanged.  The reference reads ytrainMean / ytrainStd as script
# globals; here they are the two arguments after param_seed.
module MovieLens_HIP

export GPT_fixw, GPT_fullw, GPT_fixw_sideinfo, GPT_fullw_sideinfo, GPT_fullw_sideinfo_folds,
       GPT_fixw_gibbs, GPT_fullw_gibbs

const LIB = get(ENV, "GPTSGLD_LIB", joinpath(@__DIR__, "..", "gpt_amd", "libgptsgld.so"))
lasterr() = unsafe_string(ccall((:gpt_last_error, LIB), Cstring, ()))
check(rc) = rc == 0 ? nothing : error("gptsgld error $rc: " * lasterr())

function GPT_fullw_sideinfo(Rating::Array, UserData::Array, MovieData::Array, Ratingtest::Array,
                            signal_var::Real, sigma_u::Real, sigma_w::Real, w_init::Array, m::Integer,
                            epsw::Real, epsU::Real, a::Real, b::Real, c::Real, burnin::Integer,
                            maxepoch::Integer, param_seed::Integer, ytrainMean::Real, ytrainStd::Real;
                            langevin::Bool=false, stiefel::Bool=false, avg::Bool=false)
    Rt = Float64.(Rating); Rs = Float64.(Ratingtest); Ud = Float64.(UserData); Md = Float64.(MovieData)
    N, Ntest = size(Rt, 1), size(Rs, 1); n1, D1 = size(Ud); n2, D2 = size(Md); r = size(w_init, 1)
    w_store = zeros(r, r, maxepoch); U_store = zeros(n1 + D1, r, maxepoch)
    V_store = zeros(n2 + D2, r, maxepoch); testpred_store = zeros(Ntest, maxepoch)
    trainRMSEvec = zeros(maxepoch); testRMSEvec = zeros(maxepoch)
    rc = ccall((:gpt_cf_fullw_sideinfo, LIB), Cint,
               (Ptr{Float64}, Int64, Int64, Ptr{Float64}, Int64, Int64, Ptr{Float64}, Int64, Int64,
                Ptr{Float64}, Int64, Int64, Float64, Float64, Float64, Ptr{Float64}, Int64, Int64,
                Float64, Float64, Float64, Float64, Float64, Int64, Int64, UInt64, Float64, Float64,
                Int32, Int32, Int32, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64},
                Ptr{Float64}, Ptr{Float64}),
               Rt, N, N, Ud, n1, D1, Md, n2, D2, Rs, Ntest, Ntest, signal_var, sigma_u, sigma_w,
               Float64.(w_init), r, m, epsw, epsU, a, b, c, burnin, maxepoch, param_seed, ytrainMean,
               ytrainStd, langevin, stiefel, avg, w_store, U_store, V_store, testpred_store,
               trainRMSEvec, testRMSEvec)
    rc == 1 && println("Get NaN when moving along Geodesic. Try smaller epsU")
    rc in (0, 1) || check(rc)
    return w_store, U_store, V_store, testpred_store, trainRMSEvec, testRMSEvec
end

function GPT_fullw_gibbs(Rating::Array, UserData::Array, MovieData::Array, Ratingtest::Array,
                         signal_var::Real, sigma_u::Real, sigma_w::Real, w_init::Array, burnin::Integer,
                         maxepoch::Integer, n_samples::Integer, param_seed::Integer, ytrainMean::Real,
                         ytrainStd::Real; avg::Bool=false, rotated_w::Bool=false)
    Rt = Float64.(Rating); Rs = Float64.(Ratingtest)
    N, Ntest = size(Rt, 1), size(Rs, 1); n1 = size(UserData, 1); n2 = size(MovieData, 1)
    r = size(w_init, 1)
    w_store = zeros(r, r, maxepoch); U_store = zeros(n1, r, maxepoch); V_store = zeros(n2, r, maxepoch)
    testpred_store = zeros(Ntest, maxepoch); trainRMSEvec = zeros(maxepoch); testRMSEvec = zeros(maxepoch)
    check(ccall((:gpt_cf_fullw_gibbs, LIB), Cint,
                (Ptr{Float64}, Int64, Int64, Int64, Int64, Ptr{Float64}, Int64, Int64, Float64, Float64,
                 Float64, Ptr{Float64}, Int64, Int64, Int64, Int64, UInt64, Float64, Float64, Int32,
                 Int32, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64},
                 Ptr{Float64}),
                Rt, N, N, n1, n2, Rs, Ntest, Ntest, signal_var, sigma_u, sigma_w, Float64.(w_init), r,
                burnin, maxepoch, n_samples, param_seed, ytrainMean, ytrainStd, avg, rotated_w,
                w_store, U_store, V_store, testpred_store, trainRMSEvec, testRMSEvec))
    return w_store, U_store, V_store, testpred_store, trainRMSEvec, testRMSEvec
end

# GPT_fixw_sideinfo(...)  100k_movielensExperiment.jl:282-404 (w fixed)
function GPT_fixw_sideinfo(Rating::Array, UserData::Array, MovieData::Array, Ratingtest::Array,
                           signal_var::Real, sigma_u::Real, w::Array, m::Integer, epsU::Real,
                           a::Real, b::Real, c::Real, burnin::Integer, maxepoch::Integer,
                           param_seed::Integer, ytrainMean::Real, ytrainStd::Real;
                           langevin::Bool=false, stiefel::Bool=false, avg::Bool=false)
    Rt = Float64.(Rating); Rs = Float64.(Ratingtest); Ud = Float64.(UserData); Md = Float64.(MovieData)
    N, Ntest = size(Rt, 1), size(Rs, 1); n1, D1 = size(Ud); n2, D2 = size(Md); r = size(w, 1)
    U_store = zeros(n1 + D1, r, maxepoch); V_store = zeros(n2 + D2, r, maxepoch)
    testpred_store = zeros(Ntest, maxepoch); trainRMSEvec = zeros(maxepoch); testRMSEvec = zeros(maxepoch)
    rc = ccall((:gpt_cf_fixw_sideinfo, LIB), Cint,
               (Ptr{Float64}, Int64, Int64, Ptr{Float64}, Int64, Int64, Ptr{Float64}, Int64, Int64,
                Ptr{Float64}, Int64, Int64, Float64, Float64, Ptr{Float64}, Int64, Int64, Float64,
                Float64, Float64, Float64, Int64, Int64, UInt64, Float64, Float64, Int32, Int32,
                Int32, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}),
               Rt, N, N, Ud, n1, D1, Md, n2, D2, Rs, Ntest, Ntest, signal_var, sigma_u, Float64.(w),
               r, m, epsU, a, b, c, burnin, maxepoch, param_seed, ytrainMean, ytrainStd, langevin,
               stiefel, avg, U_store, V_store, testpred_store, trainRMSEvec, testRMSEvec)
    rc == 1 && println("Get NaN when moving along Geodesic. Try smaller epsU")
    rc in (0, 1) || check(rc)
    return U_store, V_store, testpred_store, trainRMSEvec, testRMSEvec
end

# GPT_fullw(...)  100k_movielensExperiment.jl:160-279 (no side information)
function GPT_fullw(Rating::Array, UserData::Array, MovieData::Array, Ratingtest::Array,
                   signal_var::Real, sigma_u::Real, sigma_w::Real, w_init::Array, m::Integer,
                   epsw::Real, epsU::Real, burnin::Integer, maxepoch::Integer, param_seed::Integer,
                   ytrainMean::Real, ytrainStd::Real; langevin::Bool=false, stiefel::Bool=false,
                   avg::Bool=false)
    Rt = Float64.(Rating); Rs = Float64.(Ratingtest)
    N, Ntest = size(Rt, 1), size(Rs, 1); n1 = size(UserData, 1); n2 = size(MovieData, 1)
    r = size(w_init, 1)
    w_store = zeros(r, r, maxepoch); U_store = zeros(n1, r, maxepoch); V_store = zeros(n2, r, maxepoch)
    testpred_store = zeros(Ntest, maxepoch); trainRMSEvec = zeros(maxepoch); testRMSEvec = zeros(maxepoch)
    rc = ccall((:gpt_cf_fullw, LIB), Cint,
               (Ptr{Float64}, Int64, Int64, Int64, Int64, Ptr{Float64}, Int64, Int64, Float64,
                Float64, Float64, Ptr{Float64}, Int64, Int64, Float64, Float64, Int64, Int64, UInt64,
                Float64, Float64, Int32, Int32, Int32, Ptr{Float64}, Ptr{Float64}, Ptr{Float64},
                Ptr{Float64}, Ptr{Float64}, Ptr{Float64}),
               Rt, N, N, n1, n2, Rs, Ntest, Ntest, signal_var, sigma_u, sigma_w, Float64.(w_init),
               r, m, epsw, epsU, burnin, maxepoch, param_seed, ytrainMean, ytrainStd, langevin,
               stiefel, avg, w_store, U_store, V_store, testpred_store, trainRMSEvec, testRMSEvec)
    rc == 1 && println("Get NaN when moving along Geodesic. Try smaller epsU")
    rc in (0, 1) || check(rc)
    return w_store, U_store, V_store, testpred_store, trainRMSEvec, testRMSEvec
end

# GPT_fixw(...)  100k_movielensExperiment.jl:56-156 (no side information, w fixed)
function GPT_fixw(Rating::Array, UserData::Array, MovieData::Array, Ratingtest::Array,
                  signal_var::Real, sigma_u::Real, w::Array, m::Integer, epsU::Real,
                  burnin::Integer, maxepoch::Integer, param_seed::Integer, ytrainMean::Real,
                  ytrainStd::Real; langevin::Bool=false, stiefel::Bool=false, avg::Bool=false)
    Rt = Float64.(Rating); Rs = Float64.(Ratingtest)
    N, Ntest = size(Rt, 1), size(Rs, 1); n1 = size(UserData, 1); n2 = size(MovieData, 1)
    r = size(w, 1)
    U_store = zeros(n1, r, maxepoch); V_store = zeros(n2, r, maxepoch)
    testpred_store = zeros(Ntest, maxepoch); trainRMSEvec = zeros(maxepoch); testRMSEvec = zeros(maxepoch)
    rc = ccall((:gpt_cf_fixw, LIB), Cint,
               (Ptr{Float64}, Int64, Int64, Int64, Int64, Ptr{Float64}, Int64, Int64, Float64,
                Float64, Ptr{Float64}, Int64, Int64, Float64, Int64, Int64, UInt64, Float64,
                Float64, Int32, Int32, Int32, Ptr{Float64}, Ptr{Float64}, Ptr{Float64},
                Ptr{Float64}, Ptr{Float64}),
               Rt, N, N, n1, n2, Rs, Ntest, Ntest, signal_var, sigma_u, Float64.(w), r, m, epsU,
               burnin, maxepoch, param_seed, ytrainMean, ytrainStd, langevin, stiefel, avg,
               U_store, V_store, testpred_store, trainRMSEvec, testRMSEvec)
    rc == 1 && println("Get NaN when moving along Geodesic. Try smaller epsU")
    rc in (0, 1) || check(rc)
    return U_store, V_store, testpred_store, trainRMSEvec, testRMSEvec
end

# GPT_fixw_gibbs(...)  100k_movielensExperiment.jl:945-1028 (w fixed, Gibbs U / V rows)
function GPT_fixw_gibbs(Rating::Array, UserData::Array, MovieData::Array, Ratingtest::Array,
                        signal_var::Real, sigma_u::Real, w::Array, burnin::Integer,
                        maxepoch::Integer, n_samples::Integer, param_seed::Integer,
                        ytrainMean::Real, ytrainStd::Real; avg::Bool=false, rotated_w::Bool=false)
    Rt = Float64.(Rating); Rs = Float64.(Ratingtest)
    N, Ntest = size(Rt, 1), size(Rs, 1); n1 = size(UserData, 1); n2 = size(MovieData, 1)
    r = size(w, 1)
    U_store = zeros(n1, r, maxepoch); V_store = zeros(n2, r, maxepoch)
    testpred_store = zeros(Ntest, maxepoch); trainRMSEvec = zeros(maxepoch); testRMSEvec = zeros(maxepoch)
    check(ccall((:gpt_cf_fixw_gibbs, LIB), Cint,
                (Ptr{Float64}, Int64, Int64, Int64, Int64, Ptr{Float64}, Int64, Int64, Float64,
                 Float64, Ptr{Float64}, Int64, Int64, Int64, Int64, UInt64, Float64, Float64, Int32,
                 Int32, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}),
                Rt, N, N, n1, n2, Rs, Ntest, Ntest, signal_var, sigma_u, Float64.(w), r, burnin,
                maxepoch, n_samples, param_seed, ytrainMean, ytrainStd, avg, rotated_w, U_store,
                V_store, testpred_store, trainRMSEvec, testRMSEvec))
    return U_store, V_store, testpred_store, trainRMSEvec, testRMSEvec
end

# The folds loop of 100k_movielensExperiment.jl:733-736 (`@sync @parallel for i=1:5` over
# GPT_fullw_sideinfo(Ratingtrain[:,:,i], ..., Ratingtest[:,:,i], ..., ytrainMean[i],
# ytrainStd[i])) as one device launch per epoch: Ratingtrain / Ratingtest are the script's
# (N, 4, F) / (Ntest, 4, F) arrays; returns one output tuple per fold.
function GPT_fullw_sideinfo_folds(Ratingtrain::Array{Float64,3}, UserData::Array, MovieData::Array,
                                  Ratingtest::Array{Float64,3}, signal_var::Real, sigma_u::Real,
                                  sigma_w::Real, w_init::Array, m::Integer, epsw::Real, epsU::Real,
                                  a::Real, b::Real, c::Real, burnin::Integer, maxepoch::Integer,
                                  param_seed::Integer, ytrainMean::Array, ytrainStd::Array;
                                  langevin::Bool=false, stiefel::Bool=false, avg::Bool=false)
    F = size(Ratingtrain, 3)
    Rts = [Ratingtrain[:, :, f] for f = 1:F]; Rss = [Ratingtest[:, :, f] for f = 1:F]
    Ud = Float64.(UserData); Md = Float64.(MovieData)
    n1, D1 = size(Ud); n2, D2 = size(Md); r = size(w_init, 1)
    Ns = Int64[size(R, 1) for R in Rts]; Nts = Int64[size(R, 1) for R in Rss]
    outs = [(zeros(r, r, maxepoch), zeros(n1 + D1, r, maxepoch), zeros(n2 + D2, r, maxepoch),
             zeros(Nts[f], maxepoch), zeros(maxepoch), zeros(maxepoch)) for f = 1:F]
    ptrs(k) = Ptr{Float64}[pointer(o[k]) for o in outs]
    status = zeros(Int32, F)
    rc = GC.@preserve Rts Rss outs ccall((:gpt_cf_fullw_sideinfo_folds, LIB), Cint,
               (Int64, Ptr{Ptr{Float64}}, Ptr{Int64}, Ptr{Ptr{Float64}}, Ptr{Int64}, Ptr{Float64},
                Int64, Int64, Ptr{Float64}, Int64, Int64, Float64, Float64, Float64, Ptr{Float64},
                Int64, Int64, Float64, Float64, Float64, Float64, Float64, Int64, Int64, UInt64,
                Ptr{Float64}, Ptr{Float64}, Int32, Int32, Int32, Ptr{Ptr{Float64}},
                Ptr{Ptr{Float64}}, Ptr{Ptr{Float64}}, Ptr{Ptr{Float64}}, Ptr{Ptr{Float64}},
                Ptr{Ptr{Float64}}, Ptr{Int32}),
               F, Ptr{Float64}[pointer(R) for R in Rts], Ns, Ptr{Float64}[pointer(R) for R in Rss],
               Nts, Ud, n1, D1, Md, n2, D2, signal_var, sigma_u, sigma_w, Float64.(w_init), r, m,
               epsw, epsU, a, b, c, burnin, maxepoch, param_seed, Float64.(ytrainMean),
               Float64.(ytrainStd), langevin, stiefel, avg, ptrs(1), ptrs(2), ptrs(3), ptrs(4),
               ptrs(5), ptrs(6), status)
    rc == 1 && println("Get NaN when moving along Geodesic. Try smaller epsU")
    rc in (0, 1) || check(rc)
    return outs
end

end # module
