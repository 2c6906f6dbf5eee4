# MovieLens_HIP — the tensor CF samplers of 100k_movielensExperiment.jl on libgptsgld.so
# (include/gptsgld.h: gpt_cf_fullw_sideinfo, gpt_cf_fullw_gibbs).  Untested here (no Julia on the
# image); mirrors gpt_amd/movielens.py, which is tested.  In the script, replace the
# `@everywhere function GPT_fullw_sideinfo(...)` / `GPT_fullw_gibbs(...)` definitions with
# `using MovieLens_HIP`; the data processing (:561-586) is unchanged.
module MovieLens_HIP

export GPT_fullw_sideinfo, GPT_fullw_gibbs

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

end # module
