# TGP_HIP — drop-in replacement of the reference's `TGP` module (TGP.jl) on the MI355X path, via
# `ccall` into libgptsgld.so (include/gptsgld.h: gpt_feature, gpt_feature_inputs, gpt_tgp_gibbs,
# gpt_pred_mean).  Untested here (no Julia on the image); mirrors gpt_amd/TGP.py, which is tested.
#
#   UnitTest.jl:  `using TGP`  ->  `using TGP_HIP`
module TGP_HIP

export feature, GPT_inf, datawhitening, TensorRes

const LIB = get(ENV, "GPTSGLD_LIB", joinpath(@__DIR__, "..", "gpt_amd", "libgptsgld.so"))
lasterr() = unsafe_string(ccall((:gpt_last_error, LIB), Cstring, ()))
check(rc) = rc == 0 ? nothing : error("gptsgld error $rc: " * lasterr())

# TGP.jl:16-21
function datawhitening(x::Array)
    x = float(copy(x))
    for i = 1:size(x, 2)
        c = x[:, i]; mu = sum(c) / length(c)
        x[:, i] = (c .- mu) ./ sqrt(sum(abs2, c .- mu) / (length(c) - 1))
    end
    return x
end

# b (n, D, N) for all rows at once: TGP.jl:45-46 (`feature` reseeds per row, so Z and b are shared)
function features(X::Array{Float64,2}, n::Integer, sigmaRBF::Real, generator::Integer)
    N, D = size(X)
    Z = Array{Float64}(undef, n, D); B = Array{Float64}(undef, n, D)
    check(ccall((:gpt_feature_inputs, LIB), Cint, (Int64, Int64, UInt64, Ptr{Float64}, Ptr{Float64}),
                n, D, generator, Z, B))
    b = Array{Float64}(undef, n, D, N)
    check(ccall((:gpt_feature, LIB), Cint,
                (Ptr{Float64}, Int64, Int64, Ptr{Float64}, Int64, Float64, Float64, Ptr{Float64},
                 Ptr{Float64}, Int64, Ptr{Float64}),
                X, N, D, [Float64(sigmaRBF)], 1, 1.0, 1.0, Z, B, n, b))
    return b
end

# TGP.jl:6-14
feature(x, n, sigmaRBF, generator) = features(reshape(Float64.(vec(x)), 1, :), n, sigmaRBF, generator)[:, :, 1]

# TGP.jl:37-86
function GPT_inf(X, y, sigma, n, r, sigmaRBF, q, generator, num_iterations, burnin)
    X = datawhitening(X); y = datawhitening(reshape(y, :, 1))
    N, D = size(X)
    b = features(X, n, sigmaRBF, generator)
    T = num_iterations - burnin
    W = Array{Float64}(undef, q, T); V = Array{Float64}(undef, n, r, D, T)
    I = Array{Int32}(undef, q, D)
    check(ccall((:gpt_tgp_gibbs, LIB), Cint,
                (Ptr{Float64}, Ptr{Float64}, Int64, Int64, Int64, Int64, Int64, Float64, Int64, Int64,
                 UInt64, Ptr{Int32}, Ptr{Float64}, Ptr{Float64}, Ptr{Int32}),
                b, vec(y), n, D, N, r, q, sigma, num_iterations, burnin, generator, C_NULL, W, V, I))
    return W, V, I
end

# TGP.jl:89-108
function TensorRes(Xtrain, ytrain, sigma, n, r, sigmaRBF, q, generator, num_iterations, burnin, X, y)
    W, U, I = GPT_inf(Xtrain, ytrain, sigma, n, r, sigmaRBF, q, generator, num_iterations, burnin)
    ys = vec(y); ystd = sqrt(sum(abs2, ys .- sum(ys) / length(ys)) / (length(ys) - 1))
    X = datawhitening(X); y = vec(datawhitening(reshape(ys, :, 1)))
    N, D = size(X)
    b = features(X, n, sigmaRBF, generator)
    S = size(W, 2); mean = Array{Float64}(undef, N); rmse = Ref(0.0)
    check(ccall((:gpt_pred_mean, LIB), Cint,
                (Ptr{Float64}, Ptr{Float64}, Ptr{Int32}, Ptr{Float64}, Ptr{Float64}, Int64, Int64,
                 Int64, Int64, Int64, Int64, Float64, Ptr{Float64}, Ptr{Float64}),
                W, U, I, b, y, n, D, N, r, q, S, ystd, mean, rmse))
    return rmse[]
end

end # module
