cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for e in 0 1 2 4 8 12; do
  echo "== exp $e"
  GPTSGLD_CF_EXP=$e GPTSGLD_LIB=gpt_amd/libgptsgld_diag.so timeout -k 10 120 python -u scripts/ml_stamps.py > gpurun_out/r6z8_exp$e.log 2>&1 || exit $?
done
