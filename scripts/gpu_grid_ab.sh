cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for v in ${VARIANTS:-nt base}; do
  lib=gpt_amd/libgptsgld_$v.so; [ "$v" = base ] && lib=gpt_amd/libgptsgld.so
  echo "=== $v"
  GPTSGLD_LIB=$lib timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "grid or rmsprop or classif or wonly or gpnt" > gpurun_out/gt_$v.log 2>&1 || { echo "tests $v failed"; tail -15 gpurun_out/gt_$v.log; exit 1; }
  tail -1 gpurun_out/gt_$v.log
  GPTSGLD_LIB=$lib timeout -k 10 120 python scripts/phase_stamps.py --engine grid --chains 1 --steps 20 > gpurun_out/gs_$v.log 2>&1 || { echo "stamps failed"; tail -5 gpurun_out/gs_$v.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/gs_$v.log
done
