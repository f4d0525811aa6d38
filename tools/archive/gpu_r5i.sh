# round 5: the fused one-rank loss statistics (aiqmc_loss_weights): parity tests, then the Adam
# side measurements (Be, C ccECP) with the fused launch vs the torch statistics path
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_api.py tests/test_gpu_pgrad.py tests/test_gpu_complex_el.py > gpurun_out/r5i_tests.txt 2>&1 \
  || { tail -40 gpurun_out/r5i_tests.txt; exit 1; }
tail -3 gpurun_out/r5i_tests.txt
for pp in 0 1; do for lt in 1 0; do
  if [ $lt = 1 ]; then export AIQMC_LOSS_TORCH=1; else unset AIQMC_LOSS_TORCH; fi
  if [ $pp = 1 ]; then export AIQMC_PP=1; else unset AIQMC_PP; fi
  for rep in 1 2; do
    echo "== pp=$pp loss_torch=$lt rep=$rep"; timeout -k 10 200 python tools/adam_only.py 2>&1 | grep -v amdgpu.ids | tail -2 || exit 1
  done
done; done
