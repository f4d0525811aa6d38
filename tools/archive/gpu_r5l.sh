# round 5: the 46-shape library: every shape vs the fp64 oracle, the ECP goldens (CO2 included),
# golden parity, parameter gradients, and the N2 headline (library load + kernels unchanged)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_shapes.py tests/test_ecp.py tests/test_gpu_parity.py tests/test_gpu_pgrad.py tests/test_gpu_api.py \
  > gpurun_out/r5l_tests.txt 2>&1 || { tail -60 gpurun_out/r5l_tests.txt; exit 1; }
grep -E "passed|failed" gpurun_out/r5l_tests.txt | tail -2
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-ecp --no-adam --no-dmc --no-cpu-baseline \
  > gpurun_out/r5l_bench.json 2> gpurun_out/r5l_bench.err || { tail -20 gpurun_out/r5l_bench.err; exit 1; }
cut -c1-400 gpurun_out/r5l_bench.json
