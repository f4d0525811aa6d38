# round 5: parameters repacked on the device (aiqmc_set_params_device), Adam steps without a host
# round trip of the parameters: tests, then Be / C-ccECP Adam iterations, host round trip vs device
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_api.py tests/test_gpu_pgrad.py tests/test_gpu_complex_el.py -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/r5g_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5g_tests.log; echo "tests rc=$rc"
[ $rc -eq 0 ] || exit $rc
out=gpurun_out/ab_r5g.txt
: > $out
for pp in 0 1; do
  for rep in 1 2 3; do
    for hp in 1 0; do
      if [ $hp = 1 ]; then r=$(AIQMC_PP=$( [ $pp = 1 ] && echo 1 ) AIQMC_HOST_PARAMS=1 timeout -k 10 200 python tools/adam_only.py) || exit 1
      else r=$(AIQMC_PP=$( [ $pp = 1 ] && echo 1 ) timeout -k 10 200 python tools/adam_only.py) || exit 1; fi
      echo "pp=$pp host_params=$hp rep$rep $(echo "$r" | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_iteration"],4), d["energy"])')" | tee -a $out
    done
  done
done
