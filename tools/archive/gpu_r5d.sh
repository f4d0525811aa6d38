# round 5: k_param_grad with 4 (N <= 4) / 2 (N <= 8) walkers per wave vs one (AQ_PGK1 variant)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_pgrad.py tests/test_gpu_api.py -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/r5d_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r5d_tests.log; echo "tests rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
out=gpurun_out/ab_r5d.txt
: > $out
for rep in 1 2; do
  for v in pgk1 shipped; do
    if [ $v = shipped ]; then r=$(timeout -k 10 200 python tools/pgrad_ab.py gpurun_out/pg_$v.npz) || exit 1
    else r=$(AIQMC_LIB_VARIANT=$v timeout -k 10 200 python tools/pgrad_ab.py gpurun_out/pg_$v.npz) || exit 1; fi
    echo "== $v rep$rep" | tee -a $out; echo "$r" | tee -a $out
  done
done
python tools/pgrad_ab.py --cmp gpurun_out/pg_shipped.npz gpurun_out/pg_pgk1.npz | tee -a $out
for rep in 1 2; do
  for v in pgk1 shipped; do
    if [ $v = shipped ]; then r=$(timeout -k 10 200 python tools/adam_only.py) || exit 1
    else r=$(AIQMC_LIB_VARIANT=$v timeout -k 10 200 python tools/adam_only.py) || exit 1; fi
    echo "== adam $v rep$rep $(echo "$r" | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_iteration"], d["energy"])')" | tee -a $out
  done
done
rm -f gpurun_out/pg_*.npz
