set -o pipefail
cd $GRAFT_REPO_ROOT
for hp in 1 0; do
  if [ $hp = 1 ]; then export AIQMC_HOST_PARAMS=1; else unset AIQMC_HOST_PARAMS; fi
  echo "== host_params=$hp"; timeout -k 10 200 python tools/adam_breakdown.py 2>&1 | grep -v amdgpu.ids || exit 1
done
