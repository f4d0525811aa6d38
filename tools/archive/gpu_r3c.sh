set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in base lf cp5 cp6 ff; do AIQMC_LIB_VARIANT=$v timeout -k 10 120 python tools/prop_check.py 2>&1 | grep -v amdgpu.ids || exit 1; done
bash tools/ab_bitwise.sh base lf cp5 cp6
