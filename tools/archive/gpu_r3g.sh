set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for W in 512 4096; do WALKERS=$W AIQMC_LIB_VARIANT=phaseprof timeout -k 10 120 python profiles/phase_prof.py 2>&1 | grep -v amdgpu.ids | sed "s/^/B=$W /"; done
